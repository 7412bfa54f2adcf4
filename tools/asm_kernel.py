#!/usr/bin/env python3
"""Summarise one kernel of a hipcc -S listing: VGPRs, spills, and the memory / wait instructions in
order (to check where the waitcnt pass puts s_waitcnt vmcnt in a loop).

    hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S edge.hip -o /tmp/edge.s
    python tools/asm_kernel.py /tmp/edge.s edge_conv_x3_kernelILi192ELi3 [--all]
"""
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    s = open(path).read()
    m = re.search(r"^(_Z\S*" + re.escape(pat) + r"\S*):", s, re.M)
    if not m:
        sys.exit(f"no kernel matching {pat}")
    name = m.group(1)
    i = m.end()
    j = s.index(".Lfunc_end", i)
    body = s[i:j].splitlines()
    meta = re.search(re.escape(name) + r"\.num_vgpr, (\d+)", s)
    print(name, "vgpr", meta.group(1) if meta else "?", "lines", len(body))
    keep = re.compile(r"s_waitcnt|global_|buffer_|s_barrier|s_cbranch|^\.LBB|v_mfma|ds_read|ds_write|s_setprio")
    out, last = [], None
    for ln in body:
        t = ln.strip()
        if not keep.search(t):
            continue
        k = t.split()[0]
        if k.startswith("v_mfma") or k.startswith("ds_"):
            if last and last[0] == k:
                last[1] += 1
                continue
            last = [k, 1]
            out.append(last)
        else:
            last = None
            out.append([t, 0])
    for k, n in out:
        print(f"  {k} x{n}" if n else f"  {k}")


if __name__ == "__main__":
    main()
