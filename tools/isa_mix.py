#!/usr/bin/env python3
"""Instruction mix of a kernel's main loop(s) in the gfx950 ISA (hipcc -S with the build's flags): MFMA,
VALU (by opcode), SALU, DS and VMEM counts between each loop header and its back edge.  The VALU count
beside the MFMAs is what a one- or two-wave-per-SIMD MFMA kernel pays for (MI355X_MICROARCH.md: an MFMA
holds the SIMD's vector issue for 8 of its cycles; VALU past that adds its full issue cost).

    python tools/isa_mix.py image_compression_amd/csrc/igemm.hip ig_kernel_x3d [extra hipcc flags...]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "image_compression_amd", "csrc")


def main(src, kernel, *flags):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I", CSRC, "-Xclang",
                        "-target-feature", "-Xclang", "-packed-fp32-ops", *flags, "--cuda-device-only", "-S", src,
                        "-o", out], check=True, capture_output=True)
        s = open(out).read()
    for name in re.findall(r"^(_Z\S*" + re.escape(kernel) + r"\S*):", s, re.M):
        i = s.index(name + ":")
        body = s[i:s.index(".Lfunc_end", i)].splitlines()
        # basic blocks: label line -> its instructions; a loop = its header block plus every block the
        # compiler annotates "in Loop: Header=<header>" (outer loops include their inner ones' blocks)
        blocks, cur = [], None
        for line in body:
            m = re.match(r"^(\.LBB\w+):(.*)", line)
            if m:
                cur = [m.group(1), m.group(2), []]
                blocks.append(cur)
            elif cur is not None and line.strip() and not line.strip().startswith((".", ";")):
                cur[2].append(line.strip().split()[0])
        for lab, ann, _ in blocks:
            if "Loop Header" not in ann:
                continue
            hdr = lab.lstrip(".").replace("LBB", "BB")
            ins = [x for l2, a2, xs in blocks if l2 == lab or ("Header=" + hdr + " ") in a2 + " " for x in xs]
            c = collections.Counter("mfma" if x.startswith("v_mfma") else "valu" if x.startswith("v_") else
                                    "salu" if x.startswith("s_") else "ds" if x.startswith("ds_") else
                                    "vmem" if x.startswith(("global_", "buffer_", "scratch_")) else x for x in ins)
            if c["mfma"] == 0:
                continue
            h = lab
            v = collections.Counter(x for x in ins if x.startswith("v_") and not x.startswith("v_mfma"))
            print(f"{name[:70]} loop@{h}: {dict(c)}")
            print("   VALU:", ", ".join(f"{k} {n}" for k, n in v.most_common(12)))


if __name__ == "__main__":
    main(*sys.argv[1:])
