#!/usr/bin/env python3
"""Report VGPR count, scratch spills and occupancy of every kernel in the HIP
sources (hipcc -Rpass-analysis=kernel-resource-usage).  Exit 1 when a kernel
spills VGPRs.

    python tools/spills.py [file.hip ...]     # default: every csrc/*.hip
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "image_compression_amd", "csrc")
# extra hipcc flags (e.g. -DGDN_BWD_XD=0) from the environment; the Makefile's no-packed-fp32 flag is always on
EXTRA = os.environ.get("SPILLS_FLAGS", "").split()


def analyse(src):
    with tempfile.TemporaryDirectory() as td:
        r = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I", CSRC, *EXTRA,
                            "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops", "-c", src,
                            "-o", os.path.join(td, "x.o"), "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True)
    out, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            out.append(cur)
            continue
        for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("spill", r"VGPRs Spill: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, line)
            if m and cur is not None:
                cur[key] = int(m.group(1))
    return out


def main():
    files = sys.argv[1:] or sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    bad = 0
    for f in files:
        for k in analyse(f):
            if k.get("spill", 0):
                bad += 1
            flag = "  SPILL" if k.get("spill", 0) else ""
            print(f"{os.path.basename(f):18s} v{k.get('vgpr', 0):3d} a{k.get('agpr', 0):3d} "
                  f"occ{k.get('occ', 0)} lds{k.get('lds', 0):6d} spill{k.get('spill', 0):3d}{flag}  {k['name'][:90]}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
