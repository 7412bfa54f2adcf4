#!/usr/bin/env python3
"""Summarise the two rocprofv3 PMC passes of tools/gpu_pmc.sh (FETCH_SIZE and
WRITE_SIZE, one counter per run) for the dominant kernel into
profiles/<name>.json, which bench.py reports as `roofline.traffic`.

Corrections (MI355X_MICROARCH.md, HBM section): both counters are in KiB;
on gfx950 FETCH_SIZE tallies 128-B requests of wide (16 B/lane) reads at 64 B,
so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.

    python tools/pmc_summary.py gpurun_out/pmc1 profiles/r01_pmc_dominant.json
"""
import csv
import glob
import json
import os
import statistics
import sys

KERNEL = os.environ.get("PMC_KERNEL", "ig_kernel<128, 192, 64, 96, false, false>")


def _values(path, counter):
    out = []
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and KERNEL in r["Kernel_Name"]:
                out.append(float(r["Counter_Value"]))
    return out


def main(src, dst):
    fetch = _values(os.path.join(src, "fetch"), "FETCH_SIZE")
    write = _values(os.path.join(src, "write"), "WRITE_SIZE")
    if not fetch or not write:
        raise SystemExit(f"no {KERNEL} counters under {src}")
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    rec = {
        "kernel": KERNEL,
        "workload": "conv2d 5x5 s2 192->192, 32x192x128x128 fp32 (g_a.2 fwd), tools/dominant_kernel.py",
        "launches": len(fetch),
        "FETCH_SIZE_KiB_median": f_kib,
        "WRITE_SIZE_KiB_median": w_kib,
        "fetch_bytes_corrected": 2.0 * f_kib * 1024.0,
        "write_bytes": w_kib * 1024.0,
        "traffic_bytes_per_launch": 2.0 * f_kib * 1024.0 + w_kib * 1024.0,
        # bf16 DMA tiles (C3): the input's bf16 copy and the bf16 weight plane, fp32 output
        "algorithmic_bytes_per_launch": ((2.0 * (32 * 192 * 128 * 128 + 192 * 192 * 25) + 4.0 * 32 * 192 * 64 * 64)
                                         if "b16d" in KERNEL else
                                         4.0 * (32 * 192 * 128 * 128 + 192 * 192 * 25 + 32 * 192 * 64 * 64)),
        "correction": "FETCH_SIZE x2 (gfx950 128-B requests tallied at 64 B), KiB -> bytes",
    }
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
