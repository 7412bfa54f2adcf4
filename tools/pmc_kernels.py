#!/usr/bin/env python3
"""Per-kernel HBM traffic from tools/gpu_pmc_layers.sh output: FETCH_SIZE x2 (gfx950: 128-B
requests tallied at 64 B) + WRITE_SIZE, both KiB, median over launches; average duration from the
stats pass; achieved compulsory-byte bandwidth when the algorithmic bytes are given.

    python tools/pmc_kernels.py gpurun_out/TAG 'edge_conv_x3=428e6' 'edge_wgrad=428e6' ...
"""
import csv
import glob
import os
import statistics
import sys


def _vals(path, counter):
    out = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return out


def main(src, specs):
    fetch, write = _vals(os.path.join(src, "FETCH_SIZE"), "FETCH_SIZE"), _vals(os.path.join(src, "WRITE_SIZE"), "WRITE_SIZE")
    stats = {}
    for f in glob.glob(os.path.join(src, "stats", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            stats[r["Name"]] = (float(r["AverageNs"]), float(r["MinNs"]), int(r["Calls"]))
    for spec in specs:
        key, alg = spec.split("=")
        alg = float(alg)
        for name in fetch:
            if key not in name:
                continue
            if alg == 0:   # launches of several shapes: every launch's bytes, in launch order
                ws = write.get(name, [0.0] * len(fetch[name]))
                print(f"{name[:70]}: per-launch traffic MB " + " ".join(
                    f"{(2 * f + w) * 1024 / 1e6:.1f}" for f, w in zip(fetch[name], ws)))
                continue
            fb = 2 * statistics.median(fetch[name]) * 1024
            wb = statistics.median(write.get(name, [0.0])) * 1024
            st = next((v for k, v in stats.items() if k == name), None)
            line = f"{name[:70]:70s} traffic {(fb + wb) / 1e6:8.1f} MB (fetch {fb / 1e6:.1f}, write {wb / 1e6:.1f}), " \
                   f"compulsory {alg / 1e6:.1f} MB = {(fb + wb) / alg:.2f}x"
            if st:
                line += f"; avg {st[0] / 1e3:.1f} us (min {st[1] / 1e3:.1f}, {st[2]} calls) -> " \
                        f"{alg / st[0]:.0f} GB/s compulsory = {alg / st[0] / 8000:.2f} of 8 TB/s"
            print(line)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
