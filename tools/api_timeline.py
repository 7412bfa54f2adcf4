#!/usr/bin/env python3
"""One training step of a rocprofv3 kernel + HIP runtime API trace (tools/gpu_apitrace.sh): for every
launch, when the host issued it (API start, us from the step's first launch), how long the call took,
and when the GPU started the kernel and on which queue.  A kernel whose GPU start trails its launch by
only a few us ran as soon as the host issued it (the host paced that part of the step).

    python tools/api_timeline.py gpurun_out/api_TAG_C4 [--step -2]
"""
import argparse
import csv
import os
import re

SKIP = ("hipGetDevice", "hipSetDevice", "hipGetLastError", "hipGetDeviceCount", "hipStreamGetCaptureInfo",
        "hipStreamIsCapturing")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--step", type=int, default=-2)
    a = ap.parse_args()
    api = list(csv.DictReader(open(os.path.join(a.dir, "run_hip_api_trace.csv"))))
    kt = {r["Correlation_Id"]: r for r in csv.DictReader(open(os.path.join(a.dir, "run_kernel_trace.csv")))}
    api.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(api) if r["Function"] == "hipLaunchKernel" and r["Correlation_Id"] in kt
             and "philox_advance" in kt[r["Correlation_Id"]]["Kernel_Name"]]
    s, e = marks[a.step - 1], marks[a.step]
    t0 = int(api[s]["Start_Timestamp"])
    for r in api[s:e]:
        if r["Function"] in SKIP:
            continue
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = kt.get(r["Correlation_Id"])
        extra = ""
        if k:
            name = re.sub(r"\(anonymous namespace\)::", "", k["Kernel_Name"])[:50]
            extra = f"q{k['Queue_Id']} gpu_start {(int(k['Start_Timestamp']) - t0) / 1e3:8.1f} {name}"
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:8.1f} {dt:7.1f} {r['Function']:22s} {extra}")


if __name__ == "__main__":
    main()
