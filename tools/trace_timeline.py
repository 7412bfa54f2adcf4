#!/usr/bin/env python3
"""Per-step timeline of a C2 bench run from a rocprofv3 --kernel-trace CSV: which queue each kernel
ran on, the main queue's idle gaps (and what the side queue was doing meanwhile), and per-kernel
time on each queue.  Steps are delimited by philox_advance_k (the first launch of every training
forward after the first).

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline
    python tools/trace_timeline.py gpurun_out/tr/run_kernel_trace.csv [--step -2] [--list]
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"^void ", "", n)
    return re.sub(r"\((?:[^()]|\([^()]*\))*\)$", "", n)[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--step", type=int, default=-2, help="which step (python index over the delimited steps)")
    ap.add_argument("--list", action="store_true", help="print every kernel of the step")
    ap.add_argument("--gap-us", type=float, default=8.0)
    ap.add_argument("--first", default=None, help="report the first main-queue launch of this kernel in every "
                    "delimited step (ig_kernel_x3d: g_a.2 fwd, the launch bench.py's roofline times live)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    for r in rows:
        r["t0"] = int(r["Start_Timestamp"]) / 1e3   # us
        r["t1"] = int(r["End_Timestamp"]) / 1e3
        r["q"] = int(r["Queue_Id"])
        r["n"] = short(r["Kernel_Name"])
    rows.sort(key=lambda r: r["t0"])
    marks = [i for i, r in enumerate(rows) if "philox_advance" in r["n"]]
    steps = [(marks[i], marks[i + 1]) for i in range(len(marks) - 1)]
    print(f"{len(rows)} kernels, {len(steps)} delimited steps; step spans (ms): "
          + " ".join(f"{(rows[e]['t0'] - rows[b]['t0']) / 1e3:.3f}" for b, e in steps))
    if a.first:
        ds = []
        for b, e in steps:
            mq = rows[b]["q"]
            k = next((r for r in rows[b:e] if r["q"] == mq and a.first in r["n"]), None)
            if k is not None:
                ds.append(k["t1"] - k["t0"])
        if ds:
            print(f"first main-queue {a.first} per step: {len(ds)} launches, mean {sum(ds) / len(ds) / 1e3:.4f} ms, "
                  f"min {min(ds) / 1e3:.4f}, max {max(ds) / 1e3:.4f} ms")
    b, e = steps[a.step]
    st = rows[b:e]
    t_start, t_end = st[0]["t0"], rows[e]["t0"]
    qs = sorted({r["q"] for r in st})
    main_q = st[0]["q"]
    print(f"step {a.step}: {(t_end - t_start) / 1e3:.3f} ms, queues {qs} (main {main_q})")
    for q in qs:
        ks = [r for r in st if r["q"] == q]
        busy = sum(r["t1"] - r["t0"] for r in ks)
        print(f"  queue {q}: {len(ks)} kernels, busy {busy / 1e3:.3f} ms")
    # main-queue gaps
    mk = [r for r in st if r["q"] == main_q]
    side = [r for r in st if r["q"] != main_q]
    gaps = []
    for p, n in zip(mk, mk[1:]):
        g = n["t0"] - p["t1"]
        if g > a.gap_us:
            over = [s["n"] for s in side if s["t0"] < n["t0"] and s["t1"] > p["t1"]]
            gaps.append((g, p["n"], n["n"], over))
    tot = sum(g[0] for g in gaps)
    print(f"  main-queue gaps > {a.gap_us} us: {len(gaps)}, {tot / 1e3:.3f} ms")
    for g, pn, nn, over in sorted(gaps, reverse=True)[:15]:
        print(f"    {g:8.1f} us  after {pn}  before {nn}  | side: {', '.join(over[:4])}{' ...' if len(over) > 4 else ''}")
    # per-kernel totals per queue
    for q in qs:
        agg = defaultdict(lambda: [0, 0.0, 0.0])
        for r in st:
            if r["q"] == q:
                d = r["t1"] - r["t0"]
                agg[r["n"]][0] += 1
                agg[r["n"]][1] += d
                agg[r["n"]][2] = max(agg[r["n"]][2], d)
        print(f"  queue {q} kernels:")
        for n, (c, s, mx) in sorted(agg.items(), key=lambda t: -t[1][1])[:25]:
            print(f"    {s / 1e3:7.3f} ms {c:4d}x  max {mx:7.1f} us  {n}")
    if a.list:
        for r in st:
            print(f"{(r['t0'] - t_start) / 1e3:8.3f} {(r['t1'] - r['t0']):8.1f} q{r['q']} {r['n']}")


if __name__ == "__main__":
    main()
