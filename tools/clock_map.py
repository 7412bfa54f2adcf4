#!/usr/bin/env python3
"""Per-kernel clock of a step from a rocprofv3 --pmc GRBM_GUI_ACTIVE run: GRBM_GUI_ACTIVE is summed
over the 8 XCDs, so cycles / 8 / duration is the average shader clock of each launch.  A kernel whose
clock sits well below the idle-boost clock is power-limited (its cycles, not its time, are what its
code sets).

    rocprofv3 --pmc GRBM_GUI_ACTIVE -d out -o run --output-format csv -- python3 bench.py --profile-step-only ...
    python tools/clock_map.py out/run_counter_collection.csv
"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    return re.sub(r"\((?:[^()]|\([^()]*\))*\)$", "", n)[:48]


rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
agg = defaultdict(lambda: [0, 0.0, 0.0])
for r in rows:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    if d <= 0:
        continue
    a = agg[short(r["Kernel_Name"])]
    a[0] += 1
    a[1] += d
    a[2] += float(r["Counter_Value"])
print(f"{'kernel':48s} {'n':>4s} {'ms':>8s} {'Mcyc/XCD':>9s} {'GHz':>6s}")
for k, (n, d, c) in sorted(agg.items(), key=lambda t: -t[1][1])[:30]:
    print(f"{k:48s} {n:4d} {d / 1e6:8.3f} {c / 8 / 1e6:9.3f} {c / 8 / d:6.3f}")
