#!/bin/bash
# kernel stats of the C3 bf16 conv layers (tools/layer_bench.py --math 1) under rocprofv3
set -o pipefail
TAG=${1:-r07o}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/b16prof_$TAG -o run --output-format csv \
  -- python3 $R/tools/layer_bench.py --math 1 --only "g_a.2 conv fwd,g_s.4 tconv dgrad" --reps 10 > $R/gpurun_out/b16prof_$TAG.log 2>&1 || { echo PROF FAIL; tail $R/gpurun_out/b16prof_$TAG.log; exit 1; }
python3 - $R/gpurun_out/b16prof_$TAG <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:90]}")
PY
