#!/bin/bash
# r03g: confirm that only the entropy kernels' packed-fp32 code matters: in-tree (shuffle reduction,
# VALU-only files without packed fp32), LDS reduction with / without packed fp32 in entropy.hip only
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u tools/race_probe.py --reps 200 --pattern conc --check-fact > gpurun_out/race_intree.log 2>&1 || { tail -5 gpurun_out/race_intree.log; exit 1; }
echo "== in-tree"; grep -v "^ " gpurun_out/race_intree.log | tail -2
for v in ldsnopk ldspk; do
  IMGCOMP_LIB=$GRAFT_REPO_ROOT/tools/_abl/$v/libimgcomp.so timeout -k 10 400 python -u tools/race_probe.py --reps 120 --pattern conc --check-fact > gpurun_out/race_$v.log 2>&1 || { tail -5 gpurun_out/race_$v.log; exit 1; }
  echo "== $v"; grep -v "^ " gpurun_out/race_$v.log | tail -2
done
