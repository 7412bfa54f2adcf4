#!/bin/bash
# C3 GDN norm recompute v2 (norm^T in registers feeding phase A): bitwise op test, timings, C3 A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_bf16_gpu.py -k "norm_recompute or gdn" > gpurun_out/tests_r09i.log 2>&1
rc=$?; tail -3 gpurun_out/tests_r09i.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/tests_r09i.log | head -20; exit $rc; }
timeout -k 10 120 python tools/gdn_rn_time.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r09i_gdn_rn_time.txt || exit 1
for i in 1 2; do
  for v in 1 0; do
    IMGCOMP_GDN_NORM_RECOMPUTE=$v timeout -k 10 200 python3 bench.py --config C3 --no-cpu-baseline --no-roofline > gpurun_out/r09i_c3_$v.json 2>gpurun_out/r09i_c3_$v.err || { tail gpurun_out/r09i_c3_$v.err; exit 1; }
    echo "C3 norm_recompute=$v $(python3 -c "import json;d=json.load(open('gpurun_out/r09i_c3_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09i_ab.txt
  done
done
