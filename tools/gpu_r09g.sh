#!/bin/bash
# C3 GDN norm recompute: bitwise op test, the bf16 suite, the C3 step test, and C3 alternating A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -s \
  tests/test_bf16_gpu.py "tests/test_bench_plans_gpu.py::test_config_step_vs_oracle_and_bench_plans[C3]" > gpurun_out/tests_r09g.log 2>&1
rc=$?; tail -3 gpurun_out/tests_r09g.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/tests_r09g.log | head -20; exit $rc; }
for i in 1 2; do
  for v in 1 0; do
    IMGCOMP_GDN_NORM_RECOMPUTE=$v timeout -k 10 200 python3 bench.py --config C3 --no-cpu-baseline --no-roofline > gpurun_out/r09g_c3_$v.json 2>gpurun_out/r09g_c3_$v.err || { tail gpurun_out/r09g_c3_$v.err; exit 1; }
    echo "C3 norm_recompute=$v $(python3 -c "import json;d=json.load(open('gpurun_out/r09g_c3_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09g_ab.txt
  done
done
timeout -k 10 120 python tools/layer_bench.py --math 3 --gdn-math 3 --only "gdn" --reps 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r09g_gdn_layers.txt
