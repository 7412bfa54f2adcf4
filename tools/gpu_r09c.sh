#!/bin/bash
# More ablations (x3d: no DMA wait / no B DMA / no A DMA; edge conv: no MFMA / no plane build / no
# loads+stores) and the C3 tests with the hyperprior on bf16 operands.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_libab.sh r09c_abl "g_a.2 conv fwd,g_a.0 conv3->192 fwd" 2 x3dnowait x3dnob x3dnoa ecnomfma ecnobuild ecnoio || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -s \
  tests/test_bf16_gpu.py "tests/test_bench_plans_gpu.py::test_config_step_vs_oracle_and_bench_plans[C3]" > gpurun_out/tests_r09c.log 2>&1
rc=$?; tail -30 gpurun_out/tests_r09c.log; exit $rc
