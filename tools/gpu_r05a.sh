#!/bin/bash
# r05a: packed-fp32 hazard probe; eval-parity + DDP tests; no-pk-anywhere and tap-order A/B (layers + step)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 240 tools/_abl/pk_hazard_probe 4096 16 400000 > gpurun_out/r05a_pk_probe.txt 2>&1 || { echo PROBE rc=$?; cat gpurun_out/r05a_pk_probe.txt; exit 1; }
cat gpurun_out/r05a_pk_probe.txt
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_eval.py tests/test_ddp_gpu.py tests/test_dma_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05a_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error|tie flips" gpurun_out/r05a_tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_libab.sh r05a_layers "g_a.2 conv fwd,g_s.4 tconv dgrad,g_a.4 conv fwd,g_s.2 tconv dgrad,g_a.6 conv fwd,wgrad,gdn" 2 nopk_all tapnat > /dev/null || exit 1
cat gpurun_out/r05a_layers.txt
bash tools/gpu_libstep.sh r05a_step nopk_all tapnat || exit 1
