#!/bin/bash
# Round 6, first call: the changed GPU tests, the launcher's gloo rehearsal (bench.py --gpus 2 on the
# box's one GPU), the C2 bench line, and a C3 kernel trace for the idle-main-queue study.
#   gpurun -- bash tools/gpu_r09a.sh TAG
set -o pipefail
TAG=${1:-r09a}
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_ddp_gpu.py tests/test_bf16_gpu.py tests/test_eval.py > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
IMGCOMP_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-roofline \
  > gpurun_out/bench_${TAG}_gloo2.json 2> gpurun_out/bench_${TAG}_gloo2.err || { echo "GLOO2 FAIL"; tail -20 gpurun_out/bench_${TAG}_gloo2.err; exit 1; }
cut -c1-400 gpurun_out/bench_${TAG}_gloo2.json
timeout -k 10 300 python3 bench.py > gpurun_out/bench_${TAG}_C2.json 2> gpurun_out/bench_${TAG}_C2.err || { echo "C2 FAIL"; tail -20 gpurun_out/bench_${TAG}_C2.err; exit 1; }
cut -c1-300 gpurun_out/bench_${TAG}_C2.json
timeout -k 10 300 python3 bench.py --config C3 --no-cpu-baseline > gpurun_out/bench_${TAG}_C3.json 2> gpurun_out/bench_${TAG}_C3.err || { echo "C3 FAIL"; exit 1; }
cut -c1-300 gpurun_out/bench_${TAG}_C3.json
bash tools/gpu_cfgprof.sh ${TAG} C3
