#!/bin/bash
# fact_bwd_k with its parameters read before its gradient stores: entropy-model, race and model tests,
# the ISA scan, then C3 / C2 interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_ops_gpu.py tests/test_race_gpu.py tests/test_model_gpu.py > gpurun_out/tests_r09zg.log 2>&1
rc=$?; tail -2 gpurun_out/tests_r09zg.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for c in C3 C2; do
    for v in base fbw; do
      IMGCOMP_LIB=$R/tools/_abl/$v/libimgcomp.so timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --no-roofline \
        > gpurun_out/r09zg_${c}_$v.json 2>gpurun_out/r09zg_${c}_$v.err || { tail gpurun_out/r09zg_${c}_$v.err; exit 1; }
      echo "$c $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09zg_${c}_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09zg_ab.txt
    done
  done
done
