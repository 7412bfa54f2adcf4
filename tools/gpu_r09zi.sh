#!/bin/bash
# C4 / C2 / C3 with the hyperprior on the side stream (default) vs on the main stream (--serial-hyperprior).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in 1 2; do
  for c in C4 C3 C2; do
    for v in conc serial; do
      a=""; [ $v = serial ] && a="--serial-hyperprior"
      timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --no-roofline $a \
        > gpurun_out/r09zi_${c}_$v.json 2>gpurun_out/r09zi_${c}_$v.err || { tail gpurun_out/r09zi_${c}_$v.err; exit 1; }
      echo "$c $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09zi_${c}_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09zi_ab.txt
    done
  done
done
