#!/bin/bash
# wg_reduce_t_kernel with eight partial loads in flight (wr8, tools/_abl) vs the in-tree build: weight
# gradients bitwise (tools/wg_bitwise.py), the weight-gradient layers, then C4 / C2 / C3 interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python3 tools/wg_bitwise.py --out gpurun_out/r09zq_base.pt > gpurun_out/r09zq_bitwise.txt 2>&1 || { tail gpurun_out/r09zq_bitwise.txt; exit 1; }
IMGCOMP_LIB=$R/tools/_abl/wr8/libimgcomp.so timeout -k 10 200 python3 tools/wg_bitwise.py --ref gpurun_out/r09zq_base.pt >> gpurun_out/r09zq_bitwise.txt 2>&1 || { tail gpurun_out/r09zq_bitwise.txt; exit 1; }
rm -f gpurun_out/r09zq_base.pt; tail -1 gpurun_out/r09zq_bitwise.txt
bash tools/gpu_libab.sh r09zq_layers "wgrad" 2 wr8 || exit 1
for i in 1 2; do
  for c in C4 C2 C3; do
    for v in base wr8; do
      L=$R/image_compression_amd/lib/libimgcomp.so; [ $v = wr8 ] && L=$R/tools/_abl/wr8/libimgcomp.so
      IMGCOMP_LIB=$L timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --no-roofline \
        > gpurun_out/r09zq_${c}_$v.json 2>gpurun_out/r09zq_${c}_$v.err || { tail gpurun_out/r09zq_${c}_$v.err; exit 1; }
      echo "$c $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09zq_${c}_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09zq_ab.txt
    done
  done
done
