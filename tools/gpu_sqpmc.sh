#!/bin/bash
# SQ PMC passes (MFMA busy, waits, LDS conflicts) for the ops matching $1 in tools/layer_bench.py
set -o pipefail
R=$GRAFT_REPO_ROOT; F="$1"; TAG=${2:-sq}
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/$TAG/a -o a --output-format csv -- python3 $R/tools/layer_bench.py --only "$F" --reps 3 --math ${MATH:-0} > $R/gpurun_out/$TAG/a.log 2>&1 || { tail -20 $R/gpurun_out/$TAG/a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LEVEL_WAVES GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/$TAG/b -o b --output-format csv -- python3 $R/tools/layer_bench.py --only "$F" --reps 3 --math ${MATH:-0} > $R/gpurun_out/$TAG/b.log 2>&1 || { tail -20 $R/gpurun_out/$TAG/b.log; exit 1; }
echo DONE
