#!/bin/bash
# C3's main-queue gaps under the profiler: kernel + HIP API trace (launch vs start) and host pacing unprofiled.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_apitrace.sh r09m C3 || exit 1
bash tools/gpu_pace.sh r09m C3 C2 || exit 1
python3 tools/api_timeline.py gpurun_out/api_r09m_C3 > gpurun_out/api_r09m_C3_timeline.txt 2>&1 || exit 1
grep -n "quant_k\|abs_fwd_k\|cond_bwd_k\|abs_bwd" gpurun_out/api_r09m_C3_timeline.txt | head -20
