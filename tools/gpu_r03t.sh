#!/bin/bash
# r03t: PMC HBM traffic + rocprof stats of the C2 (ig_kernel_x3d) and C3 (ig_kernel_bf16) dominant kernels
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_pmc.sh r03t_pmc_split fp32_split || exit 1
bash tools/gpu_pmc.sh r03t_pmc_bf16 bf16 || exit 1
cd $GRAFT_REPO_ROOT
PMC_KERNEL="ig_kernel_x3d" python tools/pmc_summary.py gpurun_out/r03t_pmc_split gpurun_out/r03t_pmc_dominant.json
PMC_KERNEL="ig_kernel_bf16<128, 192, 64, 96>" python tools/pmc_summary.py gpurun_out/r03t_pmc_bf16 gpurun_out/r03t_bf16_pmc_dominant.json
