#!/bin/bash
# One gpurun call for a milestone: GPU tests + smoke + bench + rocprof stats (gpu_check.sh),
# then the dominant kernel's PMC passes.  usage: bash tools/gpu_round.sh TAG MATH PMC_TAG
set -o pipefail
bash tools/gpu_check.sh $1 && bash tools/gpu_pmc.sh ${3:-pmc_$1} ${2:-fp32_split}
