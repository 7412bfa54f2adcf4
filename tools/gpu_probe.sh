#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 240 python -u tools/grad_probe.py --n 16 --size 256 --math fp32_split > gpurun_out/grad_probe.txt 2>&1
timeout -k 10 240 python -u tools/grad_probe.py --n 16 --size 256 --math fp32 >> gpurun_out/grad_probe.txt 2>&1
