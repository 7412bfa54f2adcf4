#!/bin/bash
# bench.py's N > 1 path rehearsed on one GPU: two ranks sharing it over gloo (DDP eager, and the hipGraph + flat all-reduce mode)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export IMGCOMP_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04l_ddp.json 2> gpurun_out/r04l_ddp.err || { tail -20 gpurun_out/r04l_ddp.err; exit 1; }
cut -c1-400 gpurun_out/r04l_ddp.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --graph > gpurun_out/r04l_graph.json 2> gpurun_out/r04l_graph.err || { tail -20 gpurun_out/r04l_graph.err; exit 1; }
cut -c1-400 gpurun_out/r04l_graph.json
