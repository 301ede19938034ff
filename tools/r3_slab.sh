#!/bin/bash
# Rehearse the multi-rank slab bench on ONE GPU over gloo (several ranks sharing the card): 2 ranks weak scaling,
# 4 ranks strong scaling.  The driver's round-end run uses RCCL across GPUs.  Usage (inside gpurun): bash tools/r3_slab.sh <tag>
export TMPDIR=/tmp PCD_BENCH_BACKEND=gloo
tag=${1:-slab}
tools/gpu_run.sh \
  "$tag/weak2:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 3 --points 2000000 --no-cpu-baseline --no-ten --no-extras" \
  "$tag/strong4:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --steps 5 --warmup 3 --points 4000000 --strong --no-cpu-baseline --no-ten --no-extras"
