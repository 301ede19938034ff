#!/bin/bash
# Rehearse the multi-rank slab bench on ONE GPU (several ranks sharing the card, libpcd's host transport over a gloo
# group): 2 ranks weak scaling, 4 ranks strong scaling; bench.py launches its ranks itself.  The driver's round-end
# run uses libpcd's RCCL communicator across GPUs.  Usage (inside gpurun): bash tools/r3_slab.sh <tag>
export TMPDIR=/tmp
tag=${1:-slab}
tools/gpu_run.sh \
  "$tag/weak2:300:python bench.py --gpus 2 --rehearse-one-gpu --steps 5 --warmup 3 --points 2000000 --no-cpu-baseline --no-ten --no-extras" \
  "$tag/strong4:300:python bench.py --gpus 4 --rehearse-one-gpu --steps 5 --warmup 3 --points 4000000 --strong --no-cpu-baseline --no-ten --no-extras"
