#!/bin/bash
# A/B the whole iteration across library builds on the GPU box: tools/ab_bench.sh <tag>... ("cur" = in-tree
# libpcd.so, else normal-guided-pointcloud-denoiser_amd/libpcd_<tag>.so); prints ms/iteration, the first (dense)
# iteration and the stage times.
set -o pipefail
for v in "$@"; do
  if [ "$v" = cur ]; then lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd.so
  else lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd_$v.so; fi
  out=$(PCD_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-ten --steps 20 --warmup 5 2>/dev/null | grep '^{') || { echo "$v failed"; exit 1; }
  echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['value'], 'first', d['first_iteration_ms'], {k: round(v, 3) for k, v in d['kernel_ms'].items()})"
done
