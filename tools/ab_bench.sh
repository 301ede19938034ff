#!/bin/bash
# A/B the whole iteration across library builds on the GPU box: tools/ab_bench.sh <tag>... ("cur" = in-tree
# libpcd.so, else normal-guided-pointcloud-denoiser_amd/libpcd_<tag>.so); prints ms/iteration, the first (dense)
# iteration and the stage times.  AB_LONG=1 also runs the ten-iteration cloud on to iteration 100 (long_run).
set -o pipefail
ten="--no-ten"; [ "${AB_LONG:-0}" = 1 ] && ten=""
for v in "$@"; do
  if [ "$v" = cur ]; then lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd.so
  else lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd_$v.so; fi
  out=$(PCD_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline $ten --no-extras --steps 20 --warmup 5 2>/dev/null | grep '^{') || { echo "$v failed"; exit 1; }
  echo "$out" | python -c "
import json,sys; d=json.loads(sys.stdin.read()); lr=d.get('long_run') or {}
print('$v', d['ms_per_step'], d['value'], 'first', d['first_iteration_ms'], 'ten', d.get('ten_iteration_ms'), 'it100', d.get('iter_ms_at_100'), 'last20', lr.get('mean_ms_last_20'), 'max', lr.get('max_ms'), {k: round(v, 3) for k, v in d['kernel_ms'].items()})"
done
