#!/bin/bash
# A/B the fused CPSD driver across library builds on the GPU box: tools/cpsd_ab.sh <variant>... ("cur" = in-tree)
set -o pipefail
for v in "$@"; do
  if [ "$v" = cur ]; then lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd.so
  else lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd_$v.so; fi
  echo "== $v"; PCD_LIB=$lib timeout -k 10 200 python3 tools/cpsd_probe.py 50000 1000000 || exit 1
done
