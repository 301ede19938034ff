#!/bin/bash
# A/B the fused K1 across library builds on the GPU box: tools/ab_probe.sh <tag>... where each tag names
# normal-guided-pointcloud-denoiser_amd/libpcd_<tag>.so (built with `make OUT=../libpcd_<tag>.so BUILD=build_<tag>
# EXTRA=...`); "cur" is the in-tree libpcd.so.  Stops at the first failing run.
set -o pipefail
for v in "$@"; do
  if [ "$v" = cur ]; then lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd.so
  else lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd_$v.so; fi
  echo "== $v"
  PCD_LIB=$lib timeout -k 10 200 python tools/seed_probe.py 1000000 10000000 2>&1 | grep -v amdgpu || exit 1
done
