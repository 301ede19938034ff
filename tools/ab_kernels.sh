#!/bin/bash
# A/B kernel times across library builds on the GPU box: tools/ab_kernels.sh <iters> <tag>...
# ("cur" = in-tree libpcd.so, else normal-guided-pointcloud-denoiser_amd/libpcd_<tag>.so).  Per tag: the redo probe
# under rocprofv3 --kernel-trace --stats -> gpurun_out/ab/<tag>/ (probe.log + run_kernel_stats.csv).
set -o pipefail
it=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in "$@"; do
  if [ "$v" = cur ]; then lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd.so
  else lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd_$v.so; fi
  mkdir -p gpurun_out/ab/$v
  PCD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/$v -o run \
    -- python3 tools/redo_probe.py 10000000 "$it" > gpurun_out/ab/$v/probe.log 2>&1 || { echo "$v failed"; exit 1; }
  echo "== $v"; python3 tools/kstats.py gpurun_out/ab/$v/run_kernel_stats.csv gpurun_out/ab/$v/probe.log
done
