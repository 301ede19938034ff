#!/bin/bash
# Round profiling on the GPU box: kernel-trace stats, the two PMC traffic passes, traffic.json, then the bench
# line that reads it.  Usage: tools/profile_round.sh <tag> [bench args...]   (outputs under gpurun_out/<tag>/)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
args="--steps 20 --warmup 5 --profile-steps 0 --no-cpu-baseline --no-ten --no-extras $*"   # the driver's iterations 6-25
tools/gpu_run.sh \
  "$tag/prof:300:rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py $args" \
  "$tag/pmc_fetch:300:rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run -- python3 bench.py $args" \
  "$tag/pmc_write:300:rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o run -- python3 bench.py $args" || exit $?
