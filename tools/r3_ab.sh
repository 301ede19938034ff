#!/bin/bash
# Round-3 A/B call: dense probe + 30-iteration redo probe of the in-tree build, the -m gpu suite, then the bench
# A/B of the in-tree build against experiment variants.  Usage (inside gpurun): bash tools/r3_ab.sh <tag> <variant>...
export TMPDIR=/tmp
tag=${1:-ab}; shift
tools/gpu_run.sh \
  "$tag/dense:120:python tools/dense_probe.py 10000000 3" \
  "$tag/redo:200:python tools/redo_probe.py 10000000 30" \
  "$tag/t:900:python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider" \
  "$tag/ab:600:bash tools/ab_bench.sh cur $* cur"
