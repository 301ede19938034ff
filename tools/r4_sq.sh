#!/bin/bash
# SQ counters (one PMC pass) of the first two iterations (dense anchoring + one steady) for library builds:
# bash tools/r4_sq.sh <tag> <variant>...   ("cur" = in-tree libpcd.so, else libpcd_<variant>.so)
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/$tag
for v in "$@"; do
  if [ "$v" = cur ]; then lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd.so
  else lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd_$v.so; fi
  PCD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/$tag/$v -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ten --no-extras --no-slab1 > gpurun_out/$tag/$v.log 2>&1 || exit $?
  echo "== $v"; python3 tools/pmc_sq.py gpurun_out/$tag/$v/run_counter_collection.csv | grep -E "requery|dense_q|anchor" || true
done
