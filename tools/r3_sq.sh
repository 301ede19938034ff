#!/bin/bash
# SQ counters (one PMC pass) over the redo probe: the dense first anchoring + 11 steady iterations at 10M.
export TMPDIR=/tmp
tag=${1:-sq}
mkdir -p gpurun_out/$tag
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/$tag -o run -- python3 tools/redo_probe.py 10000000 12 > gpurun_out/$tag/probe.log 2>&1 || exit $?
python3 tools/pmc_sq.py gpurun_out/$tag/run_counter_collection.csv > gpurun_out/$tag/sq.txt
