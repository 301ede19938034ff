#!/bin/bash
# Round-3 GPU call: the -m gpu suite, then the traffic-counter calibration (tools/calib_traffic.hip, one PMC
# counter group per pass).  Usage (inside gpurun): bash tools/r3_call.sh <tag>
export TMPDIR=/tmp
tag=${1:-c1}
tools/gpu_run.sh \
  "$tag/t:900:python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider" \
  "$tag/cal_fetch:90:rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$tag/cal_fetch -o run -- tools/bin/calib_traffic" \
  "$tag/cal_write:90:rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$tag/cal_write -o run -- tools/bin/calib_traffic"
