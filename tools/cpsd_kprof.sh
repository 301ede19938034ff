#!/bin/bash
# k_cpsd_nvt / k_cpsd_pvt average times at 1M points for library builds (kernel tracer): tools/cpsd_kprof.sh <tag> <variant>...
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/$tag
for v in "$@"; do
  if [ "$v" = cur ]; then lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd.so
  else lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd_$v.so; fi
  PCD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/$v -o run -- \
    python3 tools/cpsd_probe.py 1000000 > gpurun_out/$tag/$v.log 2>&1 || exit $?
  python3 - "$tag" "$v" <<'PY'
import csv, sys
tag, v = sys.argv[1], sys.argv[2]
for r in csv.DictReader(open(f"gpurun_out/{tag}/{v}/run_kernel_stats.csv")):
    if "k_cpsd" in r["Name"]:
        print(v, r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
