#!/bin/bash
# Where the dense first anchoring's time goes (round 4): the first iteration under the kernel tracer for the
# in-tree build and two timing-only builds of the re-anchoring search (results wrong: PCD_EXP_RQ=2 cell phase only,
# =3 cells + candidate rows + distances, no survivors).  Usage (GPU box): bash tools/r4_rqexp.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r4rq}
mkdir -p gpurun_out/$tag
shift; vs=${@:-cur rq2 rq3 dq2 dq4}
for v in $vs; do
  if [ "$v" = cur ]; then lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd.so
  else lib=$PWD/normal-guided-pointcloud-denoiser_amd/libpcd_$v.so; fi
  PCD_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/$v -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ten --no-extras --no-slab1 > gpurun_out/$tag/$v.log 2>&1 || exit $?
  python3 - "$tag" "$v" <<'PY'
import csv, sys
tag, v = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(f"gpurun_out/{tag}/{v}/run_kernel_stats.csv")))
for r in rows:
    if "k_knn_requery" in r["Name"] or "k_knn_redo_wave" in r["Name"] or "k_knn_dense_q" in r["Name"]:
        print(v, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms")
PY
done
