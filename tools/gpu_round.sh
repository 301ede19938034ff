# Full round evidence on the GPU box: gpu tests, rocprof stats + PMC traffic (tools/profile_round.sh), the bench line.
# Usage (inside gpurun): bash tools/gpu_round.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r1}
tools/gpu_run.sh "$tag/tests:900:python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
tools/profile_round.sh $tag || exit $?
python tools/pmc_traffic.py gpurun_out/$tag/pmc_fetch/run_counter_collection.csv gpurun_out/$tag/pmc_write/run_counter_collection.csv 10000000 32 gpurun_out/$tag/traffic.json > gpurun_out/$tag/traffic.log 2>&1 || exit 1
cp gpurun_out/$tag/traffic.json profiles/traffic.json
tools/gpu_run.sh "$tag/bench:400:python bench.py --steps 20 --warmup 5" || exit $?
