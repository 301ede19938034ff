set -o pipefail
tools/gpu_run.sh "t:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" || exit $?
tools/profile_round.sh r1d || exit $?
python tools/pmc_traffic.py gpurun_out/r1d/pmc_fetch/run_counter_collection.csv gpurun_out/r1d/pmc_write/run_counter_collection.csv 10000000 32 gpurun_out/r1d/traffic.json > gpurun_out/r1d/traffic.log 2>&1 || exit 1
cp gpurun_out/r1d/traffic.json profiles/traffic.json
tools/gpu_run.sh "r1d/bench:400:python bench.py" || exit $?
