#!/bin/bash
# round-3 evidence part 2: latent-fusion tests, rocprofv3 kernel stats + PMC traffic of C3 at one lane
# (split precision), then the default bench line (3 lanes, CPU baseline) and a one-lane layer profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_sconv.py -x -q --timeout 120 --timeout-method thread -k "latent" > gpurun_out/r03w_tests.log 2>&1
rc=$?; echo "latent tests rc=$rc"; tail -3 gpurun_out/r03w_tests.log; [ $rc = 0 ] || exit $rc
PROF_ARGS="--lanes 1" bash scripts/profile_round.sh r03w || exit $?
echo profiled
timeout -k 10 400 python -u bench.py --lanes 1 --steps 12 --warmup 2 --no-cpu-baseline --profile-out gpurun_out/r03w_layers.json > gpurun_out/r03w_bench_1lane.json 2> gpurun_out/r03w_bench_1lane.err
rc=$?; echo "bench1 rc=$rc"; cut -c1-200 gpurun_out/r03w_bench_1lane.json; [ $rc = 0 ] || exit $rc
timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03w_bench_default.json 2> gpurun_out/r03w_bench_default.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/r03w_bench_default.json
exit $rc
