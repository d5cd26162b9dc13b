#!/bin/bash
# round-3 evidence part 3: C2 (HEM 1080p) and C4 (DC YUV420 4K) in split precision: rocprof stats + PMC at one
# lane, then their bench lines
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PROF_ARGS="--lanes 1 --model hem" bash scripts/profile_round.sh r03x_hem || exit $?
cp gpurun_out/prof_r03x_hem/r03x_hem_pmc.json profiles/ 2>/dev/null
timeout -k 10 600 python -u bench.py --model hem --steps 20 --warmup 5 > gpurun_out/r03x_bench_hem.json 2> gpurun_out/r03x_bench_hem.err
rc=$?; echo "hem bench rc=$rc"; cut -c1-250 gpurun_out/r03x_bench_hem.json; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --yuv420 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03x_bench_c4.json 2> gpurun_out/r03x_bench_c4.err
rc=$?; echo "c4 bench rc=$rc"; cut -c1-250 gpurun_out/r03x_bench_c4.json
exit $rc
