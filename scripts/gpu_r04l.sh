#!/bin/bash
# round 4: the other configurations' bench lines (C2 HEM 1080p, C4 DC YUV420 4K), split precision
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u bench.py --model hem --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04l_bench_hem.json 2> gpurun_out/r04l_bench_hem.err
rc=$?; echo "hem rc=$rc"; cut -c1-300 gpurun_out/r04l_bench_hem.json; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --yuv420 --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/r04l_bench_c4.json 2> gpurun_out/r04l_bench_c4.err
rc=$?; echo "c4 rc=$rc"; cut -c1-300 gpurun_out/r04l_bench_c4.json; exit $rc
