#!/bin/bash
# Round evidence, part 2: the GPU test suite, smoke(), and the bench lines of
# configs C3 (default), C2 (HEM) and C4 (YUV420 4K); each step under its own
# limit, stopping at the first crash / abort / time-out.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
STEPS="tests smoke bench" bash scripts/gpu_check.sh || exit $?
timeout -k 10 600 python bench.py --model hem > gpurun_out/bench_hem.log 2>&1; rc=$?; echo "bench hem rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py --yuv420 --steps 16 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1; rc=$?; echo "bench c4 rc=$rc"; [ $rc = 0 ] || exit $rc
