#!/bin/bash
# A/B microbenchmarks of the current kernel options (one GPU process each).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/ab_$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; case $rc in 0|1) ;; *) exit $rc ;; esac; }
run gtest python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "gemm" --timeout 120 --timeout-method thread -p no:cacheprovider
run g_u1 python scripts/gemm_f32_bench.py --reps 50 --cfgs 0 --opt gemm1x1_f32_upfront=1
run g_u0 python scripts/gemm_f32_bench.py --reps 50 --cfgs 0 --opt gemm1x1_f32_upfront=0 --opt gemm1x1_f32_direct=0
run g_u1b python scripts/gemm_f32_bench.py --reps 50 --cfgs 0 --opt gemm1x1_f32_upfront=1
run g_k3u1 python scripts/gemm_f32_bench.py --reps 50 --cfgs 0 --k3 --opt gemm1x1_f32_upfront=1
run g_k3u0 python scripts/gemm_f32_bench.py --reps 50 --cfgs 0 --k3 --opt gemm1x1_f32_upfront=0 --opt gemm1x1_f32_direct=0
