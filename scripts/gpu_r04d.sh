#!/bin/bash
# round 4: memory-bound kernels (warp, offset diversity, depthwise) tests
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "warp or offset_div or dwconv" --timeout 120 --timeout-method thread > gpurun_out/r04d_kernels.log 2>&1; rc=$?; tail -3 gpurun_out/r04d_kernels.log; [ $rc -le 1 ] || exit $rc
grep -E "^FAILED" gpurun_out/r04d_kernels.log | head || true
