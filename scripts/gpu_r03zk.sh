#!/bin/bash
# the co-running test in both precisions
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_corun.py -v --timeout 400 --timeout-method thread > gpurun_out/r03zk_corun.log 2>&1
rc=$?; echo "corun rc=$rc"; grep -E "PASS|FAIL|passed|failed" gpurun_out/r03zk_corun.log | tail -5; exit $rc
