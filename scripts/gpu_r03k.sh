#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_strict.py -q --timeout 500 --timeout-method thread -k "split" > gpurun_out/r03k_strict.log 2>&1
echo "strict rc=$?"; tail -5 gpurun_out/r03k_strict.log
timeout -k 10 600 python -u bench.py > gpurun_out/r03k_bench_default.json 2> gpurun_out/r03k_bench_default.err
echo "bench rc=$?"; cut -c1-400 gpurun_out/r03k_bench_default.json
