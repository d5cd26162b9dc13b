#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest tests/test_gpu_sconv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03j_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/r03j_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_strict.py -q --timeout 300 --timeout-method thread -k "split and (golden or c3small)" > gpurun_out/r03j_strict.log 2>&1
echo "strict rc=$?"; tail -3 gpurun_out/r03j_strict.log
timeout -k 10 300 python -u bench.py --lanes 1 --steps 8 --warmup 2 --no-cpu-baseline --profile-out gpurun_out/r03j_layers_split.json > gpurun_out/r03j_bench_split.json 2> gpurun_out/r03j_bench_split.err
echo "bench rc=$?"; cut -c1-200 gpurun_out/r03j_bench_split.json
