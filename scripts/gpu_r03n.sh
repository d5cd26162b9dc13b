#!/bin/bash
# round-3 re-entry status: split kernels, strict split parity, bench default (3 lanes) and one-lane layer profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_sconv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03n_sconv.log 2>&1
rc=$?; echo "sconv tests rc=$rc"; tail -3 gpurun_out/r03n_sconv.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_strict.py -v --timeout 500 --timeout-method thread -k "split" > gpurun_out/r03n_strict.log 2>&1
rc=$?; echo "strict rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/r03n_strict.log | tail -12; [ $rc = 0 ] || [ $rc = 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --lanes 1 --steps 12 --warmup 2 --no-cpu-baseline --profile-out gpurun_out/r03n_layers_split.json > gpurun_out/r03n_bench_1lane.json 2> gpurun_out/r03n_bench_1lane.err
rc=$?; echo "bench1 rc=$rc"; cut -c1-300 gpurun_out/r03n_bench_1lane.json; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03n_bench_default.json 2> gpurun_out/r03n_bench_default.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/r03n_bench_default.json
