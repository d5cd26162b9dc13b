#!/bin/bash
# round-3 first look: split-fp16 kernels, strict parity in split precision, bench layers
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_sconv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03a_sconv.log 2>&1
echo "sconv tests rc=$?"
tail -5 gpurun_out/r03a_sconv.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_strict.py -q --timeout 200 --timeout-method thread -k "split and (golden or c3small)" > gpurun_out/r03a_strict.log 2>&1
echo "strict rc=$?"
tail -15 gpurun_out/r03a_strict.log
timeout -k 10 300 python -u bench.py --lanes 1 --steps 8 --warmup 2 --no-cpu-baseline --profile-out gpurun_out/r03a_layers_split.json > gpurun_out/r03a_bench_split.json 2> gpurun_out/r03a_bench_split.err
echo "bench rc=$?"
tail -3 gpurun_out/r03a_bench_split.err
cut -c1-600 gpurun_out/r03a_bench_split.json
