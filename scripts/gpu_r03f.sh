#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest tests/test_gpu_sconv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03f_sconv.log 2>&1
echo "sconv tests rc=$?"; tail -2 gpurun_out/r03f_sconv.log
for w in 8 4; do
timeout -k 10 200 python -u scripts/sconv_bench.py --opt sconv_res_waves=$w > gpurun_out/r03f_bench_w$w.jsonl 2>&1 || exit 1
done
cut -c1-230 gpurun_out/r03f_bench_w8.jsonl gpurun_out/r03f_bench_w4.jsonl
