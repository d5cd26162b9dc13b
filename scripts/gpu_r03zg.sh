#!/bin/bash
# default bench line of the final tree (bench oracle with the product's stream parts)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03zg_bench_default.json 2> gpurun_out/r03zg_bench_default.err
rc=$?; echo "bench rc=$rc"; cut -c1-200 gpurun_out/r03zg_bench_default.json
exit $rc
