#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest tests/test_gpu_sconv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03e_sconv.log 2>&1
echo "sconv tests rc=$?"; tail -2 gpurun_out/r03e_sconv.log
timeout -k 10 200 python -u scripts/sconv_bench.py > gpurun_out/r03e_bench_res.jsonl 2>&1 || exit 1
cut -c1-250 gpurun_out/r03e_bench_res.jsonl
bash scripts/pmc_cmd.sh gpurun_out/r03e_pmc python scripts/sconv_bench.py --reps 5 --shapes 48x48@1088x1920k3r,64x64@544x960k3r,48x192@1088x1920k1 > gpurun_out/r03e_pmc.txt 2>&1 || exit 1
grep kernel gpurun_out/r03e_pmc.txt
