#!/bin/bash
# round-3 re-entry: split conv microbench + SQ counters on the dominant split shapes
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u scripts/sconv_bench.py > gpurun_out/r03o_sconv_bench.jsonl 2>&1 || exit 1
cut -c1-260 gpurun_out/r03o_sconv_bench.jsonl
bash scripts/pmc_cmd.sh gpurun_out/r03o_pmc python scripts/sconv_bench.py --reps 5 --shapes 48x48@1088x1920k3r,64x64@544x960k3r,128x192@544x960k3 > gpurun_out/r03o_pmc.txt 2>&1 || exit 1
cat gpurun_out/r03o_pmc.txt | tail -30
