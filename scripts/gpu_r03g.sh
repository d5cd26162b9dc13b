#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/pmc_cmd.sh gpurun_out/r03g_pmc8 python scripts/sconv_bench.py --reps 5 --opt sconv_res_waves=8 --shapes 48x48@1088x1920k3r,48x48@1088x1920k3 > gpurun_out/r03g_pmc8.txt 2>&1 || exit 1
grep '"kernel": "void sconv' gpurun_out/r03g_pmc8.txt
