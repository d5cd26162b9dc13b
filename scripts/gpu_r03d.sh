#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/pmc_cmd.sh gpurun_out/r03d_pmc4 python scripts/sconv_bench.py --reps 5 --opt sconv_waves=4 --shapes 48x48@1088x1920k3r,48x192@1088x1920k1 > gpurun_out/r03d_pmc4.txt 2>&1 || exit 1
bash scripts/pmc_cmd.sh gpurun_out/r03d_pmc8 python scripts/sconv_bench.py --reps 5 --opt sconv_waves=8 --shapes 48x48@1088x1920k3r,64x64@544x960k3r > gpurun_out/r03d_pmc8.txt 2>&1 || exit 1
grep kernel gpurun_out/r03d_pmc4.txt gpurun_out/r03d_pmc8.txt
