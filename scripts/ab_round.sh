#!/bin/bash
# A/B microbenchmarks of the current kernel options (one GPU process each).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/ab_$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; case $rc in 0|1) ;; *) exit $rc ;; esac; }
S=48x48@1088x1920r,48x48@1088x1920,96x48@1088x1920,80x48@1088x1920,32x32@1088x1920
run c3_def python scripts/conv3_bench.py --reps 30 --shapes $S
run c3_r4 python scripts/conv3_bench.py --reps 30 --shapes $S --opt conv3x3_rows4=1
run c3_def2 python scripts/conv3_bench.py --reps 30 --shapes $S
run c3_r4b python scripts/conv3_bench.py --reps 30 --shapes $S --opt conv3x3_rows4=1
