#!/bin/bash
# final-tree bench lines: C3 (the driver's default command) and C2, each with
# its cpu_baseline
# usage: bash scripts/gpu_final_bench.sh [TAG]   (output names gpurun_out/TAG_*)
T=${1:-r06u}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_c3.log 2>&1; rc=$?
echo "bench c3 rc=$rc"; tail -1 gpurun_out/${T}_bench_c3.log | cut -c1-200
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 500 python -u bench.py --model hem > gpurun_out/${T}_bench_hem.log 2>&1; rc=$?
echo "bench hem rc=$rc"; tail -1 gpurun_out/${T}_bench_hem.log | cut -c1-200
exit $rc
