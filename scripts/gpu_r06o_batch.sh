#!/bin/bash
# round-6 evidence, part 2: the C2 (DCVC-HEM) and C4 (YUV420 4K) bench lines, each
# with its cpu_baseline
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u bench.py --model hem > gpurun_out/r06o_bench_hem.log 2>&1; rc=$?
echo "bench hem rc=$rc"; tail -1 gpurun_out/r06o_bench_hem.log | cut -c1-200
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python -u bench.py --yuv420 --steps 16 > gpurun_out/r06o_bench_c4.log 2>&1; rc=$?
echo "bench c4 rc=$rc"; tail -1 gpurun_out/r06o_bench_c4.log | cut -c1-200
exit $rc
