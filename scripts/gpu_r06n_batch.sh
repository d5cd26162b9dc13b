#!/bin/bash
# round-6 evidence, part 1: rocprofv3 trace + FETCH/WRITE passes of the C3 bench
# (one lane), then the default C3 bench line with its cpu_baseline and roofline
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
PROF_ARGS="--lanes 1" bash scripts/profile_round.sh r06 || exit $?
cp gpurun_out/prof_r06/r06_pmc.json gpurun_out/prof_r06/r06_kernel_stats.csv profiles/
timeout -k 10 600 python -u bench.py > gpurun_out/r06n_bench_c3.log 2>&1; rc=$?
echo "bench c3 rc=$rc"; tail -1 gpurun_out/r06n_bench_c3.log | cut -c1-300
exit $rc
