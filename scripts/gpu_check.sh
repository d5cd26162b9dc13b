#!/bin/bash
# One gpurun session: GPU tests, a short bench, and a rocprofv3 kernel-trace
# summary.  Each GPU step has its own time limit; the script stops at the
# first step that crashes, aborts or times out (exit 124/134/137/139), and
# carries on past plain test failures (exit 1) so the bench still reports.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-tests bench prof}
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "pytest gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
      fatal $rc && exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
      fatal $rc && exit $rc ;;
    bench)
      timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
      rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
      fatal $rc && exit $rc ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv \
        -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof.log
      fatal $rc && exit $rc ;;
  esac
done
exit 0
