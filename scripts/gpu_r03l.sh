#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_sconv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03l_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/r03l_tests.log; [ $rc = 0 ] || exit $rc
SH=1024x384@68x120k1,384x384@68x120k1,384x1024@68x120k1,768x192@68x120k1,192x768@68x120k1,192x192@68x120k1,128x128@272x480k1,48x48@1088x1920k1,128x64@544x960k1r
for o in -1 0 1 2 3 4 5 6; do
  timeout -k 10 120 python -u scripts/sconv_bench.py --shapes $SH --opt sgemm=$o > gpurun_out/r03l_sgemm_$o.log 2>&1 || exit 1
done
echo done
