#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
( while true; do date >> gpurun_out/r06j_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_wconv.py -m gpu -v -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r06j_wconv_pytest.log 2>&1 || { echo wconv tests failed; tail -30 gpurun_out/r06j_wconv_pytest.log; exit 1; }
echo wconv tests ok
S=48x48@1088x1920k3,48x48@1088x1920k3r,64x64@544x960k3r,64x64@544x960k3,128x64@544x960k3,192x48@272x480k3,64x48@544x960k3
for rep in 1 2; do
  for w in 0 1; do
    timeout -k 10 120 python -u scripts/sconv_bench.py --shapes $S --opt wconv=$w >> gpurun_out/r06j_wconv_ab.jsonl 2>> gpurun_out/r06j_wconv_ab.err || exit 1
  done
done
echo wconv ab ok
timeout -k 10 900 python -u -m pytest tests/test_gpu_split_range.py tests/test_gpu_parity_strict.py -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r06j_pytest.log 2>&1
rc=$?
echo pytest rc=$rc
exit $rc
