#!/bin/bash
# round 4: xconv (static-shape split 3x3) correctness and A/B against sconv
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_xconv.py tests/test_gpu_split_range.py -q --timeout 120 --timeout-method thread > gpurun_out/r04a_xconv_tests.log 2>&1
rc=$?; echo "xconv tests rc=$rc"; tail -15 gpurun_out/r04a_xconv_tests.log
# a fault, abort or time limit ends the call here; ordinary test failures go on to the timing
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SH=48x48@1088x1920k3,48x48@1088x1920k3r,64x64@544x960k3r,96x48@1088x1920k3,128x64@544x960k3,128x192@544x960k3u,32x64@1088x1920k7
rm -f gpurun_out/r04a_ab.jsonl
for o in "xconv=1"; do
  timeout -k 10 200 python -u scripts/sconv_bench.py --reps 20 --shapes $SH --opt $o >> gpurun_out/r04a_ab.jsonl 2>&1 || exit 1
done
cut -c1-200 gpurun_out/r04a_ab.jsonl
rm -f gpurun_out/r04a_abl.jsonl
for d in; do
  timeout -k 10 120 python -u scripts/sconv_bench.py --reps 10 --shapes 48x48@1088x1920k3r,96x48@1088x1920k3 --opt xconv_dbg=$d >> gpurun_out/r04a_abl.jsonl 2>&1 || exit 1
done
grep shape gpurun_out/r04a_abl.jsonl | cut -c1-200
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "warp or offset_div" --timeout 120 --timeout-method thread > gpurun_out/r04a_warp.log 2>&1; rc=$?; tail -3 gpurun_out/r04a_warp.log; [ $rc -le 1 ] || exit $rc
