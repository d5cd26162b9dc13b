#!/bin/bash
# sconvr (register-image 3x3 split kernel): correctness, then A/B against sconv.hip on the P-frame shapes
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_sconv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03p_sconv.log 2>&1
rc=$?; echo "sconv tests rc=$rc"; tail -15 gpurun_out/r03p_sconv.log; [ $rc = 0 ] || exit $rc
SH=48x48@1088x1920k3r,64x64@544x960k3r,96x48@1088x1920k3,128x192@544x960k3,96x96@272x480k3,80x48@1088x1920k3,128x64@544x960k3,64x128@544x960k3
for o in "sconvr=0" "sconvr_waves=4" "sconvr_waves=8"; do
  timeout -k 10 200 python -u scripts/sconv_bench.py --shapes $SH --opt $o > gpurun_out/r03p_bench_$o.jsonl 2>&1 || exit 1
  cut -c1-200 gpurun_out/r03p_bench_$o.jsonl
done
