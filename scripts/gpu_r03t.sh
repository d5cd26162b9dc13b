#!/bin/bash
# tightened bf16 kernel tests; sconv A/B: resident vs streamed weights (two workgroups per CU)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q --timeout 120 --timeout-method thread > gpurun_out/r03t_kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/r03t_kernels.log | tail -15
SH=48x48@1088x1920k3r,64x64@544x960k3r,96x96@272x480k3,96x48@1088x1920k3,128x64@544x960k3,128x192@544x960k3
for o in "sconv_resident=1" "sconv_resident=0 --opt sconv_waves=4" "sconv_resident=0 --opt sconv_waves=8" "sconv_resident=0 --opt sconv_waves=4 --opt sconv_occupancy=2"; do
  timeout -k 10 120 python -u scripts/sconv_bench.py --shapes $SH --opt $o > gpurun_out/r03t_ab.jsonl 2>&1 || exit 1
  grep shape gpurun_out/r03t_ab.jsonl | python -c "import sys,json; print('$o', [ (json.loads(l)['shape'][:9], json.loads(l)['kernel'][13:34], json.loads(l)['us']) for l in sys.stdin])"
done
