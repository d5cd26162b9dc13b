#!/bin/bash
# sconv.hip with pipelined operand reads + residual prefetch: correctness and A/B of waves per workgroup
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_sconv.py -x -q --timeout 120 --timeout-method thread -k "not sconvr" > gpurun_out/r03s_sconv.log 2>&1
rc=$?; echo "sconv tests rc=$rc"; tail -3 gpurun_out/r03s_sconv.log; [ $rc = 0 ] || exit $rc
SH=48x48@1088x1920k3r,64x64@544x960k3r,96x96@272x480k3,96x48@1088x1920k3,128x64@544x960k3
for o in "sconv_res_waves=8" "sconv_res_waves=4"; do
  for d in 0 8; do
  timeout -k 10 120 python -u scripts/sconv_bench.py --shapes $SH --opt $o --opt sconv_dbg=$d > gpurun_out/r03s_$o$d.jsonl 2>&1 || exit 1
  grep shape gpurun_out/r03s_$o$d.jsonl | python -c "import sys,json; print('$o dbg$d', [ (json.loads(l)['shape'][:9], json.loads(l)['kernel'][13:30], json.loads(l)['us']) for l in sys.stdin])"
  done
done
