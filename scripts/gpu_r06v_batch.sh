#!/bin/bash
# xconv two workgroups per CU ("xconv_wpc2"): bit-identity test, then timing A/B
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_xconv_wpc2.py -m gpu -v -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r06v_pytest.log 2>&1 || { echo test failed; tail -30 gpurun_out/r06v_pytest.log; exit 1; }
echo tests ok
S=48x48@1088x1920k3,48x48@1088x1920k3r,64x48@544x960k3,48x96@544x960k3r,64x96@272x480k3
for rep in 1 2; do
  for w in 0 1; do
    timeout -k 10 120 python -u scripts/sconv_bench.py --shapes $S --opt xconv_wpc2=$w >> gpurun_out/r06v_wpc2_ab.jsonl 2>> gpurun_out/r06v.err || exit 1
  done
done
echo ab ok
