#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_wconv.py -m gpu -v -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r06h_wconv_pytest.log 2>&1 || { echo wconv tests failed; tail -30 gpurun_out/r06h_wconv_pytest.log; exit 1; }
echo wconv tests ok
S=48x48@1088x1920k3,48x48@1088x1920k3r,64x64@544x960k3r,64x64@544x960k3,128x64@544x960k3,192x192@68x120k3r
for rep in 1 2; do
  for w in 0 1; do
    timeout -k 10 120 python -u scripts/sconv_bench.py --shapes $S --opt wconv=$w >> gpurun_out/r06h_wconv_ab.jsonl 2>> gpurun_out/r06h_wconv_ab.err || exit 1
  done
done
echo wconv ab ok
bash scripts/wconv_ablate.sh gpurun_out/r06h_wconv_ablation.jsonl 48x48@1088x1920k3,64x64@544x960k3 "0 128 1 2 4 8 16 32 64 31" && echo ablation ok
