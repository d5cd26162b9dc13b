#!/bin/bash
# round 4: split kernels after a change to the split arithmetic: their tests, then timings
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_xconv.py tests/test_gpu_split_range.py tests/test_gpu_sconv.py -q --timeout 200 --timeout-method thread > gpurun_out/r04g_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^FAILED" gpurun_out/r04g_tests.log | tail -8; [ $rc -le 1 ] || exit $rc
SH=48x48@1088x1920k3,48x48@1088x1920k3r,96x48@1088x1920k3,128x64@544x960k3,128x192@544x960k3u,32x64@1088x1920k7
timeout -k 10 200 python -u scripts/sconv_bench.py --reps 20 --shapes $SH > gpurun_out/r04g_ab.jsonl 2>&1 || exit 1
cut -c1-200 gpurun_out/r04g_ab.jsonl | grep shape
