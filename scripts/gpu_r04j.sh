#!/bin/bash
# round 4: depthwise kernel tests; per-layer PMC traffic of the xconv layers
# that used 16-channel n-blocks in sconv
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "dwconv or warp or offset_div" --timeout 120 --timeout-method thread > gpurun_out/r04j_kernels.log 2>&1
rc=$?; tail -3 gpurun_out/r04j_kernels.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 bash scripts/pmc_layer.sh r04j 96x48@1088x1920k3 80x48@1088x1920k3 128x64@544x960k3 48x48@1088x1920k3 48x48@1088x1920k3r
