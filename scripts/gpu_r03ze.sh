#!/bin/bash
# the wide-layer n-block rule: split conv tests and the affected shapes
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_sconv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ze_sconv.log 2>&1
rc=$?; echo "sconv tests rc=$rc"; tail -2 gpurun_out/r03ze_sconv.log; [ $rc = 0 ] || exit $rc
timeout -k 10 150 python -u scripts/sconv_bench.py --shapes 128x192@544x960k3,192x256@272x480k3,96x48@1088x1920k3,128x64@544x960k3 > gpurun_out/r03ze_ab.jsonl 2>&1 || exit 1
cut -c1-200 gpurun_out/r03ze_ab.jsonl
