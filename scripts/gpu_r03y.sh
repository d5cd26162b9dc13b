#!/bin/bash
# final tree: sgemm 2-stage A/B on short-K 1x1 layers, the whole GPU suite and smoke()
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SH=48x48@1088x1920k1,48x48@1088x1920k1r,64x64@544x960k1,32x128@1088x1920k1,64x256@272x480k1
for o in "sgemm_pd=3" "sgemm_pd=0"; do
  timeout -k 10 120 python -u scripts/sconv_bench.py --shapes $SH --opt $o > gpurun_out/r03y_ab.jsonl 2>&1 || exit 1
  grep shape gpurun_out/r03y_ab.jsonl | python -c "import sys,json; print('$o', [ (json.loads(l)['shape'][:12], json.loads(l)['kernel'][:22], json.loads(l)['us']) for l in sys.stdin])"
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03y_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "passed|failed|^FAILED|^ERROR" gpurun_out/r03y_pytest_gpu.log | tail -15
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03y_smoke.log 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -2 gpurun_out/r03y_smoke.log
[ $rc = 0 ] && [ $rc2 = 0 ]
