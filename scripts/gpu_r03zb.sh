#!/bin/bash
# sgemm depth 1 vs 2 A/B, the whole GPU suite, smoke, one-lane bench with the layer profile, default bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SH=128x128@272x480k1,128x64@544x960k1r,192x192@68x120k1,384x384@68x120k1,128x128@544x960k1,96x48@1088x1920k1,48x48@1088x1920k1
for o in "sgemm_pd=1" "sgemm_pd=2"; do
  timeout -k 10 120 python -u scripts/sconv_bench.py --shapes $SH --opt $o > gpurun_out/r03zb_ab.jsonl 2>&1 || exit 1
  grep shape gpurun_out/r03zb_ab.jsonl | python -c "import sys,json; print('$o', [ (json.loads(l)['shape'][:14], json.loads(l)['us']) for l in sys.stdin])"
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03zb_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "passed|failed|^FAILED|^ERROR" gpurun_out/r03zb_pytest_gpu.log | tail -15; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03zb_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r03zb_smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --lanes 1 --steps 12 --warmup 2 --no-cpu-baseline --profile-out gpurun_out/r03zb_layers.json > gpurun_out/r03zb_bench_1lane.json 2> gpurun_out/r03zb_bench_1lane.err
rc=$?; echo "bench1 rc=$rc"; cut -c1-200 gpurun_out/r03zb_bench_1lane.json; [ $rc = 0 ] || exit $rc
timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03zb_bench_default.json 2> gpurun_out/r03zb_bench_default.err
rc=$?; echo "bench rc=$rc"; cut -c1-200 gpurun_out/r03zb_bench_default.json
exit $rc
