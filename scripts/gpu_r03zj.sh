#!/bin/bash
# final tree: wide-layer rule at 8+ n-blocks; split conv tests, the whole GPU suite, smoke, one-lane profile, bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 150 python -u scripts/sconv_bench.py --shapes 192x96@272x480k3,192x256@272x480k3,128x192@544x960k3 > gpurun_out/r03zj_ab.jsonl 2>&1 || exit 1
cut -c1-160 gpurun_out/r03zj_ab.jsonl | grep shape
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03zj_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "passed|failed|^FAILED|^ERROR" gpurun_out/r03zj_pytest_gpu.log | tail -15; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03zj_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r03zj_smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --lanes 1 --steps 12 --warmup 2 --no-cpu-baseline --profile-out gpurun_out/r03zj_layers.json > gpurun_out/r03zj_bench_1lane.json 2> gpurun_out/r03zj_bench_1lane.err
rc=$?; echo "bench1 rc=$rc"; cut -c1-200 gpurun_out/r03zj_bench_1lane.json; [ $rc = 0 ] || exit $rc
timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03zj_bench_default.json 2> gpurun_out/r03zj_bench_default.err
rc=$?; echo "bench rc=$rc"; cut -c1-200 gpurun_out/r03zj_bench_default.json
exit $rc
