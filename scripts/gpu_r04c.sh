#!/bin/bash
# round 4 tree: the whole GPU suite, smoke, one-lane layer profile, default bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r04c}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "passed|failed|^FAILED|^ERROR" gpurun_out/${T}_pytest_gpu.log | tail -15; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${T}_smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --lanes 1 --steps 12 --warmup 2 --no-cpu-baseline --profile-out gpurun_out/${T}_layers.json > gpurun_out/${T}_bench_1lane.json 2> gpurun_out/${T}_bench_1lane.err
rc=$?; echo "bench1 rc=$rc"; cut -c1-200 gpurun_out/${T}_bench_1lane.json; [ $rc = 0 ] || exit $rc
timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/${T}_bench_default.json
exit $rc
