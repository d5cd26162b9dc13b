#!/bin/bash
# round-3 evidence part 1: the whole GPU suite and smoke() on this tree
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03v_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "passed|failed|^FAILED|^ERROR" gpurun_out/r03v_pytest_gpu.log | tail -15
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03v_smoke.log 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -3 gpurun_out/r03v_smoke.log
exit $rc
