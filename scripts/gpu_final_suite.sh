#!/bin/bash
# usage: bash scripts/gpu_final_suite.sh [TAG]   (output names gpurun_out/TAG_*)
# the full GPU suite (verbose, heartbeat file), then smoke()
T=${1:-r06t}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
( while true; do date >> gpurun_out/${T}_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 1080 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
echo "smoke rc=$?"; tail -2 gpurun_out/${T}_smoke.log
exit $rc
