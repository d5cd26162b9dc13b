#!/bin/bash
# GOP-lane scan of the split-precision C3 bench (2, 4, 5 lanes; 3 is the default line)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for L in 2 4 5; do
  timeout -k 10 500 python -u bench.py --lanes $L --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03zi_lanes$L.json 2> gpurun_out/r03zi_lanes$L.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r03zi_lanes$L.json')); print($L, d['value'], d['config']['ms_P'])"
done
