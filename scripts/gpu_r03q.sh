#!/bin/bash
# sconv.hip timing ablations (dbg mask: 1 no MFMA, 2 no publish, 4 no image loads, 8 no epilogue)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SH=48x48@1088x1920k3r,64x64@544x960k3r,96x96@272x480k3
for d in 0 1 2 4 8 6 9 14 13 15; do
  timeout -k 10 120 python -u scripts/sconv_bench.py --shapes $SH --opt sconvr=0 --opt sconv_dbg=$d > gpurun_out/r03q_dbg$d.jsonl 2>&1 || exit 1
  grep shape gpurun_out/r03q_dbg$d.jsonl | python -c "import sys,json; print($d, [ (json.loads(l)['shape'][:9], json.loads(l)['us']) for l in sys.stdin])"
done
