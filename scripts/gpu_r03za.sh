#!/bin/bash
# sgemm stages-in-flight A/B on the mid-K 1x1 layers
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
SH=128x128@272x480k1,128x64@544x960k1r,192x192@68x120k1,384x384@68x120k1,128x128@544x960k1,96x48@1088x1920k1
for o in "sgemm_pd=2" "sgemm_pd=3"; do
  timeout -k 10 120 python -u scripts/sconv_bench.py --shapes $SH --opt $o > gpurun_out/r03za_ab.jsonl 2>&1 || exit 1
  grep shape gpurun_out/r03za_ab.jsonl | python -c "import sys,json; print('$o', [ (json.loads(l)['shape'][:14], json.loads(l)['kernel'][:22], json.loads(l)['us']) for l in sys.stdin])"
done
