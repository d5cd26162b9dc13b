#!/bin/bash
# sconv knob A/B on the SpyNet 7x7 layers, the stride-2 and the BN=16 layers
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
SH=32x64@1088x1920k7,64x32@1088x1920k7,32x16@1088x1920k7,56x64@1088x1920k3s2,128x192@544x960k3,96x48@1088x1920k3
for o in "sconv_rw=0" "sconv_waves=4" "sconv_rw=4" "sconv_rw=1" "sconv_resident=0" "sconv_res_waves=4"; do
  timeout -k 10 150 python -u scripts/sconv_bench.py --shapes $SH --opt $o > gpurun_out/r03zd_ab.jsonl 2>&1 || exit 1
  grep shape gpurun_out/r03zd_ab.jsonl | python -c "import sys,json; print('$o', [ (json.loads(l)['shape'][:13], json.loads(l)['kernel'][13:40], json.loads(l)['us']) for l in sys.stdin])"
done
