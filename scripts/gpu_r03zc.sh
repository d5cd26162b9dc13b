#!/bin/bash
# sconv A/B: streamed weights with short tiles (two or three workgroups per CU) vs resident
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
SH=48x48@1088x1920k3r,64x64@544x960k3r,96x96@272x480k3,64x64@1088x1920k3,96x48@1088x1920k3,128x64@544x960k3
for o in "sconv_rw=0" "sconv_resident=0 --opt sconv_waves=4 --opt sconv_rw=2" "sconv_resident=0 --opt sconv_waves=4 --opt sconv_rw=1" "sconv_res_waves=4 --opt sconv_rw=2"; do
  timeout -k 10 150 python -u scripts/sconv_bench.py --shapes $SH --opt $o > gpurun_out/r03zc_ab.jsonl 2>&1 || exit 1
  grep shape gpurun_out/r03zc_ab.jsonl | python -c "import sys,json; print('$o', [ (json.loads(l)['shape'][:13], json.loads(l)['kernel'][13:40], json.loads(l)['us']) for l in sys.stdin])"
done
