#!/bin/bash
# round 4: stride-2 3x3 split conv (sconv) dispatch A/B on the DC 1080p P-frame shapes
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
S=56x64@1088x1920k3s2,48x64@1088x1920k3s2,128x96@544x960k3s2,64x64@1088x1920k3s2
out=gpurun_out/r04o_sconv_s2_ab.jsonl
: > $out
for o in "" "--opt sconv_rw=2" "--opt sconv_rw=4" "--opt sconv_res_waves=4" "--opt sconv_resident=0" \
         "--opt sconv_resident=0 --opt sconv_waves=4" "--opt sconv_resident=0 --opt sconv_rw=2"; do
  timeout -k 10 120 python -u scripts/sconv_bench.py --reps 20 --shapes $S $o >> $out 2> gpurun_out/r04o.err
  rc=$?; echo "[$o] rc=$rc"; [ $rc = 0 ] || exit $rc
done
cat $out
