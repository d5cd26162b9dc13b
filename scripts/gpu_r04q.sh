#!/bin/bash
# round 4: 1x1 split GEMM (sgemm) configuration A/B on the DC P-frame 1x1 shapes
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
S=128x128@272x480k1,384x384@68x120k1,48x48@1088x1920k1,48x192@1088x1920k1,192x48@1088x1920k1r
out=gpurun_out/r04q_sgemm_ab.jsonl
: > $out
for o in "" "--opt sgemm=1" "--opt sgemm=2" "--opt sgemm=3" "--opt sgemm=4" "--opt sgemm=5" "--opt sgemm=6"; do
  timeout -k 10 120 python -u scripts/sconv_bench.py --reps 30 --shapes $S $o >> $out 2> gpurun_out/r04q.err
  rc=$?; echo "[$o] rc=$rc"; [ $rc = 0 ] || exit $rc
done
cat $out
