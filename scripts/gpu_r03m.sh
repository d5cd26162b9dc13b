#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SH=1024x384@68x120k1,384x384@68x120k1,384x1024@68x120k1,768x192@68x120k1,192x768@68x120k1,192x192@68x120k1,128x128@272x480k1,48x48@1088x1920k1,128x64@544x960k1r
for pd in 2 5; do for o in 1 2 4 5 6; do
  timeout -k 10 120 python -u scripts/sconv_bench.py --shapes $SH --opt sgemm=$o --opt sgemm_pd=$pd > gpurun_out/r03m_sgemm_${o}_$pd.log 2>&1 || exit 1
done; done
echo done
