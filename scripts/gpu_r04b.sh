#!/bin/bash
# round 4: xconv timing ablations (xconv_dbg bits)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SH=48x48@1088x1920k3r,96x48@1088x1920k3,128x64@544x960k3,64x64@544x960k3r
rm -f gpurun_out/r04b_abl.jsonl
for nw in 8 4; do
for d in 0 192 194 198 206 222 254 255 64 128 2; do
  timeout -k 10 120 python -u scripts/sconv_bench.py --reps 10 --shapes $SH --opt xconv_dbg=$d --opt xconv_nw=$nw >> gpurun_out/r04b_abl.jsonl 2>&1 || exit 1
done
done
python - <<'PY'
import json
for l in open("gpurun_out/r04b_abl.jsonl"):
    if not l.startswith("{"): continue
    r = json.loads(l)
    print(r["shape"], r["opt"], r["kernel"].split("@")[0], r["us"], r["frac_mfma"])
PY
