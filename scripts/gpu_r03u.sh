#!/bin/bash
# latent fused FFN (slffn): parity tests, then the C3 bench at one lane with the per-layer profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_sconv.py -x -q --timeout 120 --timeout-method thread -k "latent_ffn or fused_ffn or sgemm" > gpurun_out/r03u_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r03u_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --lanes 1 --steps 12 --warmup 2 --no-cpu-baseline --profile-out gpurun_out/r03u_layers.json > gpurun_out/r03u_bench_1lane.json 2> gpurun_out/r03u_bench_1lane.err
rc=$?; echo "bench1 rc=$rc"; cut -c1-300 gpurun_out/r03u_bench_1lane.json; [ $rc = 0 ] || exit $rc
python - <<'PY'
import json
d=json.load(open('gpurun_out/r03u_layers.json'))
fam={}
for r in d:
    f=r['op'].split('<')[0].split(' ')[0]; fam[f]=fam.get(f,0)+r['ms']
print({k: round(v,2) for k,v in sorted(fam.items(), key=lambda kv:-kv[1])})
for r in d:
    if 'ffn' in r['op'] or 'sgemm' in r['op'] and '68x120' in r['op']: print(round(r['ms'],3), r['n'], r['op'][:90])
PY
