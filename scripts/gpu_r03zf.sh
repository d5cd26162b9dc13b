#!/bin/bash
# sgemm pixel shuffle: split conv tests, the 1x1 shuffle shapes, whole GPU suite, one-lane and default bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_sconv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03zf_sconv.log 2>&1
rc=$?; echo "sconv tests rc=$rc"; tail -2 gpurun_out/r03zf_sconv.log; [ $rc = 0 ] || exit $rc
SH=64x256@272x480k1,64x128@544x960k1,128x256@272x480k1
for o in "sgemm=-1" "sgemm=0"; do
  timeout -k 10 150 python -u - > gpurun_out/r03zf_ab_$o.txt 2>&1 <<PY || exit 1
import sys, json, re, torch
sys.argv = ["x"]
from dcvc_amd import hip as K
K.set_option("sgemm", int("$o".split("=")[1]))
dev = torch.device("cuda", 0)
for sh in "$SH".split(","):
    m = re.fullmatch(r"(\d+)x(\d+)@(\d+)x(\d+)k1", sh)
    cin, cout, H, W = (int(m.group(i)) for i in range(1, 5))
    cw = K.ConvW(torch.randn(cout, cin, 1, 1) / cin ** 0.5, torch.randn(cout) * 0.1, 1, K.F16X3, dev)
    x = K.from_nchw(torch.randn(1, cin, H, W, device=dev), K.F32)
    for _ in range(3):
        K.conv(cw, x, shuffle=True, act=K.ACT_LRELU, slope=0.01)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        K.conv(cw, x, shuffle=True, act=K.ACT_LRELU, slope=0.01)
    e1.record(); torch.cuda.synchronize()
    print(json.dumps({"shape": sh, "opt": "$o", "kernel": K.lib().dcvc_last_kernel().decode(), "us": round(e0.elapsed_time(e1) * 50, 2)}))
PY
  cat gpurun_out/r03zf_ab_$o.txt | grep shape
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03zf_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "passed|failed|^FAILED|^ERROR" gpurun_out/r03zf_pytest_gpu.log | tail -15; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03zf_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r03zf_smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --lanes 1 --steps 12 --warmup 2 --no-cpu-baseline --profile-out gpurun_out/r03zf_layers.json > gpurun_out/r03zf_bench_1lane.json 2> gpurun_out/r03zf_bench_1lane.err
rc=$?; echo "bench1 rc=$rc"; cut -c1-200 gpurun_out/r03zf_bench_1lane.json; [ $rc = 0 ] || exit $rc
timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03zf_bench_default.json 2> gpurun_out/r03zf_bench_default.err
rc=$?; echo "bench rc=$rc"; cut -c1-200 gpurun_out/r03zf_bench_default.json
exit $rc
