#!/bin/bash
# A/B session: bit-identity tests of the changed kernels, microbench
# timings per epilogue mode, then the C3 bench.
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "persistent_kernel or conv3x3 or conv7 or dcb" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_ab.log 2>&1 || { tail -30 gpurun_out/t_ab.log; exit 1; }
tail -1 gpurun_out/t_ab.log
S=48x48@1088x1920r,64x64@544x960r,96x96@272x480r,96x48@1088x1920r,128x64@544x960r,64x64@1088x1920r
for m in 0 2; do timeout -k 10 120 python scripts/conv3_bench.py --shapes $S --opt conv3x3_epilogue=$m; done
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_ab.log 2>&1
grep '^{' gpurun_out/bench_ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['ms_P'], d['roofline']['avg_launch_us'], d['roofline']['P_frame_kernels'], d['roofline']['families_ms_per_P_frame'])"
