#!/bin/bash
# (one gpurun call: latent-kernel A/B, then the GPU parity / range / repeat suites with a heartbeat file)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=ffn384@68x120,dwc384@68x120,ffn192@68x120,dwc192@68x120
for rep in 1 2; do
  timeout -k 10 120 python -u scripts/block_bench.py --shapes $S --opt arm=A >> gpurun_out/r06e_lat_ab.jsonl 2>> gpurun_out/r06e_lat_ab.err || exit 1
  DCVC_HIP_LIB=libdcvc_hip_c.so timeout -k 10 120 python -u scripts/block_bench.py --shapes $S --opt arm=B >> gpurun_out/r06e_lat_ab.jsonl 2>> gpurun_out/r06e_lat_ab.err || exit 1
done
echo ab ok
( while true; do date >> gpurun_out/r06e_heartbeat.txt; sleep 50; done ) &
HB=$!
timeout -k 10 1050 python -u -m pytest tests/test_gpu_split_range.py tests/test_gpu_repeat.py tests/test_gpu_sconv.py tests/test_gpu_parity_strict.py -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r06e_pytest.log 2>&1
rc=$?
kill $HB
echo pytest rc=$rc
exit $rc
