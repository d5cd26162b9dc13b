#!/bin/bash
# dconv 1x1: per-tile input offsets (product) against the previous build
# (libdcvc_hip_dc0.so); then its tests
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=48x192@1088x1920k1,192x48@1088x1920k1r,64x64@544x960k1,128x128@272x480k1,64x256@544x960k1u,48x64@1088x1920k1,56x64@1088x1920k3s2
for rep in 1 2; do
  timeout -k 10 120 python -u scripts/sconv_bench.py --shapes $S --opt arm=A >> gpurun_out/r06s_dconv_ab.jsonl 2>> gpurun_out/r06s.err || exit 1
  DCVC_HIP_LIB=libdcvc_hip_dc0.so timeout -k 10 120 python -u scripts/sconv_bench.py --shapes $S --opt arm=B >> gpurun_out/r06s_dconv_ab.jsonl 2>> gpurun_out/r06s.err || exit 1
done
echo ab ok
timeout -k 10 600 python -u -m pytest tests/test_gpu_dconv.py tests/test_gpu_repeat.py tests/test_gpu_split_range.py "tests/test_gpu_parity_strict.py::test_strict_parity_golden" -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06s_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r06s_pytest.log
exit $rc
