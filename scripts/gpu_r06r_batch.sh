#!/bin/bash
# sgemm: compile-time stage buffers + max-form input leaky ReLU (product) against the
# previous build (libdcvc_hip_sg0.so), latent-rate 1x1 shapes; then its tests
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=384x384@68x120k1,192x192@68x120k1,256x1024@68x120k1,1024x256@68x120k1,384x256@68x120k1,1536x768@68x120k1g,128x128@68x120k1
for rep in 1 2; do
  timeout -k 10 120 python -u scripts/sconv_bench.py --shapes $S --opt arm=A >> gpurun_out/r06r_sgemm_ab.jsonl 2>> gpurun_out/r06r.err || exit 1
  DCVC_HIP_LIB=libdcvc_hip_sg0.so timeout -k 10 120 python -u scripts/sconv_bench.py --shapes $S --opt arm=B >> gpurun_out/r06r_sgemm_ab.jsonl 2>> gpurun_out/r06r.err || exit 1
done
echo ab ok
( while true; do date >> gpurun_out/r06r_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 700 python -u -m pytest tests/test_gpu_dconv.py tests/test_gpu_sconv.py tests/test_gpu_repeat.py "tests/test_gpu_parity_strict.py::test_strict_parity_golden" -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06r_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r06r_pytest.log
case $rc in 124|134|137|139) exit $rc;; esac
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/r06r_A$rep.log 2>&1 || exit 1
  DCVC_HIP_LIB=libdcvc_hip_sg0.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/r06r_B$rep.log 2>&1 || exit 1
done
echo bench ok
exit $rc
