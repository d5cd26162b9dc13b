#!/bin/bash
# whole-bench A/B (C3, 3 lanes): product / slffn+sldc 4 pixel blocks at C=384 / wconv on
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/r06l_A$rep.log 2>&1 || exit 1
  tail -1 gpurun_out/r06l_A$rep.log | cut -c1-200
  DCVC_HIP_LIB=libdcvc_hip_pb4.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/r06l_P$rep.log 2>&1 || exit 1
  tail -1 gpurun_out/r06l_P$rep.log | cut -c1-200
  DCVC_HIP_OPTIONS=wconv=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/r06l_W$rep.log 2>&1 || exit 1
  tail -1 gpurun_out/r06l_W$rep.log | cut -c1-200
done
