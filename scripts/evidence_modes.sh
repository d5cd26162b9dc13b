#!/bin/bash
# Extra bench lines for the record: C3 in fp32 parity precision, C3 at one
# GOP lane (per-frame latency), C3 with the labelled bf16 entropy tail.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for m in "parity:--precision parity" "1lane:--lanes 1" "bf16tail:--precision fast-bf16-tail"; do
  n=${m%%:*}; a=${m#*:}
  timeout -k 10 600 python bench.py $a --no-cpu-baseline > gpurun_out/bench_$n.log 2>&1
  rc=$?; echo "bench $n rc=$rc"; [ $rc = 0 ] || exit $rc
done
