#!/bin/bash
# fps of the default C3 bench at several GOP-lane counts (no CPU baseline,
# no roofline pass), one bench process per count, each under its own limit.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for L in ${LANES:-2 3 4 5}; do
  timeout -k 10 300 python bench.py --lanes $L --no-cpu-baseline --no-roofline > gpurun_out/lanes_$L.log 2>&1
  rc=$?; echo "lanes=$L rc=$rc"; tail -1 gpurun_out/lanes_$L.log | cut -c1-200
  case $rc in 0) ;; *) exit $rc ;; esac
done
