#!/bin/bash
# HBM traffic of ONE layer shape of a split conv (scripts/sconv_bench.py), for
# bench lines whose dominant persistent kernel runs several shapes under one
# instantiation@grid (the whole-frame PMC average then mixes them): separate
# FETCH_SIZE / WRITE_SIZE passes, summarised as profiles/<name>_pmc_layers.json
#   bash scripts/pmc_layer.sh r03z_hem 64x64@1088x1920k3 64x64@1088x1920k3r
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
name=$1; shift
out=gpurun_out/pmcl_$name
mkdir -p "$out"
for sh in "$@"; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d "$out/$sh.$ctr" -o run --output-format csv \
      -- python scripts/sconv_bench.py --reps 5 --shapes "$sh" > "$out/$sh.$ctr.log" 2>&1
    rc=$?
    echo "$sh $ctr rc=$rc"
    case $rc in 0) ;; *) tail -5 "$out/$sh.$ctr.log"; exit $rc ;; esac
  done
done
python scripts/pmc_layer_summary.py "$out" "$name" "$@"
