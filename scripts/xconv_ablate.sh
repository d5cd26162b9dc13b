#!/bin/bash
# Timing ablations of xconv3_kernel (diagnostics, wrong results): the
# XCONV_DBG build (dcvc_amd/lib/libdcvc_hip_dbg.so: build/hip_dbg/xconv.o with
# -DXCONV_DBG linked to the product's other objects) with phases skipped by
# dcvc_set_option("xconv_dbg", mask): 1 MFMAs, 2 stage barrier, 4 weight-DMA
# wait, 8 weight DMA, 16 image publish, 32 image-operand reads, 64 image
# loads, 128 residual loads and output stores.  One JSON line per (mask, shape).
#   bash scripts/xconv_ablate.sh OUT.jsonl [SHAPES]
set -u
cd "$(dirname "$0")/.."
out=$1
shapes=${2:-48x48@1088x1920k3,48x48@1088x1920k3r,96x48@1088x1920k3}
: > "$out"
for m in 0 1 192 194 252 254 253 255 16 32 48 8 12; do
  DCVC_HIP_LIB=libdcvc_hip_dbg.so timeout -k 10 120 python -u scripts/sconv_bench.py --shapes "$shapes" \
    --opt xconv_dbg=$m >> "$out" || exit 1
done
