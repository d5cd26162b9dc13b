#!/bin/bash
# Timing ablations of wconv3_kernel (diagnostics, wrong results): the
# WCONV_DBG build (dcvc_amd/lib/libdcvc_hip_wdbg.so: build/hip_wdbg/wconv.o
# with -DWCONV_DBG linked to the product's other objects) with phases skipped
# by dcvc_set_option("wconv_dbg", mask): 1 consumer MFMAs, 2 consumer LDS
# operand reads, 4 producer publish, 8 producer image loads, 16 weight DMA and
# its waits, 32 stage barriers, 64 residual loads and output stores, 128 the
# consumer waves' raised priority.  One JSON line per (mask, shape).
#   bash scripts/wconv_ablate.sh OUT.jsonl [SHAPES] [MASKS]
set -u
cd "$(dirname "$0")/.."
out=$1
shapes=${2:-48x48@1088x1920k3,64x64@544x960k3}
masks=${3:-0 128 1 2 3 4 8 12 16 28 32 64 31}
: > "$out"
for m in $masks; do
  DCVC_HIP_LIB=libdcvc_hip_wdbg.so timeout -k 10 120 python -u scripts/sconv_bench.py --shapes "$shapes" \
    --opt wconv=1 --opt wconv_dbg=$m >> "$out" || exit 1
done
