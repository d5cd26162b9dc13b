#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over one microbench shape.
#   bash scripts/pmc_conv.sh SHAPE_INDEX OUTDIR
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
idx=${1:-0}; out=${2:-gpurun_out/pmc}
mkdir -p "$out"
passes=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for ctr in "${passes[@]}"; do
  timeout -k 10 240 rocprofv3 --pmc $ctr -d "$out/p$i" -o run --output-format csv \
    -- python scripts/conv_microbench.py --only "$idx" --reps 3 --fixed > "$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  case $rc in 0) ;; 124|134|137|139) exit $rc ;; *) tail -5 "$out/p$i.log" ;; esac
  i=$((i+1))
done
exit 0
