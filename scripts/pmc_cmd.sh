#!/bin/bash
# SQ / LDS / MFMA counters of any short GPU command, one counter group per
# rocprofv3 pass, summarised per kernel by scripts/pmc_table.py.
#   bash scripts/pmc_cmd.sh gpurun_out/pmc_gemm python scripts/gemm_f32_bench.py --cfgs 0 --shapes 384x384
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
passes=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for ctr in "${passes[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d "$out/p$i" -o run --output-format csv -- "$@" > "$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  case $rc in 0) ;; *) tail -5 "$out/p$i.log"; exit $rc ;; esac
  i=$((i+1))
done
python scripts/pmc_table.py "$out"
