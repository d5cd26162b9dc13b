#!/bin/bash
# Effective shader clock and MFMA busy of one conv shape under a given library /
# option set: a kernel-trace pass (durations), a GRBM pass (GPU-active cycles)
# and an SQ pass (MFMA instructions and busy cycles, waits), each its own
# rocprofv3 run.  Output under gpurun_out/pmcc_<name>/.
#   bash scripts/pmc_clock.sh NAME SHAPE LIB "OPT OPT"
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
name=$1 sh=$2 lib=$3 opts=${4:-}
out=gpurun_out/pmcc_$name
mkdir -p "$out"
args=(); for o in $opts; do args+=(--opt "$o"); done
cmd=(python scripts/sconv_bench.py --reps 5 --shapes "$sh" "${args[@]}")
run() {
  local tag=$1; shift
  DCVC_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 "$@" -d "$out/$tag" -o run --output-format csv -- "${cmd[@]}" \
    > "$out/$tag.log" 2>&1
  local rc=$?; echo "$name $tag rc=$rc"; [ $rc = 0 ] || { tail -5 "$out/$tag.log"; exit $rc; }
}
run trace --kernel-trace
run grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT
run sq --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
