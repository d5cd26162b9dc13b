#!/bin/bash
# PMC counters of the fused block, latent-rate and gather kernels
# (scripts/block_bench.py shapes; "k1:" prefix = a 1x1 conv of
# scripts/sconv_bench.py), one rocprofv3 pass per counter group and shape:
#   L2   TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum      (L2 requests and hit rate)
#   HBM  FETCH_SIZE / WRITE_SIZE                    (separate passes)
#   SQ   wave cycles, waits, instruction mix
#   TA   TA / TCP busy and request counts           (gather kernels)
# Counters missing from `rocprofv3 -L` are dropped from their pass.  Summary:
# scripts/pmc_blocks_summary.py -> gpurun_out/pmcb_<name>/<name>_pmc_blocks.json
#   bash scripts/pmc_blocks.sh r06 ffn384@68x120 dwc384@68x120 k1:384x384@68x120k1 od@1088x1920
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
name=$1; shift
out=gpurun_out/pmcb_$name
mkdir -p "$out"
timeout -s KILL 60 rocprofv3 -L > "$out/counters.txt" 2>&1 || true
have() { grep -qw "$1" "$out/counters.txt"; }
pick() { local r="" b; for c in "$@"; do b=${c%_sum}; b=${b%_avr}; have "$b" && r="$r $c"; done; echo $r; }
declare -A G
G[L2]=$(pick TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum)
G[FETCH]=FETCH_SIZE
G[WRITE]=WRITE_SIZE
G[SQ]=$(pick SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS)
G[TA]=$(pick TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum)
echo "groups: L2=[${G[L2]}] SQ=[${G[SQ]}] TA=[${G[TA]}]"
for sh in "$@"; do
  if [[ $sh == k1:* ]]; then cmd=(python scripts/sconv_bench.py --reps 5 --shapes "${sh#k1:}")
  else cmd=(python scripts/block_bench.py --reps 5 --shapes "$sh"); fi
  for g in L2 FETCH WRITE SQ TA; do
    [ -n "${G[$g]}" ] || continue
    timeout -s KILL 120 rocprofv3 --pmc ${G[$g]} -d "$out/$sh.$g" -o run --output-format csv -- "${cmd[@]}" \
      > "$out/$sh.$g.log" 2>&1
    rc=$?
    echo "$sh $g rc=$rc"
    case $rc in 0) ;; *) tail -5 "$out/$sh.$g.log"; exit $rc ;; esac
  done
done
python scripts/pmc_blocks_summary.py "$out" "$name" "$@"
