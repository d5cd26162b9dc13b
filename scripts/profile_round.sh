#!/bin/bash
# rocprofv3 evidence for one round: kernel trace + stats, then separate
# FETCH_SIZE and WRITE_SIZE PMC passes of the same bench command, summarised
# by scripts/pmc_summary.py.  Output under gpurun_out/prof_<round>/; copy the
# summaries into profiles/ to commit them.
#   bash scripts/profile_round.sh r01
#   PROF_ARGS=--yuv420 bash scripts/profile_round.sh r01_c4   (config C4)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=${1:-r01}
O=gpurun_out/prof_$R
mkdir -p "$O"
CMD=(python bench.py --steps ${PROF_STEPS:-6} --warmup 2 --no-cpu-baseline --no-roofline ${PROF_ARGS:-})
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 600 rocprofv3 "$@" -d "$O/$name" -o run --output-format csv -- "${CMD[@]}" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 0) return 0 ;; *) tail -5 "$O/$name.log"; exit $rc ;; esac
}
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
python scripts/pmc_summary.py --trace "$O/trace" --fetch "$O/fetch" --write "$O/write" \
  --out "$O/${R}_pmc.json" --command "${CMD[*]}"
cp "$(find "$O/trace" -name '*kernel_stats.csv' | head -1)" "$O/${R}_kernel_stats.csv"
