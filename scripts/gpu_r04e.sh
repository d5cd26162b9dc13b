#!/bin/bash
# round 4 evidence: rocprofv3 kernel stats + FETCH/WRITE PMC of the one-lane
# bench, SQ counters of the dominant xconv shapes
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${1:-r04e}
PROF_ARGS="--lanes 1" timeout -k 10 1000 bash scripts/profile_round.sh $T || exit $?
timeout -k 10 300 bash scripts/pmc_cmd.sh gpurun_out/${T}_sq python scripts/sconv_bench.py --reps 3 --shapes 48x48@1088x1920k3,48x48@1088x1920k3r > gpurun_out/${T}_sq.txt 2>&1
rc=$?; grep -E "xconv|sconv" gpurun_out/${T}_sq.txt | cut -c1-400; exit $rc
