#!/bin/bash
# Round evidence, part 1: rocprofv3 kernel trace + stats and the FETCH_SIZE /
# WRITE_SIZE PMC passes for configs C3 (default), C2 (HEM) and C4 (YUV420
# 4K), each at one GOP lane (scripts/profile_round.sh).
set -u
cd "$(dirname "$0")/.."
R=${1:-r02d}
PROF_ARGS="--lanes 1" bash scripts/profile_round.sh $R || exit $?
PROF_ARGS="--lanes 1 --model hem" bash scripts/profile_round.sh ${R}_hem || exit $?
PROF_STEPS=4 PROF_ARGS="--lanes 1 --yuv420" bash scripts/profile_round.sh ${R}_c4 || exit $?
