#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash scripts/wconv_ablate.sh gpurun_out/r06i_wconv_ablation.jsonl 48x48@1088x1920k3,64x64@544x960k3 "0 94 126 28 92 30 60 62 3 66" && echo ablation ok
