#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash scripts/wconv_ablate.sh gpurun_out/r06g_wconv_ablation.jsonl && echo ablation ok
