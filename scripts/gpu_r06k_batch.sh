#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash scripts/pmc_blocks.sh r06k ffn384@68x120 dwc384@68x120 k1:384x384@68x120k1 od@1088x1920 odr@1088x1920 dc48x32a@1088x1920 ffn128@272x480
