#!/bin/bash
# per-layer PMC traffic of HEM's dominant layer (64->64 3x3 at 1088x1920, with and without a residual)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/pmc_layer.sh r03z_hem 64x64@1088x1920k3 64x64@1088x1920k3r
