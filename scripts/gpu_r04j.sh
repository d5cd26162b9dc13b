#!/bin/bash
# round 4: per-layer PMC traffic of the xconv layers that used 16-channel n-blocks in sconv
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 bash scripts/pmc_layer.sh r04j 96x48@1088x1920k3 80x48@1088x1920k3 128x64@544x960k3 48x48@1088x1920k3 48x48@1088x1920k3r
