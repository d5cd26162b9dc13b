#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=48x48@1088x1920k3
bash scripts/pmc_clock.sh xprod $S libdcvc_hip.so "" && \
bash scripts/pmc_clock.sh xmfma $S libdcvc_hip_dbg.so "xconv_dbg=254" && \
bash scripts/pmc_clock.sh wmfma $S libdcvc_hip_wdbg.so "wconv=1 wconv_dbg=126" && \
bash scripts/pmc_clock.sh wprod $S libdcvc_hip.so "wconv=1"
