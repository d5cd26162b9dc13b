#!/bin/bash
# Device-only build of xconv.hip for one input channel count, register /
# spill report per instantiation and the disassembly in /tmp/xprobe<CIN>.s.
#   bash scripts/isa_probe.sh CIN [BN [NRES [RW [KS]]]]   (RW 2: 8 waves of 2 rows; 4: 4 waves of 4 rows; KS 3 or 7)
set -eu
cd "$(dirname "$0")/.."
c=$1
bn=${2:-48}
nres=${3:-0}
rw=${4:-2}
ks=${5:-3}
B=/opt/rocm/lib/llvm/bin
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-slp-vectorize -DXCONV_ISA_PROBE=$c -DXCONV_PROBE_BN=$bn -DXCONV_PROBE_NRES=$nres -DXCONV_PROBE_RW=$rw -DXCONV_PROBE_KS=$ks ${XFLAGS:-} \
  --cuda-device-only -c -o /tmp/xprobe$c.co dcvc_amd/csrc/hip/xconv.hip -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs|AGPRs|Spill" | sed 's/.*remark: *//;s/ \[-Rpass.*//' | paste - - - - - |
  sed 's/_ZN12_GLOBAL__N_113xconv3_kernelI//;s/EEvNS_2XPE//;s/Function Name: //'
$B/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=/tmp/xprobe$c.co \
  --output=/tmp/xprobe$c.elf
$B/llvm-objdump -d /tmp/xprobe$c.elf > /tmp/xprobe$c.s
