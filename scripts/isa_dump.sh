#!/bin/bash
# Disassemble the gfx950 code object of one built object file:
#   scripts/isa_dump.sh build/hip/sgemm.o > /tmp/sgemm.s
set -eu
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
"$B/llvm-objcopy" --dump-section .hip_fatbin="$T/x.fat" "$1"
"$B/clang-offload-bundler" --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input="$T/x.fat" --output="$T/x.co"
"$B/llvm-objdump" -d "$T/x.co"
