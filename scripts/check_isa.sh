#!/bin/bash
# Build-time ISA check of libdcvc_hip's gfx950 code objects.
#
# The kernels must not contain packed-f32 VALU instructions (v_pk_mul_f32,
# v_pk_add_f32, v_pk_fma_f32): with them, kernels of a codec that shares the
# GPU with another process (or with another stream's work on a second
# hardware queue) intermittently produced wrong values in the low lane of
# packed results (the co-running divergence), while the same
# build without them ran clean.  The Makefile builds with -fno-slp-vectorize,
# which keeps the compiler from forming them; this check fails the build if
# any appear (a new source using packed math explicitly, or a flag change).
#   scripts/check_isa.sh build/hip/*.o
set -eu
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
bad=0
for o in "$@"; do
  n=$(basename "$o" .o)
  "$B/llvm-objcopy" --dump-section .hip_fatbin="$T/$n.fat" "$o"
  "$B/clang-offload-bundler" --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
    --input="$T/$n.fat" --output="$T/$n.co"
  "$B/llvm-objdump" -d "$T/$n.co" > "$T/$n.s"
  c=$(grep -cE "v_pk_(mul|add|fma)_f32" "$T/$n.s" || true)
  if [ "$c" != "0" ]; then
    echo "check_isa: $o has $c packed-f32 instructions" >&2
    bad=1
  fi
  # xconv3_kernel counts its vector-memory operations per stage for exact
  # vmcnt waits (xconv.hip): a register spill's scratch traffic would break
  # that count, so no instantiation may spill
  s=$(awk '/^[0-9a-f]+ <.*xconv3_kernel/{k=1; next} /^[0-9a-f]+ </{k=0} k && /scratch_/' "$T/$n.s" | wc -l)
  if [ "$s" != "0" ]; then
    echo "check_isa: $o has $s scratch instructions in xconv3_kernel instantiations" >&2
    bad=1
  fi
  # the split-precision kernels written since (dconv, sffn): no scratch at
  # all (a private array the compiler could not keep in registers made one
  # dconv build 9x slower, profiles/r05h_micro.jsonl)
  s=$(awk '/^[0-9a-f]+ <.*(dconv_kernel|sffn_kernel|wconv3_kernel)/{k=1; next} /^[0-9a-f]+ </{k=0} k && /scratch_/' "$T/$n.s" | wc -l)
  if [ "$s" != "0" ]; then
    echo "check_isa: $o has $s scratch instructions in dconv / sffn / wconv kernels" >&2
    bad=1
  fi
done
exit $bad
