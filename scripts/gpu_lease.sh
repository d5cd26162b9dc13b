#!/bin/bash
# One gpurun lease, steps chosen by the STEPS env var (space separated), each
# GPU step under its own time limit; the script ends at the first failing step.
#   bench1   one-lane C3 bench with the per-layer P-frame profile (--profile-out)
#   bench3   the default C3 bench line (3 lanes)
#   tests    pytest -m gpu   (PYTEST_ARGS: targets / options, default tests)
#   smoke    __graft_entry__.smoke()
#   micro    scripts/sconv_bench.py $MICRO_ARGS, then $MICRO_ARGS2..4 if set (kernel microbenchmarks)
#   prof     rocprofv3 kernel stats of a one-lane bench
#   ab       interleaved A/B of $AB_SHAPES (scripts/$AB_TOOL, default sconv_bench.py): the product library, then
#            dcvc_amd/lib/$AB_LIB (DCVC_HIP_LIB), twice each, one JSON line per shape and arm
#   bench1b  bench1 with DCVC_HIP_LIB=$AB_LIB
#   block    scripts/block_bench.py $BLOCK_ARGS (fused blocks / gathers), repeated for $BLOCK_ARGS2 if set
#   kstats   rocprofv3 kernel stats of: python $KSTATS_CMD
#   pmc      SQ / LDS / MFMA and HBM counters (scripts/pmc_cmd.sh) of: python $PMC_CMD
# TAG names the outputs: gpurun_out/$TAG_*.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-run}
STEPS=${STEPS:-bench1}
for s in $STEPS; do
  case $s in
    bench1) timeout -k 10 600 python bench.py --lanes 1 --steps 12 --warmup 3 --no-cpu-baseline \
              --profile-out gpurun_out/${TAG}_layers.json ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench1.log 2>&1 ;;
    bench3) timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench3.log 2>&1 ;;
    tests)  timeout -k 10 1000 python -u -m pytest ${PYTEST_ARGS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 600 \
              --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 ;;
    smoke)  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 ;;
    micro)  { timeout -k 10 300 python -u scripts/sconv_bench.py ${MICRO_ARGS:-} &&
              for m in "${MICRO_ARGS2:-}" "${MICRO_ARGS3:-}" "${MICRO_ARGS4:-}"; do
                if [ -n "$m" ]; then timeout -k 10 300 python -u scripts/sconv_bench.py $m || exit 1; fi
              done; } > gpurun_out/${TAG}_micro.jsonl 2> gpurun_out/${TAG}_micro.err ;;
    prof)   timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv \
              -- python bench.py --lanes 1 --steps 6 --warmup 2 --no-cpu-baseline --no-roofline \
              > gpurun_out/${TAG}_prof.log 2>&1 ;;
    block)  { timeout -k 10 300 python -u scripts/block_bench.py ${BLOCK_ARGS:-} &&
              if [ -n "${BLOCK_ARGS2:-}" ]; then timeout -k 10 300 python -u scripts/block_bench.py ${BLOCK_ARGS2}; fi; } \
              > gpurun_out/${TAG}_block.jsonl 2> gpurun_out/${TAG}_block.err ;;
    kstats) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_kstats -o run --output-format csv \
              -- python ${KSTATS_CMD} > gpurun_out/${TAG}_kstats.log 2>&1 ;;
    pmc)    bash scripts/pmc_cmd.sh gpurun_out/${TAG}_pmc python ${PMC_CMD} > gpurun_out/${TAG}_pmc.log 2>&1 ;;
    ab)     { for rep in 1 2; do
                timeout -k 10 300 python -u scripts/${AB_TOOL:-sconv_bench.py} --shapes ${AB_SHAPES} --opt arm=A || exit 1
                DCVC_HIP_LIB=${AB_LIB} timeout -k 10 300 python -u scripts/${AB_TOOL:-sconv_bench.py} --shapes ${AB_SHAPES} --opt arm=B || exit 1
              done; } > gpurun_out/${TAG}_ab.jsonl 2> gpurun_out/${TAG}_ab.err ;;
    bench1b) DCVC_HIP_LIB=${AB_LIB} timeout -k 10 600 python bench.py --lanes 1 --steps 12 --warmup 3 --no-cpu-baseline \
              --profile-out gpurun_out/${TAG}_layers_b.json ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench1b.log 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  rc=$?
  echo "step $s rc=$rc"
  [ $rc = 0 ] || exit $rc
done
exit 0
