# Two bench processes sharing the GPU (the reference's several-workers-per-GPU
# deployment); both must finish without an encoder/decoder mismatch.
#   ENVS="HSA_ENABLE_SDMA=0" bash scripts/corun_pair.sh name [bench args]
name=$1; shift
env $ENVS timeout -k 10 150 python bench.py --steps 24 --no-cpu-baseline --no-roofline "$@" > gpurun_out/co_${name}_a.log 2>&1 & A=$!
env $ENVS timeout -k 10 150 python bench.py --steps 24 --no-cpu-baseline --no-roofline "$@" > gpurun_out/co_${name}_b.log 2>&1 & B=$!
wait $A; ra=$?; wait $B; rb=$?; echo "$name [$ENVS] a=$ra b=$rb"
case "$ra$rb" in *124*|*134*|*137*|*139*) exit 1;; esac
exit 0
