# Co-running correctness: two bench processes share the GPU; with kernel
# families switched off through DCVC_OPTS.  A "malformed stream" means an
# encoder/decoder mismatch, i.e. a kernel whose result depends on co-running work.
pair() { name=$1; opts=$2
  DCVC_OPTS=$opts timeout -k 10 150 python bench.py --steps 16 --no-cpu-baseline --no-roofline > gpurun_out/co_${name}_a.log 2>&1 & A=$!
  DCVC_OPTS=$opts timeout -k 10 150 python bench.py --steps 16 --no-cpu-baseline --no-roofline > gpurun_out/co_${name}_b.log 2>&1 & B=$!
  wait $A; ra=$?; wait $B; rb=$?; echo "$name [$opts] a=$ra b=$rb"
  case "$ra$rb" in *124*|*134*|*137*|*139*) exit 1;; esac; }
pair alloff conv3x3_persistent=0,dcb_persistent=0,conv3x3_resident=0,conv3x3=0,gemm1x1=0
pair allon ""
pair gemm_only conv3x3_persistent=0,dcb_persistent=0,conv3x3_resident=0,conv3x3=0
pair conv3_fixed conv3x3_persistent=0,dcb_persistent=0,conv3x3_resident=0,gemm1x1=0
pair conv3_res conv3x3_persistent=0,dcb_persistent=0,gemm1x1=0
pair conv3p dcb_persistent=0,conv3x3_resident=0,gemm1x1=0
pair dcbp conv3x3_persistent=0,conv3x3_resident=0,conv3x3=0,gemm1x1=0
exit 0
