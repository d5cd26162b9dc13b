# Two corun_debug.py processes sharing the GPU; each exits 3 at the first
# frame whose decoder disagrees with its encoder, printing where.
#   bash scripts/corun_debug.sh [args for corun_debug.py]
timeout -k 10 200 python scripts/corun_debug.py "$@" > gpurun_out/corun_dbg_a.log 2>&1 & A=$!
timeout -k 10 200 python scripts/corun_debug.py "$@" > gpurun_out/corun_dbg_b.log 2>&1 & B=$!
wait $A; ra=$?; wait $B; rb=$?; echo "corun_debug a=$ra b=$rb"
case "$ra$rb" in *124*|*134*|*137*|*139*) exit 1;; esac
exit 0
