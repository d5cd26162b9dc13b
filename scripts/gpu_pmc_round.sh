set -u
bash scripts/pmc_cmd.sh gpurun_out/pmc_c3 python scripts/conv3_bench.py --reps 5 --shapes 48x48@1088x1920r > gpurun_out/pmc_c3.txt 2>&1 && \
bash scripts/pmc_cmd.sh gpurun_out/pmc_g python scripts/gemm_f32_bench.py --reps 5 --cfgs 0 --shapes 384x384,384x1024,1024x384 > gpurun_out/pmc_g.txt 2>&1 && \
bash scripts/pmc_cmd.sh gpurun_out/pmc_d python scripts/dcb_bench.py --reps 5 --shapes 64x48@1088x1920,128x128@272x480 --kernels stream > gpurun_out/pmc_d.txt 2>&1 && \
timeout -k 10 600 python bench.py --cpu-baseline-workers 16 > gpurun_out/cpu_workers.log 2>&1
echo rc=$?
