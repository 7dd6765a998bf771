set -u
mkdir -p gpurun_out
bash tools/gpu_r2.sh pytest smoke bench1m || exit $?
timeout -k 10 300 python bench.py --n-p 8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/np8.out 2> gpurun_out/np8.err || exit $?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/np8.out
bash tools/gpu_r2.sh bench100k bench100k_lpm benchsbm
