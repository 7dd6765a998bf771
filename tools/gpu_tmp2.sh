set -u
mkdir -p gpurun_out
for tv in 16384 4096 65536 0; do
  FC_TAIL_VISITS=$tv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/tv$tv.out 2>/dev/null || exit $?
  FC_TAIL_VISITS=$tv timeout -k 10 300 python bench.py --n-p 8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/tv8_$tv.out 2>/dev/null || exit $?
  echo "tail_visits $tv: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tv$tv.out) | np8 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tv8_$tv.out)"
done
