set -u
mkdir -p gpurun_out/exp3
for cfg in "0 0" "1 0" "1 16"; do set -- $cfg
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --prune $1 --chunk $2 > gpurun_out/exp3/p$1_c$2.json 2> gpurun_out/exp3/p$1_c$2.err || exit $?
done
