set -u
mkdir -p gpurun_out/exp4
for cfg in lfr100k lfr100k_lpm sbm4m; do
  FC_TRACE=${TRACE:-} timeout -k 10 600 python bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/exp4/$cfg.json 2> gpurun_out/exp4/$cfg.err || exit $?
  echo "$cfg done"
done
