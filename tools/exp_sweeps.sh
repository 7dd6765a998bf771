set -u
mkdir -p gpurun_out/exp2
FC_TRACE=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/exp2/trace.json 2> gpurun_out/exp2/trace.err || exit $?
for B in 8 16 64; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --buckets $B > gpurun_out/exp2/b$B.json 2> gpurun_out/exp2/b$B.err || exit $?
done
