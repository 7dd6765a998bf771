set -u
mkdir -p gpurun_out/micro2
timeout -k 10 120 tools/micro/gather > gpurun_out/micro2/gather.txt 2>&1 || exit $?
cat gpurun_out/micro2/gather.txt
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/micro2/write -o write --output-format csv -- tools/micro/gather > gpurun_out/micro2/write.log 2>&1 || exit $?
FC_TRACE=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/trace_bench.out 2> gpurun_out/trace_bench.err || exit $?
grep "cd it" gpurun_out/trace_bench.err | head -80
