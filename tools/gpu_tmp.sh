set -u
mkdir -p gpurun_out
bash tools/pmc_cd.sh r02b_louv fastconsensus_amd/lib/libfastconsensus_amd.so lfr1m 0 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/stats2_lfr1m -o stats --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/stats2_lfr1m.log 2>&1 || exit $?
grep '"metric"' gpurun_out/stats2_lfr1m.log | head -c 300
