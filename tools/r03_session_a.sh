set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ph
timeout -k 10 300 python3 tools/cd_ab.py --child fastconsensus_amd/lib/v_phase/libfastconsensus_amd.so lfr1m 0 1 > gpurun_out/ph/phase.log 2>&1 || exit 1
timeout -k 10 900 tools/pmc_cd.sh r03a > gpurun_out/pmc_r03a.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_r03a.json 2> gpurun_out/bench_r03a.err || exit 1
