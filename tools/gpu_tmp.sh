set -u
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/clo5 -o clo --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/clo5.log 2>&1 || exit $?
python3 tools/phase_windows.py gpurun_out/clo5/clo_kernel_trace.csv | tail -16
timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -q -x tests/test_gpu_parity.py tests/test_gpu_cd_parity.py -k "closure or full_run or replay" > gpurun_out/clo5_t.log 2>&1; tail -2 gpurun_out/clo5_t.log
