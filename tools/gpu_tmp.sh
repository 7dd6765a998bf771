set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -q -s -x tests/test_gpu_parity.py -k "many_isolates or replay or full_run" > gpurun_out/t_iso.log 2>&1; rc=$?; grep -E "N [0-9]+:|passed|failed" gpurun_out/t_iso.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/n1c -o n1 --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/n1c.log 2>&1 || exit $?
python3 tools/step_gaps.py gpurun_out/n1c/n1_kernel_trace.csv > gpurun_out/n1c_gaps.txt 2>&1; head -30 gpurun_out/n1c_gaps.txt
