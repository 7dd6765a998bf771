set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -q -x tests/test_gpu_parity.py -k "twin or heavy or full_run" > gpurun_out/t_ro.log 2>&1; rc=$?; tail -1 gpurun_out/t_ro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/cd_ab.py --reps 3 old base old base > gpurun_out/ab_ro.out 2>&1; rc=$?
cat gpurun_out/ab_ro.out; exit $rc
