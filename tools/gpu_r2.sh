#!/bin/bash
# Round-2 GPU-box runner: each GPU step under its own timeout; stop at the first fault/abort/timeout.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
    local name=$1 t=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 30 "gpurun_out/$name.out"; tail -n 15 "gpurun_out/$name.err"
    case $rc in 0|1|2|5) return 0;; *) echo "!! stopping: $name rc=$rc"; exit $rc;; esac
}
PYT="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -rf"
for s in "$@"; do
    case $s in
        newtests) step newtests 1200 $PYT -s -v tests/test_gpu_cd_parity.py ;;
        oldtests) step oldtests 900 $PYT -q tests/test_gpu_parity.py ;;
        pytest) step pytest_gpu 900 $PYT -q -m gpu tests ;;
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        loadprof) step loadprof 300 python tools/load_prof.py ;;
        bench1m) step bench_1m 900 python bench.py --steps 3 --warmup 1 ;;
        bench1m_fast) step bench_1m 900 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
        bench100k) step bench_100k 600 python bench.py --config lfr100k --steps 3 --warmup 1 --no-cpu-baseline ;;
        bench100k_lpm) step bench_100k_lpm 600 python bench.py --config lfr100k_lpm --steps 3 --warmup 1 --no-cpu-baseline ;;
        prof1m) step prof_1m 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_1m -o prof --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
        benchsbm) step bench_sbm 900 python bench.py --config sbm4m --steps 2 --warmup 1 --no-cpu-baseline ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
