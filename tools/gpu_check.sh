#!/bin/bash
# GPU-box runner: each GPU step under its own timeout; stop at the first fault/abort/timeout.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
    local name=$1 t=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 25 "gpurun_out/$name.out"; tail -n 15 "gpurun_out/$name.err"
    case $rc in 0|1|2|5) return 0;; *) echo "!! stopping: $name rc=$rc"; exit $rc;; esac
}
for s in "$@"; do
    case $s in
        pytest) step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider -rf ;;
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench100k) step bench_100k 600 python bench.py --config lfr100k --steps 2 --warmup 1 --no-cpu-baseline ;;
        bench1m) step bench_1m 900 python bench.py --steps 2 --warmup 1 ;;
        bench1m_fast) step bench_1m 900 python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
