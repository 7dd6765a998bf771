#!/bin/bash
# Closure records / table slots: closure + full-run parity tests, then bench phases base vs prev (HEAD)
set -u
OUT=gpurun_out/r04clo
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cd_parity.py tests/test_gpu_parity.py \
    -k "closure or full_run or c5 or block" -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in base prev base prev; do
  lib=fastconsensus_amd/lib/libfastconsensus_amd.so; [ $v = prev ] && lib=fastconsensus_amd/lib/prev/libfastconsensus_amd.so
  for cfg in "--n-p 8" "--config sbm4m --steps 2 --warmup 1"; do
    FC_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py $cfg --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { echo "bench $v failed"; tail -5 $OUT/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$v', '$cfg', round(d['ms_per_step'],2), {k: round(v,2) for k, v in d['phase_ms_per_step_rank0'].items() if v})"
  done
done
