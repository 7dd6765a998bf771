#!/bin/bash
# A/B: FC_OPT_PRUNE_MARK 1 (default) vs 2 (sweep-end marks on the input graph too), LFR-1M and LFR-100k.
set -u
OUT=gpurun_out/pm2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "prune_mark2" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $OUT/pytest.log; exit 1; }
for pm in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --opt prune_mark=$pm > $OUT/lfr1m_pm$pm.json 2> $OUT/lfr1m_pm$pm.err || { echo "bench failed"; tail $OUT/lfr1m_pm$pm.err; exit 1; }
  timeout -k 10 300 python -u bench.py --config lfr100k --steps 5 --warmup 2 --no-cpu-baseline --opt prune_mark=$pm > $OUT/lfr100k_pm$pm.json 2> $OUT/lfr100k_pm$pm.err || { echo "bench failed"; exit 1; }
done
for f in $OUT/*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],2), d['phase_ms_per_step_rank0'])"; done
