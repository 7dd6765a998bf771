#!/bin/bash
# k_mark_lm (wave-cooperative row walks): twin/full-run parity, then the LFR-1M bench and its kernel stats.
set -u
mkdir -p gpurun_out/mk
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "twin or full_run or prune_mark" > gpurun_out/mk/pytest.log 2>&1 || { tail -30 gpurun_out/mk/pytest.log; exit 1; }
tail -2 gpurun_out/mk/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mk/rp -o lfr1m --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/mk/bench.json 2> gpurun_out/mk/bench.err || { tail gpurun_out/mk/bench.err; exit 1; }
cp $(find gpurun_out/mk/rp -name "*kernel_stats.csv" | head -1) gpurun_out/mk/kernel_stats.csv
rm -rf gpurun_out/mk/rp
grep -i "mark_lm\|k_decide_light<true, int>\|k_apply<true, int>" gpurun_out/mk/kernel_stats.csv | cut -c1-160
python3 -c "import json; d=json.load(open('gpurun_out/mk/bench.json')); print(round(d['ms_per_step'],2), d['config']['m_final'])"
