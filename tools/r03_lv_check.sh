set -u
mkdir -p gpurun_out/lv1
timeout -k 10 400 python3 bench.py --config lfr1m_leiden --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/lv1/leiden.json 2> gpurun_out/lv1/leiden.err || exit 1
timeout -k 10 400 python3 bench.py --config lfr100k_infomap --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/lv1/info.json 2> gpurun_out/lv1/info.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_leiden.py tests/test_infomap.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lv1/tests.log 2>&1 || exit 1
