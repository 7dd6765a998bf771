#!/bin/bash
# Round-3 verification A: the GPU tests and smoke, then PMC passes (tools/pmc_cd.sh) at HEAD for the
# bench configs whose traffic the bench lines attach.  Stops at the first failure.
set -u
mkdir -p gpurun_out/fa
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/fa/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/fa/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 900 tools/pmc_cd.sh r03_lfr1m fastconsensus_amd/lib/libfastconsensus_amd.so lfr1m 0 > gpurun_out/fa/pmc_lfr1m.log 2>&1 || { echo "pmc lfr1m failed"; exit 1; }
echo done
