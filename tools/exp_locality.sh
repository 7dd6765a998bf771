#!/bin/bash
# storage-order experiment: planted-community-contiguous ids (engine renumbering off, per-vertex
# visit order) with implicit (position-ordered) vs materialised (vertex-ordered) bucket lists
set -u
mkdir -p gpurun_out/exp1
run() {  # run <tag> <env> <bench args...>
  local tag=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/exp1/$tag.json 2> gpurun_out/exp1/$tag.err || exit $?
  echo "$tag: $(python -c "import json;d=json.load(open('gpurun_out/exp1/$tag.json'));print(round(d['ms_per_step'],1),'ms', d['config']['iterations'], {k:round(v,1) for k,v in d['phase_ms_per_step_rank0'].items()})")"
}
run default FC_X=0
run default_fl FC_FULL_LISTS=1
run planted_ch0 FC_X=0 --ids planted --relabel 0 --chunk 0
run planted_ch0_fl FC_FULL_LISTS=1 --ids planted --relabel 0 --chunk 0
run gen_ch0_fl FC_FULL_LISTS=1 --relabel 0 --chunk 0
