set -u
# storage-order experiment: planted-community-contiguous ids with the engine's random
# renumbering off, against the default (random internal numbering, chunked order)
mkdir -p gpurun_out/exp1
run() {  # run <tag> <bench args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/exp1/$tag.json 2> gpurun_out/exp1/$tag.err || exit $?
  echo "$tag: $(python -c "import json;d=json.load(open('gpurun_out/exp1/$tag.json'));print(round(d['ms_per_step'],1),'ms', d['config']['iterations'], {k:round(v,1) for k,v in d['phase_ms_per_step_rank0'].items()})")"
}
run default
run planted_rl0_ch0 --ids planted --relabel 0 --chunk 0
run planted_rl0_ch16 --ids planted --relabel 0 --chunk 16
run gen_rl0_ch0 --relabel 0 --chunk 0
