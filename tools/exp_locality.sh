set -u
mkdir -p gpurun_out/exp1
for ids in ${IDS:-generator planted}; do for ch in 0 16; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --ids $ids --chunk $ch > gpurun_out/exp1/${ids}_${ch}.json 2> gpurun_out/exp1/${ids}_${ch}.err || exit $?
  echo "$ids $ch done"
done; done
