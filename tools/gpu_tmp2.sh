set -u
mkdir -p gpurun_out
for st in 1 0; do
  timeout -k 10 300 python bench.py --n-p 8 --steps 3 --warmup 1 --no-cpu-baseline --store $st > gpurun_out/np8s$st.out 2>/dev/null || exit $?
  echo "np8 store $st: $(grep -o '"ms_per_step": [0-9.]*\|"load_ms_per_step": [0-9.]*' gpurun_out/np8s$st.out | tr '\n' ' ')"
  timeout -k 10 300 python bench.py --n-p 16 --steps 3 --warmup 1 --no-cpu-baseline --store $st > gpurun_out/np16s$st.out 2>/dev/null || exit $?
  echo "np16 store $st: $(grep -o '"ms_per_step": [0-9.]*\|"load_ms_per_step": [0-9.]*' gpurun_out/np16s$st.out | tr '\n' ' ')"
done
