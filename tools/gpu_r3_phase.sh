set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/cd_ab.py --reps 2 base phase > gpurun_out/ab_phase.out 2> gpurun_out/ab_phase.err; rc=$?
echo "ab rc=$rc"; cat gpurun_out/ab_phase.out; grep "phase cycles" gpurun_out/ab_phase.err | tail -3
[ $rc -eq 0 ] || exit $rc
bash tools/pmc_cd.sh base
