set -u
mkdir -p gpurun_out
timeout -k 10 600 python tools/cd_ab.py --reps 2 base base@FC_TRACK_DIV=1 base@FC_TRACK_DIV=1,FC_PUSH_DIV=1 > gpurun_out/ab_trk.out 2>&1; rc=$?
cat gpurun_out/ab_trk.out; exit $rc
