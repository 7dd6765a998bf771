set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/cd_ab.py --child fastconsensus_amd/lib/phase/libfastconsensus_amd.so lfr1m 0 1 > gpurun_out/phase2.out 2> gpurun_out/phase2.err || exit $?
grep "phase cycles" gpurun_out/phase2.err
