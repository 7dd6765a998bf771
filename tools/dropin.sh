#!/bin/bash
# The drop-in host path (fast_consensus(G) on a networkx graph) at C3 and C4 sizes.
# Usage: tools/dropin.sh <tag>   -> gpurun_out/<tag>dropin/c3.json, c4.json
set -u
OUT=gpurun_out/${1}dropin
mkdir -p $OUT
timeout -k 10 400 python3 tools/dropin_bench.py 100000 64 > $OUT/c3.json 2> $OUT/c3.err || { tail -5 $OUT/c3.err; exit 1; }
timeout -k 10 900 python3 tools/dropin_bench.py 1000000 64 > $OUT/c4.json 2> $OUT/c4.err || { tail -5 $OUT/c4.err; exit 1; }
cat $OUT/c3.json $OUT/c4.json
