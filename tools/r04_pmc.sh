#!/bin/bash
# Same-source PMC for the bench lines' traffic: LFR-1M (louvain) and SBM-4M (lpm)
set -u
./tools/pmc_bench.sh lfr1m r04 && ./tools/pmc_bench.sh sbm4m r04
