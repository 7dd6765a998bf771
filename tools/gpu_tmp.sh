#!/bin/bash
set -u
export TMPDIR=/tmp
NPS="8 16" bash tools/exp_np.sh
cp gpurun_out/np/np8.json gpurun_out/np8.json
