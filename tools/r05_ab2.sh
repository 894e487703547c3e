#!/bin/bash
# A/B sweeps in one call: B=1024 wide variants, then B=256 wide; B=1024 level traces (default, wide=64).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
RLE_TRACE=1 RLE_TRACE_BATCH=1024 timeout -k 10 300 python tools/trace_levels.py 20 0,1 > gpurun_out/r05_trace_b1024.txt 2>&1 || exit 1
RLE_PLAN=wide=64 RLE_TRACE=1 RLE_TRACE_BATCH=1024 timeout -k 10 300 python tools/trace_levels.py 20 0,1 > gpurun_out/r05_trace_b1024_wide.txt 2>&1 || exit 1
bash tools/r05_ab.sh b1024 1024 600 - wide=64 wide=32 "wide=64,lpt=1" || exit 1
bash tools/r05_ab.sh b256 256 2000 - wide=64 lpt=1 || exit 1
