#!/bin/bash
# B=1024: level trace with register-blocked weight gradients, A/B rb / level caps.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
RLE_PLAN=rb=1 RLE_TRACE=1 RLE_TRACE_BATCH=1024 timeout -k 10 300 python tools/trace_levels.py 20 0,1 > gpurun_out/r05_trace_b1024_rb.txt 2>&1 || exit 1
bash tools/r05_ab.sh b1024rb 1024 600 - rb=1 "rb=1,level_cap=1024" "level_cap=1024" "rb=1,level_cap=2048" || exit 1
