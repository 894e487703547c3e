#!/bin/bash
# 64 x 16 LDS-staged tiles (wide=16): oracle agreement after a B=1024 burst, audit, A/B at B=1024 and B=512.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
RLE_AUDIT=1 timeout -k 10 200 python tools/diag_wide.py td7 Humanoid-v4 256 1024 8 wide=16 > gpurun_out/r05_w16_diag.txt 2>&1 || { tail -20 gpurun_out/r05_w16_diag.txt; exit 1; }
timeout -k 10 200 python tools/diag_wide.py td7 Humanoid-v4 256 1024 8 > gpurun_out/r05_w0_diag.txt 2>&1 || { tail -20 gpurun_out/r05_w0_diag.txt; exit 1; }
RLE_PLAN=wide=16 RLE_TRACE=1 RLE_TRACE_BATCH=1024 timeout -k 10 300 python tools/trace_levels.py 20 0,1 > gpurun_out/r05_trace_b1024_w16.txt 2>&1 || exit 1
bash tools/r05_ab.sh w16 1024 600 - wide=16 "wide=16,level_cap=1024" "wide=16,level_cap=2048" || exit 1
