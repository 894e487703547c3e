#!/bin/bash
# Pre-layer consumers at 64-wide tiles: TD3 tests, A/B over the consumer tile width, level traces.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
true && \
true

BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_p34_td3 bash tools/abenv.sh 2 2000 - RLE_PL_TN=32 RLE_PL_TN=16 RLE_NO_PRELAYER=1 || exit 1
RLE_TRACE_ALGO=td3 timeout -k 10 120 python tools/trace_levels.py > gpurun_out/p34_trace_td3.txt 2>&1 || exit 1
RLE_NO_PRELAYER=1 RLE_TRACE_ALGO=td3 timeout -k 10 120 python tools/trace_levels.py > gpurun_out/p34_trace_td3_nopl.txt 2>&1 || exit 1
