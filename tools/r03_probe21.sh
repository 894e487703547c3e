#!/bin/bash
# Round-3 probe 21: the forward pre-GEMM's one-segment fast path (A/B TD7 / TD3, fine trace).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
L=sac-td3-td7_amd/lib
AB_TAG=_oneseg_td7 bash tools/ablib.sh $L/librle.so $L/librle_oneseg.so 3 3000 || exit 1
AB_TAG=_oneseg_td3 BENCH_ARGS="--algo td3 --env HalfCheetah-v4" bash tools/ablib.sh $L/librle.so $L/librle_oneseg.so 2 4000 || exit 1
RLE_LIB=$ROOT/$L/librle_onesegfine.so RLE_TRACE=1 RLE_TRACE_OPS=1 timeout -k 10 200 python tools/trace_levels.py 32 3 > gpurun_out/r03_fine_td7_oneseg.txt 2>&1 || exit 1
