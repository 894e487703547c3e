#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
AB_TAG=_p48_td7 bash tools/abenv.sh 2 2000 - RLE_PRE_TN=32 RLE_PRE_TN=64 || exit 1
BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_p48_td3 bash tools/abenv.sh 2 2000 - RLE_PRE_TN=32 RLE_PRE_TN=64 || exit 1
