#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_p44_td3 bash tools/abenv.sh 2 2000 - RLE_LEVEL_CAP=768 RLE_LEVEL_CAP=640 RLE_LEVEL_CAP=832 || exit 1
BENCH_ARGS="--algo sac" AB_TAG=_p44_sac bash tools/abenv.sh 2 2000 - RLE_LEVEL_CAP=768 RLE_LEVEL_CAP=896 || exit 1
