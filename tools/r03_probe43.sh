#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
AB_TAG=_p43_td7 bash tools/abenv.sh 2 2000 - RLE_LEVEL_CAP=960 RLE_LEVEL_CAP=896 RLE_LEVEL_CAP=768 || exit 1
BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_p43_td3 bash tools/abenv.sh 2 2000 - RLE_LEVEL_CAP=768 RLE_LEVEL_CAP=512 || exit 1
