#!/bin/bash
# Round-3 probe 25: Polyak / copy workgroups discounted in the tile planner's level capacity.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
AB_TAG=_flat_sac BENCH_ARGS="--algo sac" bash tools/abenv.sh 2 3000 - RLE_FLAT_DIV=4 RLE_FLAT_DIV=1000 || exit 1
AB_TAG=_flat_td3 BENCH_ARGS="--algo td3 --env HalfCheetah-v4" bash tools/abenv.sh 2 4000 - RLE_FLAT_DIV=4 RLE_FLAT_DIV=1000 || exit 1
AB_TAG=_flat_td7 bash tools/abenv.sh 2 3000 - RLE_FLAT_DIV=4 RLE_FLAT_DIV=1000 || exit 1
