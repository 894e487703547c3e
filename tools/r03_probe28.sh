#!/bin/bash
# Round-3 probe 28: step-end lists of a wave all in flight at once (A/B, 3 agents).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
L=sac-td3-td7_amd/lib
AB_TAG=_endb_td3 BENCH_ARGS="--algo td3 --env HalfCheetah-v4" bash tools/ablib.sh $L/librle.so $L/librle_endb.so 2 4000 || exit 1
AB_TAG=_endb_sac BENCH_ARGS="--algo sac" bash tools/ablib.sh $L/librle.so $L/librle_endb.so 2 3000 || exit 1
AB_TAG=_endb_td7 bash tools/ablib.sh $L/librle.so $L/librle_endb.so 2 3000 || exit 1
