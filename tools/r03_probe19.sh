#!/bin/bash
# Round-3 probe 19: activation / gradient tile stores as streaming stores (A/B, 3 agents).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
L=sac-td3-td7_amd/lib
AB_TAG=_actnt_td7 bash tools/ablib.sh $L/librle.so $L/librle_actnt.so 3 3000 || exit 1
AB_TAG=_actnt_sac BENCH_ARGS="--algo sac" bash tools/ablib.sh $L/librle.so $L/librle_actnt.so 2 3000 || exit 1
AB_TAG=_actnt_td3 BENCH_ARGS="--algo td3 --env HalfCheetah-v4" bash tools/ablib.sh $L/librle.so $L/librle_actnt.so 2 4000 || exit 1
