#!/bin/bash
# Round-3 probe 14: fused heads with the DX operand ring issued before the head (A/B, 3 agents).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
L=sac-td3-td7_amd/lib
AB_TAG=_hdxe_td7 bash tools/ablib.sh $L/librle.so $L/librle_hdxearly.so 3 3000 || exit 1
BENCH_ARGS="--algo sac" AB_TAG=_hdxe_sac bash tools/ablib.sh $L/librle.so $L/librle_hdxearly.so 2 3000 || exit 1
BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_hdxe_td3 bash tools/ablib.sh $L/librle.so $L/librle_hdxearly.so 2 4000 || exit 1
