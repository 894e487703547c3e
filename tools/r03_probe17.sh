#!/bin/bash
# Round-3 probe 17: wave-parallel step-end sums: bitwise against the previous kernels (64K
# trajectory; TD3 trajectory through the GPU tests), then A/B on the three agents.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
L=sac-td3-td7_amd/lib
bash tools/determinism.sh end $L/librle_prev.so $L/librle.so 8 > /dev/null 2>&1 || { echo DET FAILED; exit 1; }
tail -4 gpurun_out/end_bitcmp.txt
AB_TAG=_end2_td3 BENCH_ARGS="--algo td3 --env HalfCheetah-v4" bash tools/ablib.sh $L/librle_prev.so $L/librle.so 3 4000 || exit 1
AB_TAG=_end2_td7 bash tools/ablib.sh $L/librle_prev.so $L/librle.so 3 3000 || exit 1
AB_TAG=_end2_sac BENCH_ARGS="--algo sac" bash tools/ablib.sh $L/librle_prev.so $L/librle.so 2 3000 || exit 1
