#!/bin/bash
# Round-6 probe 2: write-through Adam stores (m, v, T image: sc1 instead of nt), A/B against the product library;
# and the same with no release fence between levels (timing only).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
L=sac-td3-td7_amd/lib
AB_TAG=_adamwt bash tools/ablib.sh $L/librle.so $L/librle_adamwt.so 3 2000 || exit 1
AB_TAG=_adamwt_rel0 bash tools/ablib.sh $L/librle_rel0.so $L/librle_adamwt_rel0.so 2 2000 || exit 1
AB_TAG=_adamwt_b1024 BENCH_ARGS="--batch 1024" bash tools/ablib.sh $L/librle.so $L/librle_adamwt.so 2 1000 || exit 1
