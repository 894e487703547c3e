#!/bin/bash
# Round-3 probe 20: activation stores as streaming stores; Adam operands loaded after the main
# loop, alone and with a 6-deep weight-gradient ring (A/B against the default build).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
L=sac-td3-td7_amd/lib
for v in actnt late dw6late; do
  AB_TAG=_${v}_td7 bash tools/ablib.sh $L/librle.so $L/librle_$v.so 2 3000 || exit 1
done
for v in actnt dw6late; do
  AB_TAG=_${v}_sac BENCH_ARGS="--algo sac" bash tools/ablib.sh $L/librle.so $L/librle_$v.so 2 3000 || exit 1
  AB_TAG=_${v}_td3 BENCH_ARGS="--algo td3 --env HalfCheetah-v4" bash tools/ablib.sh $L/librle.so $L/librle_$v.so 2 4000 || exit 1
done
