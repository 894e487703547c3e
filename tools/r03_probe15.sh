#!/bin/bash
# Round-3 probe 15: the step-end op moved under longer ops by the rebalance pass (A/B against
# RLE_TINY_W=0, 3 agents), level hazards of the new schedules.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -k "hazard or multistep or packed" -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/r03_tiny_tests.txt 2>&1 || { tail -40 gpurun_out/r03_tiny_tests.txt; exit 1; }
tail -2 gpurun_out/r03_tiny_tests.txt
AB_TAG=_tiny_td7 bash tools/abenv.sh 3 3000 - RLE_TINY_W=0 RLE_TINY_W=30 || exit 1
BENCH_ARGS="--algo sac" AB_TAG=_tiny_sac bash tools/abenv.sh 2 3000 - RLE_TINY_W=0 RLE_TINY_W=30 || exit 1
BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_tiny_td3 bash tools/abenv.sh 2 4000 - RLE_TINY_W=0 RLE_TINY_W=30 || exit 1
