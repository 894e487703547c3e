#!/bin/bash
# Round-3 probe 24: the step end split into a counters op and an info op (tests, A/B).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_parity_gpu.py tests/test_mirror_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/r03_split_tests.txt 2>&1 || { tail -50 gpurun_out/r03_split_tests.txt; exit 1; }
tail -2 gpurun_out/r03_split_tests.txt
AB_TAG=_split_sac BENCH_ARGS="--algo sac" bash tools/abenv.sh 2 3000 - RLE_END_SPLIT=0 || exit 1
AB_TAG=_split_td3 BENCH_ARGS="--algo td3 --env HalfCheetah-v4" bash tools/abenv.sh 2 4000 - RLE_END_SPLIT=0 || exit 1
AB_TAG=_split_td7 bash tools/abenv.sh 3 3000 - RLE_END_SPLIT=0 || exit 1
