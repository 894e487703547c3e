#!/bin/bash
# Round-3 probe 11: step-end sums loaded in one batch (A/B against the previous kernels on all
# three agents), the wide-launch lookup's cost (no-wide timing variant), GPU tests of the step end.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -k "trajectory and (tiny or humanoid)" -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r03_end_tests.txt 2>&1 || { tail -40 gpurun_out/r03_end_tests.txt; exit 1; }
tail -2 gpurun_out/r03_end_tests.txt
L=sac-td3-td7_amd/lib
AB_TAG=_end_td7 bash tools/ablib.sh $L/librle_prev.so $L/librle.so 3 3000 || exit 1
BENCH_ARGS="--algo sac" AB_TAG=_end_sac bash tools/ablib.sh $L/librle_prev.so $L/librle.so 2 3000 || exit 1
BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_end_td3 bash tools/ablib.sh $L/librle_prev.so $L/librle.so 2 4000 || exit 1
AB_TAG=_nowide bash tools/ablib.sh $L/librle.so $L/librle_nowide.so 3 3000 || exit 1
