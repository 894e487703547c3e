#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
  > gpurun_out/p49_gpu_tests.txt 2>&1 || { grep -E "FAIL|Error" gpurun_out/p49_gpu_tests.txt | head; tail -30 gpurun_out/p49_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/p49_gpu_tests.txt
AB_TAG=_p49_td7 bash tools/abenv.sh 2 2000 - RLE_PRE_TN=16 || exit 1
BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_p49_td3 bash tools/abenv.sh 2 2000 - RLE_PRE_TN=16 || exit 1
