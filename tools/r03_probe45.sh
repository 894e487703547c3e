#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/p45_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/p45_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/p45_gpu_tests.txt
BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_p45_td3 bash tools/abenv.sh 2 2000 - RLE_LEVEL_CAP=1024 || exit 1
timeout -k 10 300 python bench.py --algo td3 --env HalfCheetah-v4 --steps 2000 --warmup 50 > gpurun_out/p45_td3.json 2> gpurun_out/p45_td3.err || exit 1
