#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/p39_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/p39_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/p39_gpu_tests.txt
BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_p39_td3 bash tools/abenv.sh 2 2000 - RLE_NO_PRELAYER=1 || exit 1
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > gpurun_out/p39_bench.json 2> gpurun_out/p39_bench.err || exit 1
cat gpurun_out/p39_bench.json
