#!/bin/bash
# Round-3 probe 26: planner discount for elementwise ops (default 4) + the small-op move rule
# extended to the uniform sampler (tests, A/B against RLE_TINY_WG=2 / RLE_UNI_W=60).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_parity_gpu.py tests/test_mirror_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/r03_p26_tests.txt 2>&1 || { tail -50 gpurun_out/r03_p26_tests.txt; exit 1; }
tail -2 gpurun_out/r03_p26_tests.txt
AB_TAG=_uni_sac BENCH_ARGS="--algo sac" bash tools/abenv.sh 2 3000 - RLE_TINY_WG=2 RLE_UNI_W=60 || exit 1
AB_TAG=_uni_td3 BENCH_ARGS="--algo td3 --env HalfCheetah-v4" bash tools/abenv.sh 2 4000 - RLE_TINY_WG=2 RLE_UNI_W=60 || exit 1
AB_TAG=_uni_td7 bash tools/abenv.sh 2 3000 - RLE_TINY_WG=2 || exit 1
