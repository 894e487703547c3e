#!/bin/bash
# Pre-layer (has_pre 3): address audit first (host-side, before any launch), then the TD3 parity
# tests, the whole GPU suite, the TD3 A/B against RLE_NO_PRELAYER=1 and the level structure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "audit or hazard or prelayer or td3" > gpurun_out/p33_td3_tests.txt 2>&1 || { tail -60 gpurun_out/p33_td3_tests.txt; exit 1; }
tail -3 gpurun_out/p33_td3_tests.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/p33_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/p33_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/p33_gpu_tests.txt
RLE_DESC_CRIT=1 RLE_DESC_WG=1 timeout -k 10 120 python tools/describe.py td3 > gpurun_out/crit_td3_pl.txt 2>&1 || exit 1
BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_p33_td3 bash tools/abenv.sh 3 2000 - RLE_NO_PRELAYER=1 || exit 1
