#!/bin/bash
# Round-3 probe 8: TD3 / SAC loss and objective heads fused into the critics' DX (parity tests,
# then A/B against RLE_NO_HEADDX=1), and the weights' T image as streaming stores (A/B).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_parity_gpu.py -k "td3 or sac or hazard or audit" -x -v \
  --timeout 200 --timeout-method thread > gpurun_out/r03_mlp_hdx_tests.txt 2>&1 || { tail -60 gpurun_out/r03_mlp_hdx_tests.txt; exit 1; }
tail -3 gpurun_out/r03_mlp_hdx_tests.txt
BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_hdx_td3 bash tools/abenv.sh 2 4000 - RLE_NO_HEADDX=1 || exit 1
BENCH_ARGS="--algo sac" AB_TAG=_hdx_sac bash tools/abenv.sh 2 3000 - RLE_NO_HEADDX=1 || exit 1
AB_TAG=_ntp bash tools/ablib.sh sac-td3-td7_amd/lib/librle.so sac-td3-td7_amd/lib/librle_ntp.so 3 3000 || exit 1
