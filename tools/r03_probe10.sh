#!/bin/bash
# Round-3 probe 10: SAC rsample / backward fused into the actor GEMM epilogues (parity, A/B).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_parity_gpu.py tests/test_mirror_gpu.py -k "sac or hazard or audit or packed" -x -v \
  --timeout 200 --timeout-method thread > gpurun_out/r03_sac_fuse_tests.txt 2>&1 || { tail -60 gpurun_out/r03_sac_fuse_tests.txt; exit 1; }
tail -3 gpurun_out/r03_sac_fuse_tests.txt
BENCH_ARGS="--algo sac" AB_TAG=_sacfuse bash tools/abenv.sh 2 3000 - RLE_NO_SACFWD=1 RLE_NO_SACBWD=1 "RLE_NO_SACFWD=1 RLE_NO_SACBWD=1" || exit 1
AB_TAG=_td7chk bash tools/abenv.sh 1 3000 - || exit 1
RLE_DESC_WG=1 timeout -k 10 120 python tools/describe.py sac > gpurun_out/describe_sac2.txt 2>&1 || exit 1
