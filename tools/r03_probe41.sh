#!/bin/bash
# SAC: the gradient through the actor's raw head recomputed in-tile by the next input-gradient GEMM
# (pre-layer, GEMM_DX): SAC parity first (audit / hazard / goldens), the whole suite, then A/B.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "sac" > gpurun_out/p41_sac_tests.txt 2>&1 || { tail -60 gpurun_out/p41_sac_tests.txt; exit 1; }
tail -2 gpurun_out/p41_sac_tests.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/p41_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/p41_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/p41_gpu_tests.txt
BENCH_ARGS="--algo sac" AB_TAG=_p41_sac bash tools/abenv.sh 3 2000 - RLE_NO_PRELAYER=1 || exit 1
