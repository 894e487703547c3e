#!/bin/bash
# Round-3 probe 18: SAC rsample noise prefetched before the raw-head GEMM's main loop (tests, A/B).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_parity_gpu.py -k "sac" -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/r03_sacpf_tests.txt 2>&1 || { tail -40 gpurun_out/r03_sacpf_tests.txt; exit 1; }
tail -2 gpurun_out/r03_sacpf_tests.txt
L=sac-td3-td7_amd/lib
AB_TAG=_sacpf BENCH_ARGS="--algo sac" bash tools/ablib.sh $L/librle_prev.so $L/librle.so 3 3000 || exit 1
