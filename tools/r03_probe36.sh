#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -q --timeout 120 --timeout-method thread \
  -k "audit or prelayer or td3_halfcheetah" > gpurun_out/p36_tests.txt 2>&1; tail -3 gpurun_out/p36_tests.txt
for e in "RLE_LEVEL_CAP=1000000" "-"; do
  [ "$e" = "-" ] && ev="" || ev="$e"
  env $ev DIAG_TAG="$e" timeout -k 10 120 python tools/diag_packed.py td3_halfcheetah 20 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/p36_diag.txt || exit 1
done
BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_p36_td3 bash tools/abenv.sh 2 2000 - RLE_NO_PRELAYER=1 || exit 1
RLE_TRACE_ALGO=td3 timeout -k 10 120 python tools/trace_levels.py > gpurun_out/p36_trace_td3.txt 2>&1 || exit 1
