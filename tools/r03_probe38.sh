#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
for n in 20 32; do
  for e in "-" "RLE_NO_PRELAYER=1"; do
    [ "$e" = "-" ] && ev="" || ev="$e"
    env $ev DIAG_TAG="n=$n $e" timeout -k 10 120 python tools/diag_packed.py td3_halfcheetah $n 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/p38_diag.txt || exit 1
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/p38_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/p38_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/p38_gpu_tests.txt
BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_p38_td3 bash tools/abenv.sh 2 2000 - RLE_NO_PRELAYER=1 || exit 1
