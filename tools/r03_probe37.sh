#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
for n in 4 8 12 20 32; do
  for e in "-" "RLE_NO_PRELAYER=1"; do
    [ "$e" = "-" ] && ev="" || ev="$e"
    env $ev DIAG_TAG="n=$n $e" timeout -k 10 120 python tools/diag_packed.py td3_halfcheetah $n 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/p37_diag.txt || exit 1
  done
done
BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_p37_td3 bash tools/abenv.sh 2 2000 - RLE_NO_PRELAYER=1 || exit 1
