#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
for e in "-" "RLE_PL_TN=16" "RLE_NO_PRELAYER=1"; do
  [ "$e" = "-" ] && ev="" || ev="$e"
  env $ev DIAG_TAG="$e" timeout -k 10 120 python tools/diag_packed.py td3_halfcheetah 20 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/p35_diag.txt || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -q --timeout 120 --timeout-method thread \
  -k "multistep or prelayer or td3 or sac" > gpurun_out/p35_tests.txt 2>&1; tail -5 gpurun_out/p35_tests.txt
