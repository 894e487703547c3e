#!/bin/bash
# TD3: the policy Polyak fused into the actor's Adam epilogues (parity, then A/B vs
# RLE_NO_PIPOLYAK=1); seeds per GPU at the 512 level capacity for TD3 / SAC.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/p31_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/p31_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/p31_gpu_tests.txt
BENCH_ARGS="--algo td3 --env HalfCheetah-v4" AB_TAG=_p31_td3 bash tools/abenv.sh 3 2000 - RLE_NO_PIPOLYAK=1 || exit 1
for A in "td3 HalfCheetah-v4" "sac Humanoid-v4"; do
  set -- $A
  for CAP in 1024 512; do
    RLE_LEVEL_CAP=$CAP timeout -k 10 200 python bench.py --algo $1 --env $2 --steps 2000 --warmup 50 --seeds-per-gpu 3 \
      --no-cpu-baseline > gpurun_out/p31_ms_$1_$CAP.json 2>/dev/null || exit 1
    echo "$1 K=3 cap=$CAP $(python -c "import json,sys; print(json.load(open(sys.argv[1]))['value'])" gpurun_out/p31_ms_$1_$CAP.json)"
  done
done
