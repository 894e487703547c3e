#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
for K in 3 2; do
  for CAP in 512 640 768; do
    RLE_LEVEL_CAP=$CAP timeout -k 10 200 python bench.py --steps 1000 --warmup 50 --seeds-per-gpu $K --no-cpu-baseline \
      > gpurun_out/p40_ms_${K}_${CAP}.json 2>/dev/null || exit 1
    echo "TD7 K=$K cap=$CAP $(python -c "import json,sys; print(json.load(open(sys.argv[1]))['value'])" gpurun_out/p40_ms_${K}_${CAP}.json)" | tee -a gpurun_out/p40.txt
  done
done
