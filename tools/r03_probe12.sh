#!/bin/bash
# Round-3 probe 12: full GPU suite on the current tree, then the three agents' bench lines.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r03_gpu_suite.txt 2>&1 || { tail -60 gpurun_out/r03_gpu_suite.txt; exit 1; }
tail -2 gpurun_out/r03_gpu_suite.txt
for a in "" "--algo sac" "--algo td3 --env HalfCheetah-v4"; do
  timeout -k 10 200 python bench.py $a --steps 3000 --warmup 60 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print(d['metric'][:60], d['value'], d['roofline']['launches_per_step'])" || exit 1
done
for a in td3 sac; do
  RLE_TRACE=1 RLE_TRACE_ALGO=$a timeout -k 10 200 python tools/trace_levels.py 32 0,3 > gpurun_out/r03_trace_$a.txt 2>&1 || exit 1
done
