#!/bin/bash
# Round 5: seeds per GPU with rle_step_async on direct AQL dispatch (each engine its own queue, bursts
# queued back to back) against hipGraph replays on HIP streams (RLE_AQL=0), by per-seed level capacity.
# usage: tools/r05_seeds_aql.sh [full]   (full: the whole -m gpu suite first)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT && mkdir -p gpurun_out
OUT=gpurun_out/r05_seeds_aql.txt
if [ "$1" = full ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r05_gpu_tests_mid.log 2>&1 || { tail -40 gpurun_out/r05_gpu_tests_mid.log; exit 1; }
  tail -3 gpurun_out/r05_gpu_tests_mid.log
else
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_parity_gpu.py tests/test_engine_gpu.py -k "async" > gpurun_out/r05_seeds_aql_tests.log 2>&1 || { tail -30 gpurun_out/r05_seeds_aql_tests.log; exit 1; }
  tail -3 gpurun_out/r05_seeds_aql_tests.log
fi
: > $OUT
for k in 1 3 4 6; do
  for cap in 0 512; do
    for aql in 1 0; do
      [ $k = 1 ] && [ $cap != 0 ] && continue
      plan=""; [ $cap != 0 ] && plan="--plan level_cap=$cap"
      line=$(RLE_AQL=$aql timeout -k 10 200 python bench.py --steps 1500 --warmup 100 --no-cpu-baseline --seeds-per-gpu $k $plan 2>/dev/null | tail -1) || exit 1
      v=$(echo "$line" | python -c "import json,sys; print(json.load(sys.stdin)['value'])")
      echo "seeds $k cap $cap aql $aql value $v" | tee -a $OUT
    done
  done
done
