#!/bin/bash
# Re-entry check of the rebuilt tree (GPU suite + bench), then seeds per GPU on streams with the
# tile planner's level capacity lowered (RLE_LEVEL_CAP) so K seeds' levels can co-reside.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/p30_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/p30_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/p30_gpu_tests.txt
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > gpurun_out/p30_bench.json 2> gpurun_out/p30_bench.err || exit 1
cat gpurun_out/p30_bench.json
for K in 2 3 4; do
  for CAP in def 512 384 256; do
    if [ $CAP = def ]; then E=""; else E="RLE_LEVEL_CAP=$CAP"; fi
    env $E timeout -k 10 200 python bench.py --steps 1000 --warmup 50 --seeds-per-gpu $K --no-cpu-baseline \
      > gpurun_out/p30_ms_${K}_${CAP}.json 2>/dev/null || exit 1
    echo "K=$K cap=$CAP $(python -c "import json,sys; print(json.load(open(sys.argv[1]))['value'])" gpurun_out/p30_ms_${K}_${CAP}.json)"
  done
done
