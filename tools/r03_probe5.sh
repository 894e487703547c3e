#!/bin/bash
# Round-3 probe 5: packed vs per-stream multi-seed across the three agents, and the tile
# planner's capacity for packed TD7 programs.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
OUT=gpurun_out/r03_multiseed2.jsonl
run() {
  timeout -k 10 240 "$@" --steps 2000 --warmup 60 --no-cpu-baseline >> $OUT 2> gpurun_out/r03_ms2_err.txt || { tail -30 gpurun_out/r03_ms2_err.txt; exit 1; }
  tail -1 $OUT | python -c "import json,sys; d=json.load(sys.stdin); print(d['metric'][:70], d['value'], d['config'].get('packed'))"
}
for a in "--algo td3 --env HalfCheetah-v4" "--algo sac --env Humanoid-v4"; do
  run python bench.py $a --seeds-per-gpu 3
  run python bench.py $a --seeds-per-gpu 3 --packed
  run python bench.py $a --seeds-per-gpu 2 --packed
  run python bench.py $a
done
RLE_LEVEL_CAP=2048 run python bench.py --seeds-per-gpu 3 --packed
RLE_LEVEL_CAP=4096 run python bench.py --seeds-per-gpu 3 --packed
