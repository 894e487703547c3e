#!/bin/bash
# rocprofv3 --kernel-trace over the default bench (no RLE_AQL): the engine falls back to hipGraph replays
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_auto -o run --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline --steps 2000 --warmup 50 > $OUT/prof_auto.json 2> $OUT/prof_auto.log || { tail -5 $OUT/prof_auto.log; exit 1; }
find $OUT/prof_auto -name "*kernel_trace*" -delete
grep rle_level $OUT/prof_auto/run_kernel_stats.csv | cut -c1-120
python3 -c "import json; d=json.load(open('$OUT/prof_auto.json')); print(d['value'], d['engine_timer'])"
