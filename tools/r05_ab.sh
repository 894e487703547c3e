#!/bin/bash
# A/B of plan variants on one box: bash tools/r05_ab.sh <tag> <batch> <steps> "<plan1>" "<plan2>" ...
# (plan "-": the default plan); one JSON summary line per run into gpurun_out/r05_ab_<tag>.txt
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT && mkdir -p gpurun_out
TAG=$1; BATCH=$2; STEPS=$3; shift 3
OUT=gpurun_out/r05_ab_${TAG}.txt
: > $OUT
for rnd in 1 2; do
  for p in "$@"; do
    PL=$p; [ "$p" = "-" ] && PL=""
    timeout -k 10 300 python bench.py --batch $BATCH --steps $STEPS --warmup 20 --no-cpu-baseline --plan "$PL" > /tmp/ab.json 2>/tmp/ab.err || { echo "FAILED $p"; tail -5 /tmp/ab.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1])
print('round $rnd plan [$p]', d['value'], d['roofline']['launches_per_step'], d['roofline']['avg_launch_us'])" >> $OUT
  done
done
cat $OUT
