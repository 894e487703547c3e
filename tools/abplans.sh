#!/bin/bash
# Interleaved A/B of rle_plan variants on one box (the product library): bash tools/abplans.sh <rounds> <steps> <plan>...
# (a plan is bench.py --plan text; "-" = the default plan).  Extra bench args via $BENCH_ARGS.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
OUT=$ROOT/gpurun_out/abplans${AB_TAG}.txt
: > $OUT
R=$1; S=$2; shift 2
for i in $(seq 1 $R); do
  line=""
  for p in "$@"; do
    pp=$p; [ "$p" = "-" ] && pp=""
    v=$(timeout -k 10 120 python bench.py --steps $S --warmup 100 --no-cpu-baseline --plan "$pp" $BENCH_ARGS | python -c "import json,sys; print(json.load(sys.stdin)['value'])") || exit 1
    line="$line  [$p] $v"
  done
  echo "$line" | tee -a $OUT
done
