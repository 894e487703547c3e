#!/bin/bash
# Headline bench under several step-program plans, interleaved (GPU box):
#   bash tools/abplan.sh <rounds> <steps> "rb=1" "rb=2,level_cap=512" "-" ...   ("-" = default plan)
# BENCH_ARGS: extra bench.py arguments (e.g. "--batch 1024").
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
R=$1; N=$2; shift 2
for i in $(seq 1 $R); do
  line=""
  for e in "$@"; do
    [ "$e" = "-" ] && pl="" || pl="$e"
    x=$(timeout -k 10 120 python bench.py --steps $N --warmup 100 --no-cpu-baseline --plan "$pl" $BENCH_ARGS | python -c "import json,sys; d=json.load(sys.stdin); print(round(d['value'],1), round(d['roofline']['launches_per_step'],2))") || exit 1
    line="$line | $e: $x"
  done
  echo "$line" | tee -a $ROOT/gpurun_out/abplan${AB_TAG}.txt
done
