#!/bin/bash
# Headline bench under several engine environments, interleaved (GPU box):
#   bash tools/abenv.sh <rounds> <steps> "ENV=1 ENV2=0" "ENV=0" ...   ("-" = no extra environment)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
R=$1; N=$2; shift 2
for i in $(seq 1 $R); do
  line=""
  for e in "$@"; do
    [ "$e" = "-" ] && ev="" || ev="$e"
    x=$(env $ev timeout -k 10 120 python bench.py --steps $N --warmup 100 --no-cpu-baseline $BENCH_ARGS | python -c "import json,sys; d=json.load(sys.stdin); print(round(d['value'],1), round(d['roofline']['launches_per_step'],2))") || exit 1
    line="$line | $e: $x"
  done
  echo "$line" | tee -a $ROOT/gpurun_out/abenv${AB_TAG}.txt
done
