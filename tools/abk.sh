#!/bin/bash
# Headline bench under several values of one engine environment variable (GPU box):
#   bash tools/abk.sh VAR "v1 v2 ..." [rounds] [steps]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
OUT=$ROOT/gpurun_out/abk${AB_TAG}.txt
: > $OUT
for i in $(seq 1 ${3:-2}); do
  line=""
  for v in $2; do
    x=$(env $1=$v timeout -k 10 120 python bench.py --steps ${4:-4000} --warmup 100 --no-cpu-baseline $BENCH_ARGS | python -c "import json,sys; print(json.load(sys.stdin)['value'])") || exit 1
    line="$line $1=$v:$x"
  done
  echo "$line" | tee -a $OUT
done
