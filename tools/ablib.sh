#!/bin/bash
# A/B of two engine libraries on the headline bench (GPU box), alternating runs:
#   bash tools/ablib.sh <libA.so> <libB.so> [rounds] [steps]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
OUT=$ROOT/gpurun_out/ablib${AB_TAG}.txt
: > $OUT
for i in $(seq 1 ${3:-3}); do
  a=$(RLE_LIB=$ROOT/$1 timeout -k 10 120 python bench.py --steps ${4:-4000} --warmup 100 --no-cpu-baseline $BENCH_ARGS | python -c "import json,sys; print(json.load(sys.stdin)['value'])") || exit 1
  b=$(RLE_LIB=$ROOT/$2 timeout -k 10 120 python bench.py --steps ${4:-4000} --warmup 100 --no-cpu-baseline $BENCH_ARGS | python -c "import json,sys; print(json.load(sys.stdin)['value'])") || exit 1
  echo "$(basename $1) $a  $(basename $2) $b" | tee -a $OUT
done
