#!/bin/bash
# A/B of an engine environment toggle on the headline bench (GPU box):
#   bash tools/ab.sh VAR=VALUE [rounds] [steps]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
OUT=$ROOT/gpurun_out/ab${AB_TAG}.txt
: > $OUT
for i in $(seq 1 ${2:-3}); do
  a=$(timeout -k 10 120 python bench.py --steps ${3:-4000} --warmup 100 --no-cpu-baseline $BENCH_ARGS | python -c "import json,sys; print(json.load(sys.stdin)['value'])") || exit 1
  b=$(env $1 timeout -k 10 120 python bench.py --steps ${3:-4000} --warmup 100 --no-cpu-baseline $BENCH_ARGS | python -c "import json,sys; print(json.load(sys.stdin)['value'])") || exit 1
  echo "default $a  $1 $b" | tee -a $OUT
done
