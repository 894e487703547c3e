#!/bin/bash
# Secondary BASELINE configs and several seeds per GPU (GPU box), each bench line with its
# CPU oracle baseline:  bash tools/secondary.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
: > $OUT/secondary.jsonl
for args in "--env Ant-v4" "--algo sac" "--algo td3 --env HalfCheetah-v4" "--batch 1024"; do
  timeout -k 10 300 python bench.py --steps 2000 --warmup 50 $args >> $OUT/secondary.jsonl 2> $OUT/secondary.err || { echo "FAILED: $args"; tail -5 $OUT/secondary.err; exit 1; }
  echo "done $args"
done
: > $OUT/multiseed.jsonl
for k in 2 3 4; do
  timeout -k 10 300 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline --seeds-per-gpu $k >> $OUT/multiseed.jsonl 2> $OUT/multiseed.err || { echo "FAILED: seeds $k"; tail -5 $OUT/multiseed.err; exit 1; }
  echo "done seeds $k"
done
