#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
: > gpurun_out/r03_multiseed_td3_sac.jsonl
for a in "--algo td3 --env HalfCheetah-v4" "--algo sac"; do
  timeout -k 10 300 python bench.py $a --steps 2000 --warmup 50 --seeds-per-gpu 3 --no-cpu-baseline >> gpurun_out/r03_multiseed_td3_sac.jsonl 2>/dev/null || exit 1
done
python -c "import json; [print(json.loads(l)['value']) for l in open('gpurun_out/r03_multiseed_td3_sac.jsonl')]"
