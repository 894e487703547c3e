#!/bin/bash
# Round 5: seeds per GPU on direct AQL queues against the HIP runtime's own hardware queues
# (GPU_MAX_HW_QUEUES), to find where the device's queue slots run out.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT && mkdir -p gpurun_out
OUT=gpurun_out/r05_hwq.txt
: > $OUT
for q in 1 2; do
  for k in 4 5 6 8; do
    line=$(GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 1500 --warmup 100 --no-cpu-baseline --seeds-per-gpu $k 2>/dev/null | tail -1) || exit 1
    echo "hwq $q seeds $k $(echo "$line" | python -c "import json,sys; print(json.load(sys.stdin)['value'])")" | tee -a $OUT
  done
done
