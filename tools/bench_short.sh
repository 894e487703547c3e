#!/bin/bash
# The driver's round-end bench command (20 timed steps after 5 warmup steps) and longer lines, with the
# host-thread share of the timed region: bash tools/bench_short.sh [repeats]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
for i in $(seq 1 ${1:-3}); do
  for a in "--steps 20 --warmup 5" "--steps 200 --warmup 20" "--steps 2000 --warmup 50"; do
    timeout -k 10 120 python3 bench.py --gpus 1 $a --no-cpu-baseline 2>/dev/null | python3 -c "
import json,sys; d=json.load(sys.stdin); print('$a', d['value'], d['ms_per_step'], 'host busy', d['host_thread_busy_frac'])" || exit 1
  done
done
