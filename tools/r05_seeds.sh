#!/bin/bash
# Round 5: host core during an AQL burst (bench line's host_thread_busy_frac), and rocprofv3 kernel traces of
# 1 / 3 / 4 TD7 seeds per GPU (which levels of different seeds overlap: tools/seed_overlap.py).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline > gpurun_out/r05_host_busy.json 2>/dev/null || exit 1
cd /tmp && export TMPDIR=/tmp
for k in 1 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/r05_seeds$k -o run -- python3 $ROOT/bench.py --steps 120 --warmup 20 --no-cpu-baseline --seeds-per-gpu $k > $ROOT/gpurun_out/r05_seeds$k.log 2>&1 || exit 1
done
