#!/bin/bash
# GPU tests, then the headline bench three times (GPU box): bash tools/bench3.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $ROOT/gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 $ROOT/gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 4000 --warmup 100 --no-cpu-baseline | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['roofline']['launches_per_step'], d['roofline']['avg_launch_us'])" || exit 1
done
