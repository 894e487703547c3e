#!/bin/bash
# Round-5 closing call: the whole -m gpu suite, then the evidence (tools/r05_ev_prof.sh) and the driver's
# own bench command (20 steps after 5 warmup steps) three times.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r05_final_tests.log 2>&1 || { tail -30 gpurun_out/r05_final_tests.log; exit 1; }
tail -1 gpurun_out/r05_final_tests.log
bash tools/r05_ev_prof.sh || exit 1
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_driver_cmd_$i.json 2>/dev/null || exit 1
done
