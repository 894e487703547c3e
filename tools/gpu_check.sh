#!/bin/bash
# GPU box: parity tests (-m gpu) then a short headline bench (no CPU baseline).
# Usage: bash tools/gpu_check.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-chk}
shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
cd $ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt_$TAG.log 2>&1
rc=$?
tail -4 gpurun_out/gt_$TAG.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gt_$TAG.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 3000 --no-cpu-baseline "$@" > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { tail -5 gpurun_out/b_$TAG.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/b_$TAG.json').read().strip().splitlines()[-1]);print('$TAG value',d['value'],'launches',d['roofline']['launches_per_step'],'us/launch',d['roofline']['avg_launch_us'])"
