#!/bin/bash
# GPU test pass (gpurun): the -m gpu suite, one process, per-test timeout; log under gpurun_out/.
# Usage: bash tools/gpu_tests.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-t}
mkdir -p gpurun_out
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread "${K[@]}" > gpurun_out/gt_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/gt_$TAG.log | sed 's/^.*::/  /' | tail -120
tail -3 gpurun_out/gt_$TAG.log
exit $rc
