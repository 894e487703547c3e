#!/bin/bash
# Round 5: the -m gpu suite (optionally a -k filter first, which stops the call on failure).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT && mkdir -p gpurun_out
TAG=${1:-t}
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests -m gpu -k "$2" > gpurun_out/r05_${TAG}_k.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/r05_${TAG}_k.log | tail -40; tail -3 gpurun_out/r05_${TAG}_k.log
  [ $rc = 0 ] || exit $rc
fi
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r05_${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/r05_${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/r05_${TAG}_tests.log
