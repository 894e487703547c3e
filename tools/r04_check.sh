#!/bin/bash
# Round-4 check pass (gpurun): GPU suite (optional -k filter), then a short bench line.
# Usage: bash tools/r04_check.sh <tag> [pytest -k expr] [bench steps]
set -o pipefail
TAG=${1:-c}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread "${K[@]}" \
  > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.txt | head -30
tail -2 gpurun_out/${TAG}_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps ${3:-1000} --warmup 50 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
