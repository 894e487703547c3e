#!/bin/bash
# Round 5: the whole -m gpu suite, then the headline bench line and extra seeds-per-GPU points.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT && mkdir -p gpurun_out
TAG=${1:-check}
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r05_${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/r05_${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/r05_${TAG}_tests.log
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline > gpurun_out/r05_${TAG}_bench.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r05_${TAG}_bench.json')); print('bench', d['value'], d['ms_per_step'])"
shift
for k in "$@"; do
  line=$(timeout -k 10 200 python bench.py --steps 1500 --warmup 100 --no-cpu-baseline --seeds-per-gpu $k 2>/dev/null | tail -1) || exit 1
  echo "seeds $k $(echo "$line" | python -c "import json,sys; print(json.load(sys.stdin)['value'])")" | tee -a gpurun_out/r05_${TAG}_seeds.txt
done
