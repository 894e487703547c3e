#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
  > gpurun_out/p46_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/p46_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/p46_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/p46_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/p46_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/p46_bench.json 2> gpurun_out/p46_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/p46_bench.json')); print(d['value'], d['roofline']['frac'])"
