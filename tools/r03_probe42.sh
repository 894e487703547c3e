#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "prelayer or audit or hazard" > gpurun_out/p42_tests.txt 2>&1 || { tail -60 gpurun_out/p42_tests.txt; exit 1; }
tail -2 gpurun_out/p42_tests.txt
timeout -k 10 300 python bench.py --algo sac --steps 2000 --warmup 50 > gpurun_out/p42_sac.json 2> gpurun_out/p42_sac.err || exit 1
timeout -k 10 300 python bench.py --algo sac --steps 2000 --warmup 50 --seeds-per-gpu 3 --no-cpu-baseline > gpurun_out/p42_sac3.json 2>> gpurun_out/p42_sac.err || exit 1
RLE_TRACE_ALGO=sac timeout -k 10 120 python tools/trace_levels.py > gpurun_out/p42_trace_sac.txt 2>&1 || exit 1
python -c "import json; [print(json.load(open(f))['value']) for f in ('gpurun_out/p42_sac.json','gpurun_out/p42_sac3.json')]"
