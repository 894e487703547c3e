#!/bin/bash
# Round-5 GPU check after the 64-row tiles, batched AvgL1Norm tables and rb at B >= 512: the wide / large-batch
# parity tests, B = 1024 / 512 / 256 bench lines, B = 1024 level trace.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT && mkdir -p gpurun_out
T=${1:-c7}
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 240 --timeout-method thread \
  -k "wide or B1024 or B512 or b1024" > gpurun_out/r05_${T}_tests.txt 2>&1
tail -3 gpurun_out/r05_${T}_tests.txt
timeout -k 10 300 python bench.py --batch 1024 --steps 500 --warmup 20 --no-cpu-baseline > gpurun_out/r05_${T}_b1024.json 2> gpurun_out/r05_${T}_b1024.err || exit 1
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline > gpurun_out/r05_${T}_b256.json 2>&1 || exit 1
RLE_TRACE=1 RLE_TRACE_BATCH=1024 timeout -k 10 300 python tools/trace_levels.py 20 3 > gpurun_out/r05_${T}_trace_b1024.txt 2>&1
