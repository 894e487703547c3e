#!/bin/bash
# Round-4 closing evidence in one GPU call: the whole GPU suite (verbose listing), then
# tools/round_evidence.sh r04 (level trace + PMC + smoke + bench + rocprofv3 summary), the
# traffic model of the 6-step graph, and the secondary configs / seeds per GPU.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
  > gpurun_out/r04_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r04_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r04_gpu_tests.txt
bash tools/round_evidence.sh r04 2000 || exit 1
RLE_TRAFFIC=1 timeout -k 10 120 python tools/describe.py td7 > gpurun_out/describe_td7_traffic.txt 2>&1 || exit 1
bash tools/secondary.sh || exit 1
RLE_TRACE_ALGO=td3 timeout -k 10 120 python tools/trace_levels.py > gpurun_out/r04_level_trace_td3.txt 2>&1 || exit 1
RLE_DESC_CRIT=1 RLE_DESC_WG=1 timeout -k 10 120 python tools/describe.py td3 > gpurun_out/r04_crit_td3.txt 2>&1 || exit 1
RLE_DESC_CRIT=1 RLE_DESC_WG=1 timeout -k 10 120 python tools/describe.py td7 > gpurun_out/r04_crit_td7.txt 2>&1 || exit 1
RLE_TRACE_ALGO=sac timeout -k 10 120 python tools/trace_levels.py > gpurun_out/r04_level_trace_sac.txt 2>&1 || exit 1
