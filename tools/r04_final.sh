#!/bin/bash
# Round-4 closing evidence, call A: the whole GPU suite (verbose listing), then tools/round_evidence.sh r04
# (level trace + PMC + smoke + bench + rocprofv3 summary), the per-level PMC table and the traffic model
# of the 6-step graph.  Call B is tools/r04_final2.sh.  Copy gpurun_out/r04_* into profiles/ afterwards.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
  > gpurun_out/r04_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r04_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r04_gpu_tests.txt
bash tools/round_evidence.sh r04 2000 || exit 1
python3 tools/pmc_levels.py gpurun_out/pmc_r04 > gpurun_out/r04_pmc_levels.txt 2>&1 || exit 1
RLE_TRAFFIC=1 timeout -k 10 120 python tools/describe.py td7 > gpurun_out/describe_td7_traffic.txt 2>&1 || exit 1
