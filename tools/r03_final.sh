#!/bin/bash
# Round-3 evidence in one GPU call: level trace + PMC + smoke + bench + rocprofv3 summary
# (tools/round_evidence.sh), the traffic model of the 6-step graph, secondary configs and
# several seeds per GPU.  Copy the results into profiles/ afterwards.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
bash tools/round_evidence.sh r03 2000 || exit 1
RLE_TRAFFIC=1 timeout -k 10 120 python tools/describe.py td7 > gpurun_out/describe_td7_traffic.txt 2>&1 || exit 1
bash tools/secondary.sh || exit 1
