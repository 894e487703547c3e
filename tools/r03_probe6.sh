#!/bin/bash
# Round-3 probe 6: Adam moments as streaming stores (A/B), the traffic model of the 6-step graph.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
AB_TAG=_adamnt bash tools/ablib.sh sac-td3-td7_amd/lib/librle.so sac-td3-td7_amd/lib/librle_adamnt.so 3 3000 || exit 1
RLE_TRAFFIC=1 timeout -k 10 120 python tools/describe.py td7 > gpurun_out/describe_td7_traffic.txt 2>&1 || exit 1
