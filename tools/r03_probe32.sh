#!/bin/bash
# Level structure with the longest-chain marks (RLE_DESC_CRIT=1) of TD7 / TD3 / SAC.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
for a in td7 td3 sac; do
  RLE_DESC_CRIT=1 RLE_DESC_WG=1 timeout -k 10 120 python tools/describe.py $a > gpurun_out/crit_$a.txt 2>&1 || exit 1
done
echo ok
