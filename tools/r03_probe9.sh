#!/bin/bash
# Round-3 probe 9: level structure of the TD3 and SAC step graphs.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
for a in td3 sac; do
  RLE_DESC_WG=1 timeout -k 10 120 python tools/describe.py $a > gpurun_out/describe_$a.txt 2>&1 || exit 1
done
