#!/bin/bash
# Round-4 closing evidence, call B: secondary configs and seeds per GPU (tools/secondary.sh), the TD3 / SAC
# level traces and critical-chain listings, and PMC passes of TD3 HalfCheetah, SAC Humanoid and TD7 B=1024.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
bash tools/secondary.sh || exit 1
RLE_TRACE_ALGO=td3 timeout -k 10 120 python tools/trace_levels.py > gpurun_out/r04_level_trace_td3.txt 2>&1 || exit 1
RLE_TRACE_ALGO=sac timeout -k 10 120 python tools/trace_levels.py > gpurun_out/r04_level_trace_sac.txt 2>&1 || exit 1
RLE_DESC_CRIT=1 RLE_DESC_WG=1 timeout -k 10 120 python tools/describe.py td3 > gpurun_out/r04_crit_td3.txt 2>&1 || exit 1
RLE_DESC_CRIT=1 RLE_DESC_WG=1 timeout -k 10 120 python tools/describe.py sac > gpurun_out/r04_crit_sac.txt 2>&1 || exit 1
bash tools/pmc.sh td3 --algo td3 --env HalfCheetah-v4 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_td3 --json gpurun_out/r04_pmc_td3_halfcheetah.json || exit 1
bash tools/pmc.sh sac --algo sac || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_sac --json gpurun_out/r04_pmc_sac_humanoid.json || exit 1
