#!/bin/bash
# Whole round evidence in one GPU call: level trace + PMC (tools/evidence.sh), copied into the
# box's profiles/ so that the bench line that follows cites them, then smoke + bench + rocprofv3
# kernel-trace summary (tools/gpu_round.sh).  Copy gpurun_out/<tag>_* into profiles/ afterwards.
# Usage (via gpurun): bash tools/round_evidence.sh <tag> [bench steps]
set -o pipefail
TAG=${1:-r02}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
bash tools/evidence.sh $TAG || exit 1
cp gpurun_out/${TAG}_pmc.json gpurun_out/${TAG}_level_trace.json profiles/ || exit 1
bash tools/gpu_round.sh $TAG ${2:-2000} || exit 1
