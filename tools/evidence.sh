#!/bin/bash
# Round evidence on the GPU box: level trace (text + JSON) and the PMC passes with their summary.
# Usage (via gpurun): bash tools/evidence.sh <tag>
set -o pipefail
TAG=${1:-r02}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
RLE_TRACE=1 timeout -k 10 300 python tools/trace_levels.py 20 0,1,3 $OUT/${TAG}_level_trace.json > $OUT/${TAG}_level_trace.txt 2>&1 || { echo TRACE FAILED; tail -20 $OUT/${TAG}_level_trace.txt; exit 1; }
bash tools/pmc.sh $TAG || exit 1
python tools/pmc_summary.py $OUT/pmc_$TAG --json $OUT/${TAG}_pmc.json
