#!/bin/bash
# PMC passes over a short bench run (GPU box): one rocprofv3 process per counter group.
# Usage: bash tools/pmc.sh <tag> [extra bench.py args, e.g. --batch 1024]
set -o pipefail
TAG=${1:-r01}
shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU" "SQC_ICACHE_MISSES SQC_ICACHE_HITS TCC_HIT_sum TCC_MISS_sum" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $ROOT/bench.py --steps 200 --warmup 20 --no-cpu-baseline "$@" > $OUT/p$i.log 2>&1 || { echo "PMC pass $i ($grp) FAILED"; tail -5 $OUT/p$i.log; exit 1; }
done
find $OUT -name "*counter_collection*" | head
