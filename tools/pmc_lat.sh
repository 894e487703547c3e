#!/bin/bash
# Memory-pipeline PMC passes per rle_level dispatch (GPU box): TA busy, TCP -> L2 read latency and
# stalls, VMEM instruction level (latency) -- one rocprofv3 --pmc pass each, then per-level means.
# Usage: bash tools/pmc_lat.sh <tag>
set -o pipefail
TAG=${1:-lat}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" "SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $ROOT/bench.py --steps 60 --warmup 10 --no-cpu-baseline > $OUT/p$i.log 2>&1 || { echo "PMC pass $i ($grp) FAILED"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 $ROOT/tools/pmc_levels.py $OUT > $OUT/levels.txt 2>&1; tail -3 $OUT/levels.txt
