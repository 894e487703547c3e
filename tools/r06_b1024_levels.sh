#!/bin/bash
# Per-level traffic at B = 1024: FETCH_SIZE / WRITE_SIZE passes of the B = 1024 bench against
# the engine's per-XCD traffic model (RLE_TRAFFIC=1 describe of the same program), tools/pmc_levels.py
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT/pmc_b1024
cd $ROOT
RLE_DESC_B=1024 RLE_TRAFFIC=1 RLE_DESC_ONLY=3 timeout -k 10 120 python tools/describe.py td7 > $OUT/r06_describe_traffic_b1024.txt 2>&1 \
  || { echo DESCRIBE FAILED; tail -5 $OUT/r06_describe_traffic_b1024.txt; exit 1; }
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_b1024/p$i -o run \
     -- python3 $ROOT/bench.py --steps 200 --warmup 20 --no-cpu-baseline --batch 1024 > $OUT/pmc_b1024/p$i.log 2>&1) \
    || { echo "PMC pass $grp FAILED"; tail -5 $OUT/pmc_b1024/p$i.log; exit 1; }
done
python3 tools/pmc_levels.py $OUT/pmc_b1024 $OUT/r06_describe_traffic_b1024.txt > $OUT/r06_pmc_levels_b1024.txt 2>&1 || { tail -5 $OUT/r06_pmc_levels_b1024.txt; exit 1; }
rm -rf $OUT/pmc_b1024
tail -15 $OUT/r06_pmc_levels_b1024.txt
