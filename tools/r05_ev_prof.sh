#!/bin/bash
# Round-5 closing evidence in one GPU call: main (trace, PMC + per-level table, smoke, bench, rocprof stats),
# then the secondary configs; raw counter / trace CSVs removed once summarized (gpurun_out/ < 64 MiB).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
cd $ROOT
bash tools/r05_evidence.sh main || exit 1
python3 tools/pmc_levels.py $OUT/pmc_r05 > $OUT/r05_pmc_levels.txt 2>&1 || echo "(no per-level table)"
rm -rf $OUT/pmc_r05
bash tools/r05_evidence.sh second || exit 1
du -sh $OUT
