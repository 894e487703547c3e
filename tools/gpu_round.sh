#!/bin/bash
# One GPU-box pass: smoke, bench (N=1) and a rocprofv3 kernel-trace summary of the bench.
# Usage (via gpurun): bash tools/gpu_round.sh <tag> [bench steps]
set -o pipefail
TAG=${1:-r01}
STEPS=${2:-2000}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke_$TAG.log; exit 1; }
timeout -k 10 600 python bench.py --steps $STEPS --warmup 50 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo BENCH FAILED; tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_$TAG -o run --output-format csv -- python3 $ROOT/bench.py --steps 500 --warmup 20 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_$TAG.log; exit 1; }
find $OUT/prof_$TAG -name "*stats*" | head
