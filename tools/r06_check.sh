#!/bin/bash
# Round-6 GPU check: the -m gpu suite, the headline bench line (2000 steps and the driver's 20-step
# command), then the same bench under rocprofv3 --kernel-trace --stats on the DEFAULT dispatch path
# (direct AQL; its own line kept beside the kernel stats).  Each GPU step under its own time limit.
set -o pipefail
TAG=${1:-r06}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/${TAG}_gpu_tests.txt 2>&1 \
  || { echo "GPU TESTS FAILED"; tail -40 $OUT/${TAG}_gpu_tests.txt; exit 1; }
tail -1 $OUT/${TAG}_gpu_tests.txt
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err \
  || { echo BENCH FAILED; tail -20 $OUT/${TAG}_bench.err; exit 1; }
cat $OUT/${TAG}_bench.json
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/${TAG}_driver_cmd.json 2>&1 \
  || { echo DRIVER CMD FAILED; tail -20 $OUT/${TAG}_driver_cmd.json; exit 1; }
cat $OUT/${TAG}_driver_cmd.json
if [ -x build/mbsplit ]; then
  timeout -k 10 300 build/mbsplit build/mbsplit_k.co > $OUT/${TAG}_mbsplit.txt 2>&1 || { echo "MBSPLIT FAILED"; tail -20 $OUT/${TAG}_mbsplit.txt; exit 1; }
  cat $OUT/${TAG}_mbsplit.txt
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_$TAG -o run --output-format csv -- \
  python3 $ROOT/bench.py --no-cpu-baseline --steps 1000 --warmup 50 > $OUT/${TAG}_kernel_stats_line.json 2> $OUT/prof_$TAG.log \
  || { echo "PROF FAILED rc=$?"; tail -40 $OUT/prof_$TAG.log; exit 1; }
cat $OUT/${TAG}_kernel_stats_line.json
f=$(find $OUT/prof_$TAG -name "*kernel_stats*" | head -1); cp $f $OUT/${TAG}_kernel_stats.csv; cat $f | head -8
find $OUT/prof_$TAG -name "*kernel_trace*" -delete
