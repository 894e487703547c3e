#!/bin/bash
# Round-6 sampler check (GPU box): the -m gpu suite, the headline bench, the standalone sampler's kernel
# trace and FETCH/WRITE counters (tools/sampler_prof.py), and the in-graph level trace.
set -o pipefail
TAG=${1:-r06}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/${TAG}_gpu_tests.txt 2>&1 \
  || { echo "GPU TESTS FAILED"; tail -40 $OUT/${TAG}_gpu_tests.txt; exit 1; }
tail -1 $OUT/${TAG}_gpu_tests.txt
L=sac-td3-td7_amd/lib
if [ -n "$AB_BASE" ]; then AB_TAG=_$TAG bash tools/ablib.sh $AB_BASE $L/librle.so 3 2000 || exit 1; fi
RLE_TRACE=1 timeout -k 10 300 python tools/trace_levels.py 20 0,1,3 $OUT/${TAG}_level_trace.json > $OUT/${TAG}_level_trace.txt 2>&1 || { echo TRACE FAILED; tail -20 $OUT/${TAG}_level_trace.txt; exit 1; }
if [ -n "$PMC_LEVELS" ]; then
  RLE_TRAFFIC=1 RLE_DESC_ONLY=3 timeout -k 10 120 python tools/describe.py td7 > $OUT/${TAG}_describe_traffic.txt 2>&1 || { echo DESCRIBE FAILED; tail -5 $OUT/${TAG}_describe_traffic.txt; exit 1; }
  bash tools/pmc.sh $TAG || exit 1
  python3 tools/pmc_summary.py $OUT/pmc_$TAG --json $OUT/${TAG}_pmc.json > /dev/null || exit 1
  python3 tools/pmc_levels.py $OUT/pmc_$TAG $OUT/${TAG}_describe_traffic.txt > $OUT/${TAG}_pmc_levels.txt 2>&1 || { echo LEVELS FAILED; tail -5 $OUT/${TAG}_pmc_levels.txt; }
  rm -rf $OUT/pmc_$TAG
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/samp -o run -- python3 $ROOT/tools/sampler_prof.py 300 > $OUT/samp.log 2>&1 || { tail -20 $OUT/samp.log; exit 1; }
python3 $ROOT/tools/sampler_summary.py $OUT/samp $OUT/${TAG}_sampler.csv || exit 1
mkdir -p $OUT/samp_pmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/samp_pmc/$c -o run -- python3 $ROOT/tools/sampler_prof.py 100 > $OUT/samp_pmc/$c.log 2>&1 || { tail -5 $OUT/samp_pmc/$c.log; exit 1; }
done
python3 $ROOT/tools/pmc_summary.py $OUT/samp_pmc --grid 16384 --json $OUT/${TAG}_sampler_pmc.json || exit 1
rm -rf $OUT/samp $OUT/samp_pmc
