#!/bin/bash
# Round-3 probe: GPU tests, graph description for the PMC table, rocprofv3 under RLE_AQL=1.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
bash tools/gpu_tests.sh r03e > gpurun_out/gt_r03e_summary.txt; rc=$?
grep -E "FAILED|ERROR" gpurun_out/gt_r03e_summary.txt | head -20; tail -2 gpurun_out/gt_r03e_summary.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/describe.py td7 > gpurun_out/describe_td7.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
RLE_AQL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_aql -o run --output-format csv -- python3 $ROOT/bench.py --steps 300 --warmup 20 --no-cpu-baseline > $ROOT/gpurun_out/prof_aql.log 2>&1 || exit 1
find $ROOT/gpurun_out/prof_aql -name "*stats*"
