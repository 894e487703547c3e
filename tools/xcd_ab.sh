#!/bin/bash
# XCD-aware tile order: parity subset, A/B bench, FETCH_SIZE per launch for both (GPU box).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "trajectory or multistep" > gpurun_out/xcd_tests.log 2>&1 || { tail -30 gpurun_out/xcd_tests.log; exit 1; }
tail -2 gpurun_out/xcd_tests.log
AB_TAG=_xcd bash tools/abk.sh RLE_XCD "0 1" 3 3000 || exit 1
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  RLE_XCD=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcx$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmcx$v.log 2>&1 || { echo pmc fail; tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmcx$v.log; exit 1; }
  echo "RLE_XCD=$v"; python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $GRAFT_REPO_ROOT/gpurun_out/pmcx$v
done
