#!/bin/bash
# Round-3 probe 4: packed multi-seed groups (parity tests, then the K-seed bench with and
# without packing), the timing-only variants (no MFMA anywhere; no DW instruction priority)
# and the traffic model of the 6-step graph.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -k "packed or group_rejects" -x -v --timeout 200 \
  --timeout-method thread > gpurun_out/r03_group_tests.txt 2>&1 || { tail -40 gpurun_out/r03_group_tests.txt; exit 1; }
tail -3 gpurun_out/r03_group_tests.txt
for K in 3 2; do
  for mode in "" "--packed"; do
    timeout -k 10 240 python bench.py --seeds-per-gpu $K $mode --steps 2000 --warmup 60 --no-cpu-baseline \
      >> gpurun_out/r03_multiseed.jsonl 2> gpurun_out/r03_multiseed_err.txt || { tail -30 gpurun_out/r03_multiseed_err.txt; exit 1; }
    tail -1 gpurun_out/r03_multiseed.jsonl | cut -c1-200
  done
done
timeout -k 10 200 python bench.py --steps 3000 --warmup 60 --no-cpu-baseline > gpurun_out/r03_single.json 2>&1 || exit 1
cut -c1-200 gpurun_out/r03_single.json
AB_TAG=_maxops bash tools/abenv.sh 2 3000 - RLE_MAX_OPS=32 RLE_MAX_OPS=16 || exit 1
for v in nomfma noprio; do
  AB_TAG=_$v bash tools/ablib.sh sac-td3-td7_amd/lib/librle.so sac-td3-td7_amd/lib/librle_$v.so 2 3000 || exit 1
done
RLE_TRAFFIC=1 timeout -k 10 120 python tools/describe.py td7 > gpurun_out/describe_td7_traffic.txt 2>&1 || exit 1
