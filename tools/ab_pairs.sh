#!/bin/bash
# A/B of the MFMA-pairs build (lib/librle_pairs.so, make variant V=pairs VFLAGS=-DRLE_MFMA_PAIRS=1) against the product
# library: bitwise per-step comparison on goldens, then interleaved bench pairs (headline, B=1024, TD3).
set -o pipefail
L=sac-td3-td7_amd/lib
for g in td7_tiny_zs td3_tiny_deep td7_humanoid; do
  timeout -k 10 120 python tools/bitcmp.py dump $g 4 gpurun_out/bc_a_$g.npz > gpurun_out/bc_$g.log 2>&1 || { echo dumpA $g failed; tail -5 gpurun_out/bc_$g.log; continue; }
  RLE_LIB=$L/librle_pairs.so timeout -k 10 120 python tools/bitcmp.py dump $g 4 gpurun_out/bc_b_$g.npz >> gpurun_out/bc_$g.log 2>&1 || { echo dumpB $g failed; exit 1; }
  echo "$g: $(python tools/bitcmp.py cmp gpurun_out/bc_a_$g.npz gpurun_out/bc_b_$g.npz | grep -c differ) arrays differ"
done
AB_TAG=_pairs bash tools/ab.sh RLE_LIB=$L/librle_pairs.so 3 4000 || exit 1
AB_TAG=_pairs1024 BENCH_ARGS="--batch 1024" bash tools/ab.sh RLE_LIB=$L/librle_pairs.so 2 2000 || exit 1
AB_TAG=_pairstd3 BENCH_ARGS="--algo td3 --env HalfCheetah-v4" bash tools/ab.sh RLE_LIB=$L/librle_pairs.so 2 4000
