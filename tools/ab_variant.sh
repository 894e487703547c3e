#!/bin/bash
# Bitwise check + interleaved A/B of experiment builds (make variant V=<name> ...: lib/librle_<name>.so) against the
# product library: bash tools/ab_variant.sh <name>...  (goldens via tools/bitcmp.py, then bench pairs: headline
# x3, B=1024 x2, TD3 x2)
set -o pipefail
L=sac-td3-td7_amd/lib
for v in "$@"; do
  for g in td7_tiny td7_tiny_zs td3_tiny_deep td7_humanoid; do
    [ -f gpurun_out/bc_a_$g.npz ] || timeout -k 10 120 python tools/bitcmp.py dump $g 4 gpurun_out/bc_a_$g.npz > gpurun_out/bc_$g.log 2>&1 || { echo dumpA $g failed; tail -3 gpurun_out/bc_$g.log; exit 1; }
    RLE_LIB=$L/librle_$v.so timeout -k 10 120 python tools/bitcmp.py dump $g 4 gpurun_out/bc_${v}_$g.npz >> gpurun_out/bc_$g.log 2>&1 || { echo dump $v $g failed; exit 1; }
    echo "$v $g: $(python tools/bitcmp.py cmp gpurun_out/bc_a_$g.npz gpurun_out/bc_${v}_$g.npz | grep -c differ || true) arrays differ"
  done
done
for v in "$@"; do
  AB_TAG=_$v bash tools/ab.sh RLE_LIB=$L/librle_$v.so 3 4000 || exit 1
  AB_TAG=_${v}1024 BENCH_ARGS="--batch 1024" bash tools/ab.sh RLE_LIB=$L/librle_$v.so 2 2000 || exit 1
  AB_TAG=_${v}td3 BENCH_ARGS="--algo td3 --env HalfCheetah-v4" bash tools/ab.sh RLE_LIB=$L/librle_$v.so 2 4000 || exit 1
done
