#!/bin/bash
# Run-to-run determinism evidence (GPU box): the cross-launch coherence microbenchmark, then the
# td7_humanoid_64k trajectory dumped by builds A and B (RLE_LIB) twice each and compared bitwise.
# Usage (via gpurun): bash tools/determinism.sh <tag> <libA> <libB> [steps]
set -o pipefail
TAG=${1:-det}
A=${2:-sac-td3-td7_amd/lib/librle.so}
B=${3:-sac-td3-td7_amd/lib/librle_early.so}
STEPS=${4:-12}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
if [ -x build/mbcoh ]; then
  timeout -k 10 120 build/mbcoh 200 20 | tee $OUT/${TAG}_mbcoh.txt || exit 1
fi
# BITCMP_BURST=6 (env): compare after whole 6-step graph replays instead of single steps
for run in 1 2; do
  RLE_LIB=$ROOT/$A timeout -k 10 300 python tools/bitcmp.py dump td7_humanoid_64k $STEPS $OUT/${TAG}_a$run.npz || exit 1
  RLE_LIB=$ROOT/$B timeout -k 10 300 python tools/bitcmp.py dump td7_humanoid_64k $STEPS $OUT/${TAG}_b$run.npz || exit 1
done
{
  echo "== A run 1 vs A run 2 ($A)"; python tools/bitcmp.py cmp $OUT/${TAG}_a1.npz $OUT/${TAG}_a2.npz
  echo "== B run 1 vs B run 2 ($B)"; python tools/bitcmp.py cmp $OUT/${TAG}_b1.npz $OUT/${TAG}_b2.npz
  echo "== A vs B"; python tools/bitcmp.py cmp $OUT/${TAG}_a1.npz $OUT/${TAG}_b1.npz
} 2>&1 | tee $OUT/${TAG}_bitcmp.txt
rm -f $OUT/${TAG}_a?.npz $OUT/${TAG}_b?.npz
