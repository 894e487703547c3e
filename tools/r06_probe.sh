#!/bin/bash
# Round-6 probes (GPU box): fence-scope timing variants of the AQL path (results invalid: timing only)
# A/B against the product library, then the standalone sampler's kernel trace + PMC on this tree.
set -o pipefail
TAG=${1:-r06}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
L=sac-td3-td7_amd/lib
for v in acq0 rel0 none; do
  AB_TAG=_$v bash tools/ablib.sh $L/librle.so $L/librle_$v.so 2 2000 || { echo "AB $v FAILED"; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/samp -o run -- python3 $ROOT/tools/sampler_prof.py 300 > $OUT/samp.log 2>&1 || { tail -20 $OUT/samp.log; exit 1; }
python3 $ROOT/tools/sampler_summary.py $OUT/samp $OUT/${TAG}_sampler.csv || exit 1
mkdir -p $OUT/samp_pmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/samp_pmc/$c -o run -- python3 $ROOT/tools/sampler_prof.py 100 > $OUT/samp_pmc/$c.log 2>&1 || { tail -5 $OUT/samp_pmc/$c.log; exit 1; }
done
python3 $ROOT/tools/pmc_summary.py $OUT/samp_pmc --grid 16384 --json $OUT/${TAG}_sampler_pmc.json || exit 1
rm -rf $OUT/samp $OUT/samp_pmc
