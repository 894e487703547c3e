#!/bin/bash
# Round-4 evidence pass 1 (gpurun): standalone sampler kernel trace + its FETCH/WRITE counters,
# and PMC passes of the secondary configs (B=1024, TD3 HalfCheetah, SAC Humanoid).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/samp -o run -- python3 $ROOT/tools/sampler_prof.py 300 > $OUT/samp.log 2>&1 || { tail -20 $OUT/samp.log; exit 1; }
python3 $ROOT/tools/sampler_summary.py $OUT/samp $OUT/r04_sampler.csv || exit 1
mkdir -p $OUT/samp_pmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $OUT/samp_pmc/$c -o run -- python3 $ROOT/tools/sampler_prof.py 100 > $OUT/samp_pmc/$c.log 2>&1 || { tail -5 $OUT/samp_pmc/$c.log; exit 1; }
done
python3 $ROOT/tools/pmc_summary.py $OUT/samp_pmc --grid 16384 --json $OUT/r04_sampler_pmc.json > /dev/null || exit 1
cd $ROOT
bash tools/pmc.sh b1024 --batch 1024 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_b1024 --json gpurun_out/r04_pmc_td7_b1024.json || exit 1
bash tools/pmc.sh td3 --algo td3 --env HalfCheetah-v4 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_td3 --json gpurun_out/r04_pmc_td3_halfcheetah.json || exit 1
bash tools/pmc.sh sac --algo sac || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_sac --json gpurun_out/r04_pmc_sac_humanoid.json || exit 1
