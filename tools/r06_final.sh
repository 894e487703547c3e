#!/bin/bash
# Round-6 closing evidence, one GPU call per part (each GPU step under its own time limit):
#   bash tools/r06_final.sh main   -- -m gpu suite, level trace, PMC passes + per-level table with the per-XCD traffic
#                                     model, the standalone sampler's trace + counters, smoke, the headline line (2000
#                                     steps) and the driver's 20-step command x3, then the same bench under rocprofv3
#                                     --kernel-trace --stats on the default direct-AQL path and on hipGraph replays
#                                     (plan dispatch=0), each with its own line
#   bash tools/r06_final.sh second -- B=1024, TD7 Ant, SAC Humanoid, TD3 HalfCheetah: PMC (into profiles/), bench line,
#                                     kernel stats (AQL path); then 2 / 4 TD7 seeds per GPU
set -o pipefail
PART=${1:-main}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
prof_run() {  # <tag> <bench args...>: kernel stats of a bench run under rocprofv3, its own line beside them
  local tag=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_$tag -o run \
     --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline "$@" > $OUT/r06_kernel_stats_${tag}_line.json 2> $OUT/prof_$tag.log) \
     || { echo "PROF $tag FAILED"; tail -20 $OUT/prof_$tag.log; return 1; }
  cp $(find $OUT/prof_$tag -name "*kernel_stats*" | head -1) $OUT/r06_kernel_stats_$tag.csv || return 1
  rm -rf $OUT/prof_$tag
  head -2 $OUT/r06_kernel_stats_$tag.csv
}
if [ $PART = main ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/r06_gpu_tests.txt 2>&1 \
    || { echo "GPU TESTS FAILED"; tail -30 $OUT/r06_gpu_tests.txt; exit 1; }
  tail -1 $OUT/r06_gpu_tests.txt
  RLE_TRACE=1 timeout -k 10 300 python tools/trace_levels.py 20 0,1,3 $OUT/r06_level_trace.json > $OUT/r06_level_trace.txt 2>&1 \
    || { echo TRACE FAILED; tail -20 $OUT/r06_level_trace.txt; exit 1; }
  RLE_TRAFFIC=1 RLE_DESC_ONLY=3 timeout -k 10 120 python tools/describe.py td7 > $OUT/r06_describe_traffic.txt 2>&1 \
    || { echo DESCRIBE FAILED; exit 1; }
  bash tools/pmc.sh r06 || exit 1
  python3 tools/pmc_summary.py $OUT/pmc_r06 --json $OUT/r06_pmc.json > /dev/null || exit 1
  python3 tools/pmc_levels.py $OUT/pmc_r06 $OUT/r06_describe_traffic.txt > $OUT/r06_pmc_levels.txt 2>&1 || echo "(no per-level table)"
  rm -rf $OUT/pmc_r06
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/samp -o run \
     -- python3 $ROOT/tools/sampler_prof.py 300 > $OUT/samp.log 2>&1) || { tail -20 $OUT/samp.log; exit 1; }
  python3 tools/sampler_summary.py $OUT/samp $OUT/r06_sampler.csv || exit 1
  mkdir -p $OUT/samp_pmc
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/samp_pmc/$c -o run \
       -- python3 $ROOT/tools/sampler_prof.py 100 > $OUT/samp_pmc/$c.log 2>&1) || { tail -5 $OUT/samp_pmc/$c.log; exit 1; }
  done
  python3 tools/pmc_summary.py $OUT/samp_pmc --grid 16384 --json $OUT/r06_sampler_pmc.json > /dev/null || exit 1
  rm -rf $OUT/samp $OUT/samp_pmc
  # (the bench lines below cite this round's PMC and sampler files)
  cp $OUT/r06_pmc.json $OUT/r06_sampler.csv $OUT/r06_sampler_pmc.json profiles/ || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r06_smoke.txt 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/r06_smoke.txt; exit 1; }
  timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > $OUT/r06_bench.json 2> $OUT/r06_bench.err || { echo BENCH FAILED; tail -20 $OUT/r06_bench.err; exit 1; }
  cat $OUT/r06_bench.json
  : > $OUT/r06_driver_cmd.jsonl
  for i in 1 2 3; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 >> $OUT/r06_driver_cmd.jsonl 2> $OUT/r06_driver.err || { echo DRIVER CMD FAILED; tail -20 $OUT/r06_driver.err; exit 1; }
  done
  prof_run main --steps 1000 --warmup 50 || exit 1
  prof_run main_graph --steps 1000 --warmup 50 --plan dispatch=0 || exit 1
else
  for cfg in "b1024:td7_b1024:--batch 1024" "ant:td7_ant:--env Ant-v4" "td3:td3_halfcheetah:--algo td3 --env HalfCheetah-v4" "sac:sac_humanoid:--algo sac"; do
    tag=${cfg%%:*}; rest=${cfg#*:}; name=${rest%%:*}; args=${rest#*:}
    bash tools/pmc.sh $tag $args || exit 1
    python3 tools/pmc_summary.py $OUT/pmc_$tag --json $OUT/r06_pmc_$name.json > /dev/null || exit 1
    cp $OUT/r06_pmc_$name.json profiles/ || exit 1
    rm -rf $OUT/pmc_$tag
  done
  : > $OUT/r06_secondary_configs.jsonl
  for cfg in "b1024:--batch 1024" "ant:--env Ant-v4" "sac:--algo sac" "td3:--algo td3 --env HalfCheetah-v4"; do
    tag=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 300 python bench.py --steps 2000 --warmup 50 $args >> $OUT/r06_secondary_configs.jsonl 2> $OUT/r06_sec_$tag.err \
      || { echo "FAILED: $args"; tail -5 $OUT/r06_sec_$tag.err; exit 1; }
    prof_run $tag --steps 1000 --warmup 50 $args || exit 1
    echo "done $tag"
  done
  : > $OUT/r06_multiseed.jsonl
  for k in 2 4; do
    timeout -k 10 300 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline --seeds-per-gpu $k >> $OUT/r06_multiseed.jsonl 2> $OUT/r06_ms.err \
      || { echo "FAILED: seeds $k"; tail -5 $OUT/r06_ms.err; exit 1; }
  done
  cat $OUT/r06_multiseed.jsonl
fi
du -sh $OUT
