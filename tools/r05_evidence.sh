#!/bin/bash
# Round-5 closing evidence, one GPU call per part:
#   bash tools/r05_evidence.sh main   -- level trace, PMC, smoke, the headline bench line (2000 steps), and
#                                        the same 2000-step bench run under rocprofv3 (its own line kept beside
#                                        the kernel stats, so both come from one run)
#   bash tools/r05_evidence.sh second -- B=1024, TD7 Ant, SAC Humanoid, TD3 HalfCheetah: PMC (into profiles/),
#                                        bench line, the same run under rocprofv3 (kernel stats)
set -o pipefail
PART=${1:-main}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
prof_run() {  # <tag> <bench args...>: the bench line of a run under rocprofv3 --kernel-trace --stats
  local tag=$1; shift
  (cd /tmp && export TMPDIR=/tmp && RLE_AQL=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_$tag -o run \
     --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline "$@" > $OUT/r05_${tag}_bench_prof.json 2> $OUT/prof_$tag.log) \
     || { echo "PROF $tag FAILED"; tail -20 $OUT/prof_$tag.log; return 1; }
  find $OUT/prof_$tag -name "*kernel_stats*" | head -1
  find $OUT/prof_$tag -name "*kernel_trace*" -delete  # (the stats stay; the per-dispatch trace is tens of MB)
}
if [ $PART = main ]; then
  bash tools/evidence.sh r05 || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r05.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke_r05.log; exit 1; }
  cp $OUT/r05_pmc.json $OUT/r05_level_trace.json profiles/ || exit 1
  timeout -k 10 600 python bench.py --steps 2000 --warmup 50 > $OUT/r05_bench.json 2> $OUT/r05_bench.err || { echo BENCH FAILED; tail -20 $OUT/r05_bench.err; exit 1; }
  cat $OUT/r05_bench.json
  # (RLE_AQL=0: the profiled run replays hipGraphs -- the direct AQL path writes packets into its own HSA queue,
  # which segfaults under rocprofv3's queue interception, profiles/r05_prof_crash.txt; the run's own bench line
  # is kept beside the kernel stats)
  prof_run main --steps 1000 --warmup 50 || exit 1
else
  # PMC first, into profiles/, so that the bench lines below carry this round's traffic
  for cfg in "b1024:td7_b1024:--batch 1024" "ant:td7_ant:--env Ant-v4" "td3:td3_halfcheetah:--algo td3 --env HalfCheetah-v4" "sac:sac_humanoid:--algo sac"; do
    tag=${cfg%%:*}; rest=${cfg#*:}; name=${rest%%:*}; args=${rest#*:}
    bash tools/pmc.sh $tag $args || exit 1
    python3 tools/pmc_summary.py $OUT/pmc_$tag --json $OUT/r05_pmc_$name.json || exit 1
    cp $OUT/r05_pmc_$name.json profiles/ || exit 1
    python3 tools/pmc_levels.py $OUT/pmc_$tag > $OUT/r05_pmc_levels_$name.txt 2>&1 || echo "(no per-level table for $name)"
    rm -rf $OUT/pmc_$tag  # (summaries kept; gpurun_out/ must stay under 64 MiB)
  done
  : > $OUT/r05_secondary.jsonl
  for cfg in "b1024:--batch 1024" "ant:--env Ant-v4" "sac:--algo sac" "td3:--algo td3 --env HalfCheetah-v4"; do
    tag=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 300 python bench.py --steps 2000 --warmup 50 $args >> $OUT/r05_secondary.jsonl 2> $OUT/r05_sec_$tag.err || { echo "FAILED: $args"; tail -5 $OUT/r05_sec_$tag.err; exit 1; }
    prof_run $tag --steps 1000 --warmup 50 $args || exit 1
    echo "done $tag"
  done
fi
