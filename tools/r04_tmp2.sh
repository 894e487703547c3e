set -o pipefail
AB_TAG=_td3 BENCH_ARGS="--algo td3 --env HalfCheetah-v4" bash tools/abplan.sh 2 6000 "-" "level_cap=640" "level_cap=896" "level_cap=1024" "pl_tn=32" "steps_per_graph=8" "steps_per_graph=24" || exit 1
AB_TAG=_sac BENCH_ARGS="--algo sac" bash tools/abplan.sh 2 3000 "-" "level_cap=768" "pre_tn=64" "steps_per_graph=16" "steps_per_graph=4" "balance=0" || exit 1
