set -o pipefail
AB_TAG=_td7w BENCH_ARGS="" bash tools/abplan.sh 2 4000 "-" "lap_w=20" "lap_w=40" "head_w=30" "head_w=90" "adam_w=0" "adam_w=16" || exit 1
AB_TAG=_sacw2 BENCH_ARGS="--algo sac" bash tools/abplan.sh 2 3000 "-" "head_w=30" "adam_w=0" "adam_w=16" || exit 1
AB_TAG=_td3w2 BENCH_ARGS="--algo td3 --env HalfCheetah-v4" bash tools/abplan.sh 2 6000 "-" "head_w=30" "adam_w=0" "adam_w=16" || exit 1
