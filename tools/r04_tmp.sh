set -o pipefail
AB_TAG=_td7w2 BENCH_ARGS="" bash tools/abplan.sh 2 4000 "-" "adam_w=4" "adam_w=6" "adam_w=10" "adam_w=12" || exit 1
AB_TAG=_td3w3 BENCH_ARGS="--algo td3 --env HalfCheetah-v4" bash tools/abplan.sh 2 6000 "-" "tiny_w=15" "tiny_w=60" "pl_w=8" "adam_w=4" || exit 1
AB_TAG=_sacw4 BENCH_ARGS="--algo sac" bash tools/abplan.sh 2 3000 "-" "tiny_w=15" "tiny_w=60" "head_w=30" || exit 1
