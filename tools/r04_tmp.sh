set -o pipefail
export RLE_LIB=$PWD/sac-td3-td7_amd/lib/librle_exp8.so
AB_TAG=_td3w BENCH_ARGS="--algo td3 --env HalfCheetah-v4" bash tools/abplan.sh 2 6000 "-" "pl_w=8" "pl_w=16" "pl_w=24" || exit 1
AB_TAG=_sacw BENCH_ARGS="--algo sac" bash tools/abplan.sh 2 3000 "-" "pl_w=8" "pl_w=16" "pl_w=24" || exit 1
