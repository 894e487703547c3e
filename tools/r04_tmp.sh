set -o pipefail
AB_TAG=_td7p BENCH_ARGS="" bash tools/abplan.sh 2 4000 "-" "tn_min=32" "flat_div=2" "flat_div=8" "tiny_wg=4" "level_cap=960" "level_cap=1088" || exit 1
