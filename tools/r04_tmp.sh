set -o pipefail
export RLE_LIB_EXP=$PWD/sac-td3-td7_amd/lib/librle_exp4.so
RLE_LIB=$RLE_LIB_EXP timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/c14_tests.txt 2>&1; tail -8 gpurun_out/c14_tests.txt
v() { python -c "import json,sys; print(json.load(sys.stdin)['value'])"; }
for i in 1 2; do
  a=$(timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline --algo sac | v) || exit 1
  b=$(RLE_LIB=$RLE_LIB_EXP timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline --algo sac | v) || exit 1
  echo "sac cur $a  exp4 $b"
done
AB_TAG=_td3 BENCH_ARGS="--algo td3 --env HalfCheetah-v4" bash tools/abplan.sh 2 6000 "-" "level_cap=640" "level_cap=896" "level_cap=1024" "pl_tn=32" "steps_per_graph=8" "steps_per_graph=24" || exit 1
AB_TAG=_td7rb bash tools/abplan.sh 2 3000 "-" "rb=1" || exit 1
AB_TAG=_td7rb1024 BENCH_ARGS="--batch 1024" bash tools/abplan.sh 2 1000 "-" "rb=1" "level_cap=1536" "level_cap=2048" "rb=1,level_cap=2048" || exit 1
