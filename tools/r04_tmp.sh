set -o pipefail
export RLE_LIB_EXP=$PWD/sac-td3-td7_amd/lib/librle_exp2.so
RLE_LIB=$RLE_LIB_EXP timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "twostage or sac_target_pre or prelayer or burst or trajectory or td3 or sac" > gpurun_out/c12_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/c12_tests.txt; [ $rc -eq 0 ] || exit $rc
v() { python -c "import json,sys; print(json.load(sys.stdin)['value'])"; }
for i in 1 2; do
  a=$(timeout -k 10 120 python bench.py --steps 6000 --warmup 200 --no-cpu-baseline --algo td3 --env HalfCheetah-v4 | v) || exit 1
  b=$(RLE_LIB=$RLE_LIB_EXP timeout -k 10 120 python bench.py --steps 6000 --warmup 200 --no-cpu-baseline --algo td3 --env HalfCheetah-v4 | v) || exit 1
  echo "td3 cur $a  exp $b"
  a=$(timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline --algo sac | v) || exit 1
  b=$(RLE_LIB=$RLE_LIB_EXP timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline --algo sac | v) || exit 1
  echo "sac cur $a  exp $b"
  a=$(timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline | v) || exit 1
  b=$(RLE_LIB=$RLE_LIB_EXP timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline | v) || exit 1
  echo "td7 cur $a  exp $b"
done
