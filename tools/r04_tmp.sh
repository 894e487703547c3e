set -o pipefail
export RLE_LIB_EXP=$PWD/sac-td3-td7_amd/lib/librle_exp5.so
RLE_LIB=$RLE_LIB_EXP timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/c16_tests.txt 2>&1; tail -4 gpurun_out/c16_tests.txt; grep -q " passed" gpurun_out/c16_tests.txt && ! grep -q "failed" gpurun_out/c16_tests.txt || exit 1
v() { python -c "import json,sys; print(json.load(sys.stdin)['value'])"; }
for i in 1 2; do
  a=$(timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline | v) || exit 1
  b=$(RLE_LIB=$RLE_LIB_EXP timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline | v) || exit 1
  echo "td7 cur $a  exp5 $b"
  a=$(timeout -k 10 120 python bench.py --steps 6000 --warmup 200 --no-cpu-baseline --algo td3 --env HalfCheetah-v4 | v) || exit 1
  b=$(RLE_LIB=$RLE_LIB_EXP timeout -k 10 120 python bench.py --steps 6000 --warmup 200 --no-cpu-baseline --algo td3 --env HalfCheetah-v4 | v) || exit 1
  echo "td3 cur $a  exp5 $b"
  a=$(timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline --algo sac | v) || exit 1
  b=$(RLE_LIB=$RLE_LIB_EXP timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline --algo sac | v) || exit 1
  echo "sac cur $a  exp5 $b"
done
a=$(timeout -k 10 120 python bench.py --steps 1000 --warmup 50 --no-cpu-baseline --batch 1024 | v) || exit 1
b=$(RLE_LIB=$RLE_LIB_EXP timeout -k 10 120 python bench.py --steps 1000 --warmup 50 --no-cpu-baseline --batch 1024 | v) || exit 1
echo "b1024 cur $a  exp5 $b"
