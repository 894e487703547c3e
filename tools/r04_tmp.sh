set -o pipefail
export RLE_LIB_EXP=$PWD/sac-td3-td7_amd/lib/librle_exp3.so
RLE_LIB=$RLE_LIB_EXP timeout -k 10 300 python tools/diag_sacpre.py > gpurun_out/c13_diag.txt 2>&1; cat gpurun_out/c13_diag.txt | tail -14
RLE_LIB=$RLE_LIB_EXP timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/c13_tests.txt 2>&1; tail -8 gpurun_out/c13_tests.txt
v() { python -c "import json,sys; print(json.load(sys.stdin)['value'])"; }
for i in 1 2; do
  a=$(timeout -k 10 120 python bench.py --steps 6000 --warmup 200 --no-cpu-baseline --algo td3 --env HalfCheetah-v4 | v) || exit 1
  b=$(RLE_LIB=$RLE_LIB_EXP timeout -k 10 120 python bench.py --steps 6000 --warmup 200 --no-cpu-baseline --algo td3 --env HalfCheetah-v4 | v) || exit 1
  echo "td3 cur $a  exp3 $b"
  a=$(timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline --algo sac | v) || exit 1
  b=$(RLE_LIB=$RLE_LIB_EXP timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline --algo sac | v) || exit 1
  echo "sac cur $a  exp3 $b"
  a=$(timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline | v) || exit 1
  b=$(RLE_LIB=$RLE_LIB_EXP timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline | v) || exit 1
  c=$(RLE_LIB=$PWD/sac-td3-td7_amd/lib/librle_exp2.so timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline | v) || exit 1
  echo "td7 cur $a  exp3 $b  exp2 $c"
done
