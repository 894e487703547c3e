set -o pipefail
export RLE_LIB_EXP=$PWD/sac-td3-td7_amd/lib/librle_exp6.so
RLE_LIB=$RLE_LIB_EXP timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/c17_tests.txt 2>&1; tail -4 gpurun_out/c17_tests.txt; grep -q " passed" gpurun_out/c17_tests.txt && ! grep -q "failed" gpurun_out/c17_tests.txt || exit 1
v() { python -c "import json,sys; print(json.load(sys.stdin)['value'])"; }
for i in 1 2 3; do
  a=$(timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline --algo sac | v) || exit 1
  b=$(RLE_LIB=$RLE_LIB_EXP timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline --algo sac | v) || exit 1
  echo "sac cur $a  exp6 $b"
done
a=$(timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline | v) || exit 1
b=$(RLE_LIB=$RLE_LIB_EXP timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline | v) || exit 1
echo "td7 cur $a  exp6 $b"
RLE_LIB=$RLE_LIB_EXP RLE_TRACE_ALGO=sac timeout -k 10 120 python tools/trace_levels.py > gpurun_out/c17_trace_sac.txt 2>&1 || exit 1
