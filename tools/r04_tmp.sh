set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c11_tests.txt 2>&1; rc=$?; tail -2 gpurun_out/c11_tests.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  a=$(RLE_AQL=0 timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline | python -c "import json,sys; print(json.load(sys.stdin)['value'])") || exit 1
  b=$(timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline | python -c "import json,sys; print(json.load(sys.stdin)['value'])") || exit 1
  c=$(RLE_LIB=$PWD/sac-td3-td7_amd/lib/librle_old.so RLE_AQL=0 timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline | python -c "import json,sys; print(json.load(sys.stdin)['value'])") || exit 1
  echo "graph $a  aql $b  old $c"
done
