set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c8_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/c8_tests.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for L in librle_old.so librle_nohot.so librle.so; do
    v=$(RLE_LIB=$PWD/sac-td3-td7_amd/lib/$L timeout -k 10 120 python bench.py --steps 3000 --warmup 100 --no-cpu-baseline | python -c "import json,sys; print(json.load(sys.stdin)['value'])") || exit 1
    echo -n "$L $v  "
  done
  echo
done
