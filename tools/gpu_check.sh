set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline > gpurun_out/bench_qhead.json 2>gpurun_out/bench_qhead.err && cat gpurun_out/bench_qhead.json
