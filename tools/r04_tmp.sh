set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r04_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r04_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r04_gpu_tests.txt
bash tools/r04_final2.sh || exit 1
