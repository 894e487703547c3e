set -o pipefail
for v in dwnoloop nonstore noloop; do
  AB_TAG=_$v bash tools/ablib.sh sac-td3-td7_amd/lib/librle.so sac-td3-td7_amd/lib/librle_$v.so 2 3000 || exit 1
done
RLE_TRACE=1 timeout -k 10 200 python tools/trace_levels.py 20 3 > gpurun_out/tr3_new.txt 2>&1 || exit 1
timeout -k 10 300 python tools/cpu_multiseed.py --procs 8 --threads 16 > gpurun_out/cpu_multiseed.json 2> gpurun_out/cpu_multiseed.err; tail -1 gpurun_out/cpu_multiseed.json
