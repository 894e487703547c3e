set -o pipefail
mkdir -p gpurun_out
for r in 2 4 6 8; do
  if [ $r = 4 ]; then unset RLE_LIB; else export RLE_LIB=$PWD/sac-td3-td7_amd/lib/librle_ring$r.so; fi
  timeout -k 10 120 python bench.py --steps 3000 --no-cpu-baseline > gpurun_out/ring_$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ring_$r.json').read().strip().splitlines()[-1]);print('ring $r',d['value'],d['roofline']['avg_launch_us'])"
done
