set -o pipefail
mkdir -p gpurun_out
for c in 16 32 64; do
  RLE_PLAN=tn_min=$c timeout -k 10 120 python bench.py --steps 3000 --no-cpu-baseline > gpurun_out/tn_$c.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/tn_$c.json').read().strip().splitlines()[-1]);print('tn_min $c',d['value'],d['roofline']['avg_launch_us'])"
done
