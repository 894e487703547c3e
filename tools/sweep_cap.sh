set -o pipefail
mkdir -p gpurun_out
for c in default 1024 1280 896 768; do
  if [ $c = default ]; then unset RLE_PLAN; else export RLE_PLAN=level_cap=$c; fi
  timeout -k 10 120 python bench.py --steps 3000 --no-cpu-baseline > gpurun_out/sw_$c.json 2>&1 || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sw_$c.json'));print('$c',d['value'],d['roofline']['launches_per_step'])"
done
