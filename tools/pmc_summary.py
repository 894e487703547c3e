"""Average rocprofv3 PMC counters per dispatch of rle_level from tools/pmc.sh output."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(list)
for f in glob.glob(f"{root}/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rle_level" not in r.get("Kernel_Name", ""):
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:24s} dispatches {len(v):6d}  mean/dispatch {sum(v) / len(v):14.1f}")
