"""Average rocprofv3 PMC counters per dispatch of rle_level from tools/pmc.sh output.

Usage: python tools/pmc_summary.py <pmc dir> [--json out.json] [--grid THREADS]
(--grid: only dispatches of that many work-items, e.g. the standalone sampler's 64 x 256)
FETCH_SIZE / WRITE_SIZE are in KB as rocprofv3 reports them (bench.py applies the gfx950
x2 correction to FETCH_SIZE)."""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(list)
grid = int(sys.argv[sys.argv.index("--grid") + 1]) if "--grid" in sys.argv else None
for f in glob.glob(f"{root}/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rle_level" not in r.get("Kernel_Name", ""):
            continue
        if grid is not None and int(r.get("Grid_Size", r.get("Grid_Size_X", "0"))) != grid:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
summary = {}
for k in sorted(vals):
    v = vals[k]
    summary[k] = sum(v) / len(v)
    print(f"{k:24s} dispatches {len(v):6d}  mean/dispatch {summary[k]:14.1f}")
if "--json" in sys.argv:
    out = sys.argv[sys.argv.index("--json") + 1]
    summary["_dispatches"] = {k: len(v) for k, v in vals.items()}
    summary["_note"] = "mean per rle_level dispatch over a bench.py --steps 200 run; FETCH_SIZE/WRITE_SIZE in KB"
    json.dump(summary, open(out, "w"), indent=1, sort_keys=True)
