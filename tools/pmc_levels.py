"""Per-level PMC counters of the TD7 step from tools/pmc.sh output (GPU box CSVs).

Usage: python tools/pmc_levels.py <pmc dir>
rle_level dispatches are grouped by their grid size sequence: the steady state alternates
the plain and the policy graph; each level's counters are averaged over its occurrences
(matched by position in the graph and grid size).
"""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
disp = defaultdict(dict)  # dispatch id -> {counter: value, '_grid': n}
for f in glob.glob(f"{root}/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rle_level" not in r["Kernel_Name"]:
            continue
        key = (f.split("/")[-2], int(r["Dispatch_Id"]))
        d = disp[key]
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["_grid"] = int(r["Grid_Size"]) // 256
        d["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
# per pass: ordered sequences of dispatches
passes = defaultdict(list)
for (p, i), d in sorted(disp.items()):
    passes[p].append(d)
# find the two graphs: the sequence after the first (prime) dispatch repeats with period P
for p, seq in sorted(passes.items()):
    grids = [d["_grid"] for d in seq[1:]]
    period = next(P for P in range(2, 200) if grids[P:P * 20] == grids[:P * 19][:len(grids[P:P * 20])])
    agg = defaultdict(lambda: defaultdict(list))
    for k, d in enumerate(seq[1:]):
        for c, v in d.items():
            agg[k % period][c].append(v)
    names = sorted(c for c in agg[0] if not c.startswith("_"))
    print(f"== pass {p}: period {period} levels")
    print("lvl  grid   us   " + "  ".join(f"{n[:14]:>14s}" for n in names))
    for k in range(period):
        a = agg[k]
        mean = lambda c: sum(a[c]) / len(a[c])
        print(f"{k:3d} {int(mean('_grid')):5d} {mean('_ns') / 1000:5.1f}  " +
              "  ".join(f"{mean(n):14.1f}" for n in names))
