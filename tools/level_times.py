"""Join a rocprofv3 kernel trace of bench.py with the graph description: per-level us."""
import csv, re, statistics, sys
desc_path, trace_path = sys.argv[1], sys.argv[2]
txt = open(desc_path).read()
graphs = [g for g in txt.split("=== graph ") if g.strip()]
rows = list(csv.DictReader(open(trace_path)))
lv = [r for r in rows if "rle_level" in r["Kernel_Name"]]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in lv]
grids = [int(r["Grid_Size_X"]) // 256 for r in lv]
for g in graphs:
    lines = [l for l in g.splitlines() if l.startswith("L")]
    want = [int(re.search(r"wg=(\d+)", l).group(1)) for l in lines]
    n = len(want)
    hits = [i for i in range(len(grids) - n + 1) if grids[i:i + n] == want]
    hits = hits[len(hits) // 2:]  # steady state: second half of the run
    if not hits:
        print("no match for graph", g[:3]); continue
    per = [statistics.median(dur[i + k] for i in hits) for k in range(n)]
    print(f"=== graph {g[:1]}: {len(hits)} occurrences, sum of level medians {sum(per):.1f} us")
    for l, p in zip(lines, per):
        print(f"{p:8.2f} us  {l[:160]}")
