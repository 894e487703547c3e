"""Overlap of the level launches of several seeds on one GPU, from a rocprofv3 kernel trace
(tools/r05_seeds.sh): python tools/seed_overlap.py gpurun_out/r05_seedsK/run_kernel_trace.csv
Per queue (one per seed's HIP stream): launches, mean launch duration, mean gap between its consecutive
launches; device-wide: the union of all launch intervals (busy) against the traced window, and the time with
1, 2, 3, ... launches resident at once."""
import csv
import sys
from collections import defaultdict

import numpy as np

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "rle_level" in r["Kernel_Name"]]
if not rows:
    sys.exit("no rle_level dispatches")
# the timed region: the last 70% of the dispatches (warm-up and graph capture excluded)
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[int(len(rows) * 0.3):]
q = defaultdict(list)
for r in rows:
    q[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
t0 = min(s for v in q.values() for s, _ in v)
t1 = max(e for v in q.values() for _, e in v)
print(f"window {(t1 - t0) / 1e3:.1f} us, {len(rows)} launches, {len(q)} queues")
for k, v in sorted(q.items()):
    v.sort()
    d = np.array([e - s for s, e in v]) / 1e3
    g = np.array([v[i + 1][0] - v[i][1] for i in range(len(v) - 1)]) / 1e3
    print(f"  queue {k}: {len(v)} launches, mean {d.mean():.2f} us, gap to its next launch mean {g.mean():.2f} us"
          f" (p10 {np.percentile(g, 10):.2f}, p90 {np.percentile(g, 90):.2f})")
ev = sorted([(s, 1) for v in q.values() for s, _ in v] + [(e, -1) for v in q.values() for _, e in v])
occ = defaultdict(int)
cur, last = 0, t0
for t, d in ev:
    occ[cur] += t - last
    cur += d
    last = t
tot = t1 - t0
print("  time with n launches resident: " + ", ".join(f"{n}: {occ[n] / tot * 100:.1f}%" for n in sorted(occ)))
busy = tot - occ[0]
print(f"  device busy (any launch resident) {busy / tot * 100:.1f}%, mean concurrency while busy "
      f"{sum(n * t for n, t in occ.items()) / max(busy, 1):.2f}")
