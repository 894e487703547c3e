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
def find_period(grids, reps=6):
    """(offset, period) of the first window of `reps` identical grid-size sequences (the multi-step
    graph replays, after the warm-up's single-step graphs)."""
    for off in range(0, 400):
        for P in range(10, 200):
            w = grids[off:off + P * reps]
            if len(w) == P * reps and all(w[i] == w[i % P] for i in range(len(w))):
                return off, P
    raise SystemExit("no periodic window")


merged = {}  # level -> {column: mean}
for p, seq in sorted(passes.items()):
    grids = [d["_grid"] for d in seq]
    off, period = find_period(grids)
    agg = defaultdict(lambda: defaultdict(list))
    k = 0
    while off + (k + 1) * period <= len(seq) and grids[off + k * period:off + (k + 1) * period] == grids[off:off + period]:
        for q in range(period):
            for c, v in seq[off + k * period + q].items():
                agg[q][c].append(v)
        k += 1
    for q in range(period):
        row = merged.setdefault(q, {})
        for c, vs in agg[q].items():
            if c == "_ns":
                row.setdefault("us", []).append(sum(vs) / len(vs) / 1000)
            elif c == "_grid":
                row["grid"] = vs[0]
            else:
                row[c] = sum(vs) / len(vs)
DESC = {}
if len(sys.argv) > 2:  # level descriptions (engine describe of the multi-step graph, one "L<k> ..." line each)
    for line in open(sys.argv[2]):
        if line.startswith("L"):
            k, _, rest = line.partition(" ")
            DESC[int(k[1:])] = rest.strip()
import re

MODEL = {}  # level -> {kind: KB} from RLE_TRAFFIC=1 descriptions
for k, d in DESC.items():
    m = re.search(r"\[KB act_r (\d+) act_w (\d+) w_r (\d+) adam (\d+) other (\d+)(?: xcd_r (\d+) adam_w (\d+))?\]", d)
    if m:
        MODEL[k] = dict(zip(("act_r", "act_w", "w_r", "adam", "other", "xcd_r", "adam_w"),
                            (float(x) if x is not None else None for x in m.groups())))
cols = [c for c in ("FETCH_SIZE", "WRITE_SIZE", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY",
                    "SQ_WAVE_CYCLES", "TCC_HIT_sum", "TCC_MISS_sum") if any(c in r for r in merged.values())]
print("per level of the multi-step graph (means over its replays); traffic KB = 2 x FETCH_SIZE + WRITE_SIZE "
      "(gfx950: FETCH_SIZE counts half of a 16-B/lane streaming read)")
print(f"{'lvl':>3} {'grid':>5} {'us':>6} {'trafficKB':>9} " + " ".join(f"{c[:12]:>12}" for c in cols) + "  ops")
tot = defaultdict(float)
for q in sorted(merged):
    r = merged[q]
    us = sum(r.get("us", [0])) / max(1, len(r.get("us", [0])))
    tr = 2 * r.get("FETCH_SIZE", 0) + r.get("WRITE_SIZE", 0)
    tot["us"] += us
    tot["traffic"] += tr
    for c in cols:
        tot[c] += r.get(c, 0)
    print(f"{q:3d} {r.get('grid', 0):5d} {us:6.1f} {tr:9.0f} " + " ".join(f"{r.get(c, 0):12.0f}" for c in cols) +
          "  " + DESC.get(q, "")[:160])
print(f"sum     {tot['us']:6.1f} {tot['traffic']:9.0f} " + " ".join(f"{tot[c]:12.0f}" for c in cols))
if MODEL:
    print("\ntraffic model (RLE_TRAFFIC=1: unique bytes the level's ops must move) against the counters, KB")
    print(f"{'lvl':>3} {'act_r':>7} {'act_w':>7} {'w_r':>7} {'adam':>7} {'other':>7} {'model':>8} {'pmc':>8} {'x':>5}")
    mt = defaultdict(float)
    for q in sorted(merged):
        m = MODEL.get(q)
        if not m:
            continue
        r = merged[q]
        tr = 2 * r.get("FETCH_SIZE", 0) + r.get("WRITE_SIZE", 0)
        tot_m = sum(m[kk] for kk in ("act_r", "act_w", "w_r", "adam", "other"))
        for kk, vv in m.items():
            mt[kk] += vv or 0.0
        mt["pmc"] += tr
        print(f"{q:3d} " + " ".join(f"{m[kk]:7.0f}" for kk in ("act_r", "act_w", "w_r", "adam", "other")) +
              f" {tot_m:8.0f} {tr:8.0f} {tr / max(tot_m, 1):5.2f}")
    tm = sum(mt[kk] for kk in ("act_r", "act_w", "w_r", "adam", "other"))
    print("sum " + " ".join(f"{mt[kk]:7.0f}" for kk in ("act_r", "act_w", "w_r", "adam", "other")) +
          f" {tm:8.0f} {mt['pmc']:8.0f} {mt['pmc'] / max(tm, 1):5.2f}")
    if all(m.get("xcd_r") is not None for m in MODEL.values()):
        # per-XCD model: every XCD's L2 fetches its own copy of what its workgroups read (engine.cpp LevelTraffic)
        # + the unique bytes stored (activations, Adam's stores) + the sampler / priority / reductions' bytes
        print("\nper-XCD read model against the counters, KB: reads (2 x FETCH_SIZE) and stores (WRITE_SIZE) apart")
        print(f"{'lvl':>3} {'xcd_r':>8} {'2xFETCH':>8} {'x':>5} {'stores':>8} {'WRITE':>8} {'x':>5} {'model':>8} {'pmc':>8} {'cover':>6}")
        xt = defaultdict(float)
        for q in sorted(merged):
            m = MODEL.get(q)
            if not m:
                continue
            r = merged[q]
            rd, wr = 2 * r.get("FETCH_SIZE", 0), r.get("WRITE_SIZE", 0)
            mr, mw = m["xcd_r"] + m["other"], m["act_w"] + m["adam_w"]
            for kk, vv in (("mr", mr), ("mw", mw), ("rd", rd), ("wr", wr)):
                xt[kk] += vv
            print(f"{q:3d} {mr:8.0f} {rd:8.0f} {rd / max(mr, 1):5.2f} {mw:8.0f} {wr:8.0f} {wr / max(mw, 1):5.2f} "
                  f"{mr + mw:8.0f} {rd + wr:8.0f} {(mr + mw) / max(rd + wr, 1):6.2f}")
        print(f"sum {xt['mr']:8.0f} {xt['rd']:8.0f} {xt['rd'] / max(xt['mr'], 1):5.2f} {xt['mw']:8.0f} {xt['wr']:8.0f} "
              f"{xt['wr'] / max(xt['mw'], 1):5.2f} {xt['mr'] + xt['mw']:8.0f} {xt['rd'] + xt['wr']:8.0f} "
              f"{(xt['mr'] + xt['mw']) / max(xt['rd'] + xt['wr'], 1):6.2f}")
