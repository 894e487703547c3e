"""Per-level phase timing of the TD7 Humanoid step from in-kernel timestamps (GPU box).

RLE_TRACE=1 python tools/trace_levels.py [steps]
Phases per workgroup (s_memrealtime, 10 ns ticks): dispatch delay (entry - level's first
entry), prologue (entry -> main loop), main loop, epilogue (-> exit); the level span is
first entry -> last exit.
"""
import os
import re
import sys

import numpy as np

os.environ.setdefault("RLE_TRACE", "1")
os.environ.setdefault("RLE_DESC_WG", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd")]
from rl import _engine as E  # noqa: E402
from rl.nn.layout import init_agent  # noqa: E402

# RLE_TRACE_ALGO=td3 / sac: the secondary configs (TD3 HalfCheetah, SAC Humanoid; uniform replay)
ALGO = os.environ.get("RLE_TRACE_ALGO", "td7")
S, A, H, B = (17, 6, 256, 256) if ALGO == "td3" else (376, 17, 256, 256)
B = int(os.environ.get("RLE_TRACE_BATCH", B))  # (BASELINE config 4: 1024)
LAP = ALGO == "td7"
eng = E.Engine(E.make_config({"td7": E.RLE_TD7, "td3": E.RLE_TD3, "sac": E.RLE_SAC}[ALGO], S, A, H, B, use_lap=LAP),
               E.parse_plan(os.environ.get("RLE_PLAN", "")))  # (RLE_PLAN: the plan to trace, bench.py --plan syntax)
for net, params in init_agent(ALGO, S, A, H, 1).items():
    for k, v in params.items():
        eng.set_param(net, k, v)
rep = E.Replay(1000000, S, A, LAP)
rep.fill_random(1000000, 1)
eng.bind(rep)
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
eng.step_timed(steps)
graphs = [int(w) for w in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 3]
JSON = sys.argv[3] if len(sys.argv) > 3 else None  # per-op-kind spans (bench.py reads the sampler's)
opspans = {}
for which in graphs:
    tr = eng.trace(which).astype(np.int64)
    if which == 3 and tr.size and not tr.any():
        # (rle_graph_trace(3) reads the multi-step graph of the last single policy step's batch set;
        # SAC's trailing singles can leave it on the set whose multi-step graph did not run: one
        # more single step flips it)
        eng.step_timed(1)
        tr = eng.trace(which).astype(np.int64)
    if tr.size == 0:
        continue
    tot_t = 0.0
    desc = [l for l in eng.describe(which).splitlines() if l.startswith("L")]
    print(f"=== graph {which}")
    off = 0
    prev_end = None
    for line in desc:
        nwg = int(line.split("wg=")[1].split(":")[0])
        t = tr[off:off + nwg]
        off += nwg
        t0 = t[:, 0].min()
        span = (t[:, 3].max() - t0) * 10 / 1000
        gap = (t0 - prev_end) * 10 / 1000 if prev_end is not None else 0.0
        prev_end = t[:, 3].max()
        tot_t += gap + span
        disp = (t[:, 0] - t0) * 10 / 1000
        g = t[:, 1] > 0
        pro = ((t[g, 1] - t[g, 0]) * 10 / 1000) if g.any() else np.zeros(1)
        loop = ((t[g, 2] - t[g, 1]) * 10 / 1000) if g.any() else np.zeros(1)
        epi = ((t[g, 3] - t[g, 2]) * 10 / 1000) if g.any() else np.zeros(1)
        tot = (t[:, 3] - t[:, 0]) * 10 / 1000
        print(f"gap {gap:5.2f} span {span:6.2f} | disp max {disp.max():5.2f} | wg med {np.median(tot):5.2f} max {tot.max():5.2f}"
              f" | pro {np.median(pro):5.2f} loop {np.median(loop):5.2f} epi {np.median(epi):5.2f} | {line[:90]}")
        if JSON:  # every op's span (first entry -> last exit), all levels
            o = 0
            for name, w in re.findall(r"([a-z]+(?:\[[^\]]*\])?)/(\d+)", line.split(":", 1)[1]):
                tt = t[o:o + int(w)]
                o += int(w)
                opspans.setdefault(name.split("[")[0] + "_all", []).append(float((tt[:, 3].max() - tt[:, 0].min()) * 10 / 1000))
        if os.environ.get("RLE_DESC_WG") and span > 6.0:  # per-op longest workgroup
            o = 0
            parts = []
            for name, w in re.findall(r"([a-z]+(?:\[[^\]]*\])?)/(\d+)", line.split(":", 1)[1]):
                w = int(w)
                tt = t[o:o + w]
                o += w
                parts.append(f"{name.replace(' ', '_')}:{(tt[:, 3] - tt[:, 0]).max() * 10 / 1000:.1f}"
                             f"@{(tt[:, 0].min() - t0) * 10 / 1000:.1f}")
            print("      ops: " + " ".join(parts))
            if os.environ.get("RLE_TRACE_OPS"):  # per-op phase medians / maxima (us)
                o = 0
                for name, w in re.findall(r"([a-z]+(?:\[[^\]]*\])?)/(\d+)", line.split(":", 1)[1]):
                    w = int(w)
                    tt = t[o:o + w]
                    o += w
                    ph = lambda a, b: (tt[:, b] - tt[:, a]) * 10 / 1000
                    f = lambda x: f"{np.median(x):4.1f}/{x.max():4.1f}"
                    extra = ""
                    if tr.shape[1] == 16 and "gemm" in name and (tt[:, 11] > 0).all() and (tt[:, 12] > 0).all():
                        extra = (f" [dec {f(ph(0, 11))} desc {f(ph(11, 12))} pf {f(ph(12, 1))}"
                                 f" splitK {f(ph(2, 13))} epi {f(ph(13, 3))}]")
                        if "adam" in name and (tt[:, 4] > 0).all() and (tt[:, 5] > 0).all():  # DW: AvgL1Norm tables
                            extra += f" [ring {f(ph(1, 4))} tables {f(ph(4, 5))} run {f(ph(5, 2))}]"
                        if (tt[:, 4] > 0).all() and (tt[:, 6] > 0).all():  # pre-GEMM consumer phases
                            extra += (f" [pre issue {f(ph(1, 4))} segs {f(ph(4, 5))} finish {f(ph(5, 6))}"
                                      f" lds {f(ph(6, 2))}]")
                    if tr.shape[1] == 16 and name == "sgather" and (tt[:, 10] > 0).all():  # sampler marks
                        extra = (f" [ctrl {f(ph(0, 4))} sums+u {f(ph(4, 5))} blocks {f(ph(5, 6))} sub {f(ph(6, 7))}"
                                 f" elems {f(ph(7, 2))} gather {f(ph(2, 10))} tail {f(ph(10, 3))}]")
                    if tr.shape[1] == 16 and name == "end" and (tt[:, 8] > 0).all():  # op_step_end marks
                        extra = (f" [loads {f(ph(0, 4))} sums {f(ph(4, 5))} sync {f(ph(5, 6))} reduce {f(ph(6, 7))}"
                                 f" info {f(ph(7, 8))} tail {f(ph(8, 3))}]")
                    print(f"        {name.replace(' ', '_'):32s} start {f((tt[:, 0] - t0) * 10 / 1000)} pro {f(ph(0, 1))}"
                          f" loop {f(ph(1, 2))} epi {f(ph(2, 3))}{extra}")
        if tr.shape[1] == 16 and line.rstrip().endswith("head/64"):  # fine build: loss head phases
            med = lambda a, b: np.median((t[:, b] - t[:, a]) * 10 / 1000)
            print(f"      head: issue {med(0, 4):5.2f} loads+q {med(4, 5):5.2f} target {med(5, 1):5.2f}"
                  f" | loss {med(1, 6):5.2f} prio {med(6, 7):5.2f} | dz {med(2, 8):5.2f} sync {med(8, 9):5.2f}"
                  f" tail {med(9, 3):5.2f}")
        if tr.shape[1] == 16 and "gemm" in line:  # fine build: GEMM prologue / epilogue split
            gm = g & (t[:, 11] > 0) & (t[:, 12] > 0)
            if gm.any():
                med = lambda a, b: np.median((t[gm, b] - t[gm, a]) * 10 / 1000)
                if (t[gm, 14] > 0).all():  # gemm_v entry stamp: switch -> variant, variant entry -> hot batch done
                    print(f"      gemm: to-variant {med(11, 14):5.2f} hot {med(14, 12):5.2f}")
                print(f"      gemm: decode {med(0, 11):5.2f} desc {med(11, 12):5.2f} prefetch {med(12, 1):5.2f}"
                      f" | loop {med(1, 2):5.2f} | splitK {med(2, 13):5.2f} epi {med(13, 3):5.2f}")
    print(f"total (gaps + spans) {tot_t:7.2f} us over {len(desc)} levels")
if JSON:
    import json

    out = {k: {"n": len(v), "mean_us": float(np.mean(v)), "max_us": float(np.max(v))} for k, v in sorted(opspans.items())}
    out["_note"] = "op spans (first workgroup entry -> last exit, us) from RLE_TRACE in-kernel stamps, graphs " + str(graphs)
    json.dump(out, open(JSON, "w"), indent=1)
