"""RLE_AUDIT=1 operand-range audit of every GEMM op of every step graph, and the RLE_HAZARD=1
same-level byte-conflict check of every level (GPU box; builds and captures the graphs, launches
no step).  Usage: python tools/audit.py [audit|hazard|both]"""
import os
import sys

MODE = sys.argv[1] if len(sys.argv) > 1 else "both"
if MODE in ("audit", "both"):
    os.environ["RLE_AUDIT"] = "1"
if MODE in ("hazard", "both"):
    os.environ["RLE_HAZARD"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd")]
from rl import _engine as E  # noqa: E402

TASKS = {"Humanoid-v4": (376, 17), "Ant-v4": (27, 8), "HalfCheetah-v4": (17, 6)}
CASES = [("td7", "Humanoid-v4", 256, True), ("td7", "Humanoid-v4", 1024, True), ("td7", "Ant-v4", 256, True),
         ("sac", "Humanoid-v4", 256, False), ("td3", "HalfCheetah-v4", 256, False), ("td7", "Humanoid-v4", 32, True),
         ("td3", "HalfCheetah-v4", 256, True)]
bad = 0
for algo, env, B, lap in CASES:
    S, A = TASKS[env]
    aid = {"td7": E.RLE_TD7, "td3": E.RLE_TD3, "sac": E.RLE_SAC}[algo]
    try:
        eng = E.Engine(E.make_config(aid, S, A, 256, B, use_lap=lap))
        rep = E.Replay(4096, S, A, lap)
        rep.fill_random(4096, seed=0)
        eng.bind(rep)
        lv = eng.graph_stats()
        for w in range(8):
            try:
                eng.describe(w)
            except RuntimeError as e:
                if "audit" in str(e) or "hazard" in str(e):
                    raise
        print(f"{algo} {env} B={B} lap={lap}: ok ({lv})", flush=True)
    except RuntimeError as e:
        bad += 1
        print(f"{algo} {env} B={B} lap={lap}: {e}", flush=True)
sys.exit(1 if bad else 0)
