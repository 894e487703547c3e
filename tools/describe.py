"""Print the level structure of the step graphs (GPU box): python tools/describe.py [td7|td3|sac] [S A]
(RLE_DESC_B=1024: batch; RLE_DESC_CRIT=1 stars the ops on a longest dependency chain; RLE_DESC_ONLY=3 prints the multi-step graph
alone, as tools/pmc_levels.py takes it; RLE_TRAFFIC=1 adds each level's traffic model)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd")]
from rl import _engine as E
from rl.nn.layout import init_agent
S, A, H, B = 376, 17, 256, int(os.environ.get("RLE_DESC_B", "256"))  # (RLE_DESC_B: another batch)
algo = sys.argv[1] if len(sys.argv) > 1 else "td7"
code = {"td7": E.RLE_TD7, "td3": E.RLE_TD3, "sac": E.RLE_SAC}[algo]
if algo == "td3":
    S, A = 17, 6
if len(sys.argv) > 3:
    S, A = int(sys.argv[2]), int(sys.argv[3])
eng = E.Engine(E.make_config(code, S, A, H, B, use_lap=(algo == "td7")))
for net, params in init_agent(algo, S, A, H, 1).items():
    for k, v in params.items():
        eng.set_param(net, k, v)
rep = E.Replay(1000000, S, A, algo == "td7")
rep.fill_random(1000000, 1)
eng.bind(rep)
only = os.environ.get("RLE_DESC_ONLY")
for w in ((int(only),) if only else (0, 1, 3)):
    if not only:
        print(f"=== graph {w}")
    print(eng.describe(w))
