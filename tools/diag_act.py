import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd"), os.path.join(REPO, "tests")]
from conftest import load_golden
from harness import engine_from_golden, parse
from oracle import spec
import torch
from oracle import nets as N
name = sys.argv[1]
g = load_golden(name)
alg, env, H, B, *_ = parse(g)
S, A, hi = spec.TASKS[env]
eng, rep, tp = engine_from_golden(g)
s, a, *_ = rep.gather(np.arange(B))
data = spec.replay_data(S, A, 4, int(g["meta"][6]) + 1, hi)
print("gather rows equal spec data:", np.abs(s[:4] - data["state"].astype(np.float32)).max(), s[:3, :4])
W = 2 * A if alg == "sac" else A
for n in (B, 32, 1):
    out = eng.act(s[:n], W)
    p = {k: torch.from_numpy(v) for k, v in spec.agent_params(alg, S, A, H, int(g["meta"][6]))["policy"].items()}
    ref = N.mlp(p, torch.from_numpy(s[:n])).numpy() if alg != "td7" else None
    if ref is not None:
        d = np.abs(out - ref)
        print(n, "maxdiff", d.max(), "per-col max", d.max(0)[:40].round(4))
