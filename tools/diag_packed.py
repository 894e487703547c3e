"""Packed group vs engines alone (TD3 HalfCheetah, default planner): per-parameter fraction of
elements within 1e-5 after n steps, for the current environment (GPU box; diagnostics)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd"), os.path.join(REPO, "tests")]
from conftest import load_golden  # noqa: E402
from harness import engine_from_golden, parse  # noqa: E402
from oracle import spec  # noqa: E402
from rl import _engine as E  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "td3_halfcheetah"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
g = dict(load_golden(name))
alg, env, H = parse(g)[:3]


def make():
    out = []
    for k in range(3):
        e, r, _ = engine_from_golden(g)
        for net, params in spec.agent_params(alg, *spec.TASKS[env][:2], H, 0).items():
            for p in params:
                e.set_param(net, p, e.get_param(net, p) * np.float32(1.0 - 0.05 * k))
        out.append((e, r))
    return out


alone = make()
packed = make()
grp = E.EngineGroup([e for e, _ in packed])
for e, _ in alone:
    e.step(n)
grp.step(n)
grp.close()
worst = []
for (e1, _), (e2, _) in zip(alone, packed):
    for net, params in spec.agent_params(alg, *spec.TASKS[env][:2], H, 0).items():
        for p in params:
            d = np.abs(e1.get_param(net, p).astype(np.float64) - e2.get_param(net, p))
            worst.append(((d <= 1e-5).mean(), f"{net}.{p}"))
worst.sort()
print(os.environ.get("DIAG_TAG", "-"), [(round(f, 4), w) for f, w in worst[:4]])
