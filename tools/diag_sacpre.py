"""Where the fused SAC target pre-GEMM (has_pre 5) and fuse_off sacpre differ (GPU box)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd"), os.path.join(REPO, "tests")]
import numpy as np
from rl import _engine as E
from conftest import load_golden
from harness import engine_from_golden, parse
from oracle import spec

for name in ("sac_tiny", "sac_tiny_fixed", "sac_humanoid"):
    g = load_golden(name)
    for n in (1, 2, 3, 20):
        e1, r1, _ = engine_from_golden(g, plan=E.make_plan(level_cap=100000, pre_tn=16, pl_tn=16))
        i1 = np.array(e1.step(n))
        e2, r2, _ = engine_from_golden(g, plan=E.make_plan(["sacpre"], level_cap=100000, pre_tn=16, pl_tn=16))
        i2 = np.array(e2.step(n))
        d = np.argwhere(~((i1 == i2) | (np.isnan(i1) & np.isnan(i2))))
        alg, env, H = parse(g)[:3]
        pd = []
        for net, params in spec.agent_params(alg, *spec.TASKS[env][:2], H, 0).items():
            for p in params:
                a, b = e1.get_param(net, p), e2.get_param(net, p)
                if not np.array_equal(a, b):
                    pd.append(f"{net}.{p}:{int((a != b).sum())}")
        print(name, n, "info diffs", d.tolist()[:6], [(float(i1[tuple(x)]), float(i2[tuple(x)])) for x in d[:3]], "params", pd[:8], flush=True)
