"""Per-parameter agreement with the oracle after a short burst (GPU box, diagnostics):
python tools/diag_wide.py alg env H B n [plan]   -> one line per parameter: fraction within 1e-5, max |d|."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd"), os.path.join(REPO, "tests")]
from rl import _engine as E  # noqa: E402
from test_engine_gpu import _synthetic_golden  # noqa: E402
from harness import engine_from_golden  # noqa: E402
from test_oracle import build_from_golden  # noqa: E402
from oracle import agents  # noqa: E402

alg, env, H, B, n = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
plan = E.parse_plan(sys.argv[6]) if len(sys.argv) > 6 else None
ncap = 8192 if B > 256 else 4096
g = _synthetic_golden(alg, env, H, B, ncap, ncap, n, alg == "td7", 91)
_, orc, orep, tp, n_steps, B = build_from_golden(g)
eng, rep, tp2 = engine_from_golden(g, plan=plan)
for t in range(n_steps):
    agents.run_steps(orc, alg, orep, {k: v[t:t + 1] for k, v in tp.items()}, 1, B)
eng.set_tapes(u=tp2["u"][:n_steps], eps=tp2["eps"][:n_steps], eps_pi=tp2.get("eps_pi", None))
eng.step(n_steps)
for net, d in orc.nets().items():
    for name, v in d.items():
        got = eng.get_param(net, name, tuple(v.shape))
        dd = np.abs(got.astype(np.float64) - v.detach().numpy().astype(np.float64))
        print(f"{net:22s} {name:16s} within1e-5 {np.mean(dd <= 1e-5):.5f} max {dd.max():.3e}")
# gradients (Adam first moments) against the oracle's: error scaled by the tensor's max |m|, and where it sits
mo = agents.moments(orc)
for key, ref in mo.items():
    if not key.endswith(":m") or key.startswith("tmp."):
        continue
    net, pname = key[:-2].split(".", 1)
    got = eng.get_adam(net, pname, 0, ref.shape).astype(np.float64)
    r = ref.astype(np.float64)
    e = np.abs(got - r) / max(np.abs(r).max(), 1e-30)
    line = f"m {key:30s} max rel-to-max {e.max():.3e}"
    if e.ndim == 2 and e.max() > 1e-4:
        rows = np.argsort(-e.max(1))[:6]
        cols = np.argsort(-e.max(0))[:6]
        line += f" worst rows {rows.tolist()} ({e.max(1)[rows].round(5).tolist()}) cols {cols.tolist()}"
    print(line)
