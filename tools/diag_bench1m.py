"""The 1M-row bench program against the oracle (GPU box, diagnostics): per-parameter agreement after n steps,
step-1 gradients (Adam first moments), and where the elements off by more than 1e-5 sit.
python tools/diag_bench1m.py n [plan]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd"), os.path.join(REPO, "tests")]
from rl import _engine as E  # noqa: E402
from test_engine_gpu import _bench_program_run  # noqa: E402
from oracle import agents  # noqa: E402

n = int(sys.argv[1])
plan = E.parse_plan(sys.argv[2]) if len(sys.argv) > 2 else None
eng, rep, infos, orc, orep, infos_ref, inds, launches, amb = _bench_program_run(n, plan)
print('ambiguous q01 units', {k: sorted(v) for k, v in amb.items()})
print("indices equal", bool((eng.last_indices() == inds[-1]).all()), "launches", launches)
for net, d in orc.nets().items():
    for name, v in d.items():
        got = eng.get_param(net, name, tuple(v.shape)).astype(np.float64)
        dd = np.abs(got - v.detach().numpy().astype(np.float64))
        bad = dd > 1e-5
        line = f"{net:22s} {name:14s} within {1 - bad.mean():.5f} max {dd.max():.2e}"
        if bad.any() and dd.ndim == 2:
            cols = np.argsort(-bad.sum(0))[:6]
            rows = np.argsort(-bad.sum(1))[:4]
            line += f" bad cols {cols.tolist()} ({bad.sum(0)[cols].tolist()}) rows {rows.tolist()} ({bad.sum(1)[rows].tolist()})"
        print(line)
if n == 1:
    for key, ref in agents.moments(orc).items():
        if not key.endswith(":m"):
            continue
        net, pname = key[:-2].split(".", 1)
        g = eng.get_adam(net, pname, 0, ref.shape).astype(np.float64)
        e = np.abs(g - ref) / max(np.abs(ref).max(), 1e-30)
        print(f"m {key:32s} max err / max|g| {e.max():.2e}")
