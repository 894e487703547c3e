"""Diagnostic: per-step engine vs oracle parameter updates (run on the GPU box)."""

import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd"), os.path.join(REPO, "tests")]

from conftest import load_golden  # noqa: E402
from harness import engine_from_golden, parse  # noqa: E402
from oracle import agents  # noqa: E402
from test_oracle import build_from_golden  # noqa: E402

torch.set_num_threads(1)
name = sys.argv[1] if len(sys.argv) > 1 else "td7_tiny"
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
g = load_golden(name)
alg, env, H, B, Ncap, n_fill, n_steps, use_lap, seed, extra = parse(g)
eng, rep, tp = engine_from_golden(g)
_, orc, orep, otp, _, _ = build_from_golden(g)

grads = {}
orig = agents.Adam.step


def rec(self, gs):
    grads[id(self)] = [x.detach().clone() for x in gs]
    return orig(self, gs)


agents.Adam.step = rec
eng.set_tapes(u=tp["u"][:nsteps], eps=tp["eps"][:nsteps], eps_pi=tp.get("eps_pi"))
onets = orc.nets()
for t in range(nsteps):
    before = {n: {k: v.detach().numpy().copy() for k, v in d.items()} for n, d in onets.items()}
    ebefore = {n: {k: eng.get_param(n, k, v.shape) for k, v in d.items()} for n, d in before.items()}
    info_e = eng.step(1)[0]
    i1, _ = agents.run_steps(orc, alg, orep, {k: v[t:t + 1] for k, v in otp.items()}, 1, B)
    print(f"--- step {t} info eng {info_e[:4]} orc {list(i1[0].values())}")
    for n, d in onets.items():
        for k, v in d.items():
            ov = v.detach().numpy()
            ev = eng.get_param(n, k, ov.shape)
            do = ov - before[n][k]
            de = ev - ebefore[n][k]
            if np.abs(do).max() == 0 and np.abs(de).max() == 0:
                continue
            diff = np.abs(ev - ov)
            flips = np.mean(np.sign(do) != np.sign(de))
            print(f"{n}.{k:14s} |dp|max {np.abs(do).max():.2e} diff max {diff.max():.2e} "
                  f"frac>1e-5 {(diff > 1e-5).mean():.3f} signflip {flips:.3f}")
            if flips > 0 and n == "policy":
                gl = grads.get(id(orc.opt_pi))
                if gl is not None:
                    ks = list(d.keys())
                    gv = gl[ks.index(k)].numpy()
                    m = np.sign(do) != np.sign(de)
                    print("    oracle |g| at flips", np.sort(np.abs(gv[m]))[:8], "median |g|", np.median(np.abs(gv)))
    # resync engine to oracle params so each step is checked in isolation
    for n, d in onets.items():
        for k, v in d.items():
            eng.set_param(n, k, v.detach().numpy())
