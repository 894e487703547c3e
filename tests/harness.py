"""Drive the HIP engine in parity mode from a golden fixture (test infrastructure)."""

from __future__ import annotations

import numpy as np

from conftest import acts_of, shape_of  # noqa: F401  (re-exported for the tests)
from oracle import spec
from rl import _engine as E

ALGO = {"td7": E.RLE_TD7, "td3": E.RLE_TD3, "sac": E.RLE_SAC}
# Per-step losses / info columns against the reference or the oracle (rel 1e-3 for <= 10-step losses)
LOSS_RTOL = 1e-3


def parse(g):
    alg = str(g["meta_alg"])
    env = str(g["meta_env"])
    H, B, Ncap, n_fill, n_steps, use_lap, seed = (int(x) for x in g["meta"])
    extra = dict(zip([str(k) for k in g["meta_extra_keys"]], g["meta_extra_vals"].tolist()))
    return alg, env, H, B, Ncap, n_fill, n_steps, bool(use_lap), seed, extra


def fill_replay(rep, S, A, hi, n_fill, seed):
    data = spec.replay_data(S, A, n_fill, seed + 1, hi)
    scale = np.full(A, hi, np.float32)
    scale = (scale - (-scale)) / 2.0  # get_action_bias_scale (miscellaneous.py:59-66)
    bias = np.zeros(A, np.float32)
    act = (np.asarray(data["action"]) / scale - bias).astype(np.float32)  # lap.py:35 (Q5)
    rep.append(data["state"].astype(np.float32), act, data["reward"].astype(np.float32),
               data["next_state"].astype(np.float32), data["done"].astype(np.float32))


def engine_from_golden(g, device=0, plan=None):
    alg, env, H, B, Ncap, n_fill, n_steps, use_lap, seed, extra = parse(g)
    S, A, hi = spec.TASKS[env]
    kw = {}
    # the reference's constructor arguments (td7.py:34-43, td3.py:33-43, sac.py:27-37) -> rle_config fields
    for k, v in extra.items():
        if k in ("target_update_rate", "policy_freq"):
            kw[k] = int(v)
        elif k == "discount_factor":
            kw["discount"] = float(v)
        elif k in ("tmp", "policy_lr", "critic_lr", "tau", "target_policy_noise", "noise_clip", "min_log_std",
                   "max_log_std"):  # (tmp: SAC fixed temperature, sac.py:55-60)
            kw[k] = float(v)
        else:
            raise KeyError(f"golden hyper-parameter {k} has no rle_config field")
    shape = shape_of(g)
    acts = {f"act_{k}": v for k, v in acts_of(g).items()}  # (hidden activations beyond the defaults)
    cfg = E.make_config(ALGO[alg], S, A, H, B, use_lap=use_lap, seed=seed, device=device, **kw, **shape, **acts)
    eng = E.Engine(cfg, plan)
    for net, params in spec.agent_params(alg, S, A, H, seed, **shape).items():
        for name, v in params.items():
            eng.set_param(net, name, v)
    rep = E.Replay(Ncap, S, A, use_lap, device)
    fill_replay(rep, S, A, hi, n_fill, seed)
    if use_lap:
        p0 = spec.init_priorities(Ncap, seed + 2)
        p0[n_fill:] = 0.0
        rep.set_priority(p0, float(p0.max()))
    eng.bind(rep)
    tp = {k[5:]: v for k, v in g.items() if k.startswith("tape_")}
    return eng, rep, tp


def run_with_tapes(eng, tp, n_steps, per_step=None):
    eng.set_tapes(u=tp["u"][:n_steps], eps=tp["eps"][:n_steps],
                  eps_pi=tp.get("eps_pi", None) if "eps_pi" in tp else None)
    infos = []
    for t in range(n_steps):
        infos.append(eng.step(1)[0])
        if per_step:
            per_step(t)
    eng.set_tapes()
    return np.array(infos)
