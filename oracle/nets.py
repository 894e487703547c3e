"""Functional restatement of the reference nets (TEST INFRASTRUCTURE ONLY).

Params are plain dicts ``name -> torch.Tensor`` keyed like the reference
modules' state_dicts (see ``oracle/spec.py``).
"""

from __future__ import annotations

import torch
import torch.nn.functional as F


def _lin(x, p, name):
    return F.linear(x, p[name + ".weight"], p[name + ".bias"])


def _identity(x):
    return x


# hidden activations by name: SALE nets' `activ` (sale.py:25,67,97) and make_mlp's action_fn (mlp.py:13,23:
# "ReLU" / "ELU" / "Identity"); ELU with alpha 1 as nn.ELU() / F.elu default
ACTS = {"relu": F.relu, "elu": F.elu, "identity": _identity}


def avg_l1_norm(x, eps: float = 1e-8):
    """rl/nn/sale.py:11-13: x / clamp(mean|x|, eps) row-wise."""
    return x / x.abs().mean(-1, keepdim=True).clamp(min=eps)


# --- TD7 SALE nets (rl/nn/sale.py) -------------------------------------------

def sale_zs(p, s, act=F.elu):
    """SALEEncoder.encode_state (sale.py:41-46)."""
    h = act(_lin(s, p, "zs1"))
    h = act(_lin(h, p, "zs2"))
    return avg_l1_norm(_lin(h, p, "zs3"))


def sale_zsa(p, zs, a, act=F.elu):
    """SALEEncoder.encode_state_action (sale.py:48-55)."""
    h = act(_lin(torch.cat([zs, a], 1), p, "zsa1"))
    h = act(_lin(h, p, "zsa2"))
    return _lin(h, p, "zsa3")


def sale_actor(p, s, zs, act=F.relu):
    """SALEActor.inference_mean (sale.py:77-83)."""
    h = torch.cat([avg_l1_norm(_lin(s, p, "l0")), zs], 1)
    h = act(_lin(h, p, "l1"))
    h = act(_lin(h, p, "l2"))
    return torch.tanh(_lin(h, p, "l3"))


def sale_critic(p, s, a, zsa, zs, act=F.elu):
    """SALECritic.estimate_q_value (sale.py:106-121)."""
    x = avg_l1_norm(_lin(torch.cat([s, a], 1), p, "q01"))
    h = torch.cat([x, torch.cat([zsa, zs], 1)], 1)
    h = act(_lin(h, p, "q1"))
    h = act(_lin(h, p, "q2"))
    return _lin(h, p, "q3")


# --- MLP nets (rl/nn/mlp.py) -------------------------------------------------

def mlp(p, x, act=F.relu):
    """make_mlp: Linear-act-...-Linear at nn.Sequential indices 0, 2, 4, ... (mlp.py:10-35)."""
    w = sorted((k for k in p if k.startswith("mlp.") and k.endswith(".weight")), key=lambda k: int(k.split(".")[1]))
    h = x
    for i, k in enumerate(w):
        h = _lin(h, p, k[: -len(".weight")])
        if i + 1 < len(w):
            h = act(h)
    return h


def mlp_critic(p, s, a, act=F.relu):
    """MLPCritic.estimate_q_value (mlp.py:98-101)."""
    return mlp(p, torch.cat([s, a], -1), act)


EPS = 1e-6  # rl/utils/annotation.py:12


def gaussian_tanh(mean, log_std, eps, min_log_std=-20.0, max_log_std=2.0):
    """SAC._inference + _rsample (sac.py:154-172) with an explicit noise tensor.

    Normal(loc, scale).rsample = loc + eps*scale; log_prob follows
    torch.distributions.Normal.log_prob literally.
    """
    import math

    log_std = torch.clamp(log_std, min_log_std, max_log_std)
    scale = log_std.exp()
    u = mean + eps * scale
    a = torch.tanh(u)
    var = scale ** 2
    lp = -((u - mean) ** 2) / (2 * var) - scale.log() - math.log(math.sqrt(2 * math.pi))
    log_pi = lp.sum(-1, keepdim=True)
    log_pi = log_pi - torch.log(1 - a.pow(2.0) + EPS).sum(-1, keepdim=True)
    return a, log_pi
