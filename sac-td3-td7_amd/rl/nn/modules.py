"""Host-side (torch) modules with the reference nets' interface, for ``make_nn`` callables.

A reference user builds custom nets through the agents' ``make_nn`` hook (td7.py:46,56-61,
td3.py:45,53-56, sac.py:39,47-50), typically returning ``SALEActor`` / ``SALECritic`` /
``SALEEncoder`` (rl/nn/sale.py:16-121) or ``MLPActor`` / ``MLPCritic`` (rl/nn/mlp.py:38-104)
with chosen widths.  These classes have the same constructor arguments, state_dict names and
default initialisation (rl/nn/layout.py), and the forward methods the reference's agents call.
The engine agents read the widths and the initial weights off them; training runs on the device.
"""

from __future__ import annotations

import torch
from torch import nn
from torch.nn import functional as F

from rl.nn.layout import SALE_ACTOR, SALE_CRITIC, SALE_ENCODER, _dim


def avg_l1_norm(x: torch.Tensor, eps: float = 1e-8) -> torch.Tensor:
    """sale.py:11-13: x / clamp(mean |x| over the last dim, eps)."""
    return x / x.abs().mean(-1, keepdim=True).clamp(min=eps)


class _Linears(nn.Module):
    """nn.Linear layers named after a layout table (nn.Linear default initialisation)."""

    def __init__(self, table, env):
        super().__init__()
        for name, fin, fout in table:
            self.add_module(name, nn.Linear(_dim(fin, env), _dim(fout, env)))


class SALEEncoder(_Linears):
    """sale.py:16-55: zs = AvgL1Norm(zs3(elu(zs2(elu(zs1(s)))))), zsa = zsa3(elu(zsa2(elu(zsa1([zs, a])))))."""

    def __init__(self, state_dim: int, action_dim: int, zs_dim: int = 256, hdim: int = 256, activ=F.elu):
        super().__init__(SALE_ENCODER, {"S": state_dim, "A": action_dim, "H": hdim, "Z": zs_dim})
        self.state_dim, self.action_dim, self.zs_dim, self.hdim, self.activ = state_dim, action_dim, zs_dim, hdim, activ

    def encode_state(self, state: torch.Tensor) -> torch.Tensor:
        h = self.activ(self.zs2(self.activ(self.zs1(state))))
        return avg_l1_norm(self.zs3(h))

    def encode_state_action(self, zs: torch.Tensor, action: torch.Tensor) -> torch.Tensor:
        h = self.activ(self.zsa1(torch.cat([zs, action], -1)))
        return self.zsa3(self.activ(self.zsa2(h)))


class SALEActor(_Linears):
    """sale.py:58-83: tanh(l3(relu(l2(relu(l1([AvgL1Norm(l0(s)), zs]))))))."""

    def __init__(self, state_dim: int, action_dim: int, zs_dim: int = 256, hdim: int = 256, activ=F.relu):
        super().__init__(SALE_ACTOR, {"S": state_dim, "A": action_dim, "H": hdim, "Z": zs_dim})
        self.state_dim, self.action_dim, self.zs_dim, self.hdim, self.activ = state_dim, action_dim, zs_dim, hdim, activ

    def inference_mean(self, obs: torch.Tensor, zs: torch.Tensor) -> torch.Tensor:
        h = torch.cat([avg_l1_norm(self.l0(obs)), zs], -1)
        h = self.activ(self.l2(self.activ(self.l1(h))))
        return torch.tanh(self.l3(h))


class SALECritic(_Linears):
    """sale.py:86-121: q3(elu(q2(elu(q1([AvgL1Norm(q01([s, a])), zsa, zs])))))."""

    def __init__(self, state_dim: int, action_dim: int, zs_dim: int = 256, hdim: int = 256, activ=F.elu):
        super().__init__(SALE_CRITIC, {"S": state_dim, "A": action_dim, "H": hdim, "Z": zs_dim})
        self.state_dim, self.action_dim, self.zs_dim, self.hdim, self.activ = state_dim, action_dim, zs_dim, hdim, activ

    def estimate_q_value(self, obs, action, zsa, zs) -> torch.Tensor:
        h = torch.cat([avg_l1_norm(self.q01(torch.cat([obs, action], -1))), zsa, zs], -1)
        return self.q3(self.activ(self.q2(self.activ(self.q1(h)))))


def _mlp(fin: int, fout: int, hidden_sizes) -> nn.Sequential:
    """make_mlp (mlp.py:10-35): Linear-ReLU-...-Linear (indices 0, 2, 4, ...), xavier_normal weights,
    zero bias."""
    dims = [fin] + list(hidden_sizes) + [fout]
    mods = []
    for i in range(len(dims) - 1):
        mods += [nn.Linear(dims[i], dims[i + 1]), nn.ReLU()]
    seq = nn.Sequential(*mods[:-1])
    for m in seq:
        if isinstance(m, nn.Linear):
            nn.init.xavier_normal_(m.weight)
            nn.init.zeros_(m.bias)
    return seq


def _sizes(hidden_sizes):
    sizes = [hidden_sizes] * 2 if isinstance(hidden_sizes, int) else list(hidden_sizes)
    if not 2 <= len(sizes) <= 6:  # (make_mlp takes any depth, mlp.py:10-35; the engine builds 2..6, rle.h)
        raise NotImplementedError(f"hidden_sizes {sizes}: the engine builds MLPs of 2 to 6 hidden layers")
    return sizes


class MLPActor(nn.Module):
    """mlp.py:38-72: mean = mlp(s); SAC heads chunk it into (mean, log_std)."""

    def __init__(self, state_dim: int, action_dim: int, hidden_sizes=256, **mlp_kwargs):
        super().__init__()
        if mlp_kwargs:
            raise NotImplementedError(f"make_mlp options {sorted(mlp_kwargs)} (the engine builds ReLU MLPs)")
        self.state_dim, self.action_dim, self.hidden_sizes = state_dim, action_dim, _sizes(hidden_sizes)
        self.mlp = _mlp(state_dim, action_dim, self.hidden_sizes)

    def inference_mean(self, state):
        return self.mlp(state)

    def inference_mean_logvar(self, state):
        return self.mlp(state).chunk(2, -1)


class MLPCritic(nn.Module):
    """mlp.py:75-104: q = mlp([s, a])."""

    def __init__(self, state_dim: int, action_dim: int, hidden_sizes=256, **mlp_kwargs):
        super().__init__()
        if mlp_kwargs:
            raise NotImplementedError(f"make_mlp options {sorted(mlp_kwargs)} (the engine builds ReLU MLPs)")
        self.state_dim, self.action_dim, self.hidden_sizes = state_dim, action_dim, _sizes(hidden_sizes)
        self.mlp = _mlp(state_dim + action_dim, 1, self.hidden_sizes)

    def estimate_q_value(self, state, action):
        return self.mlp(torch.cat([state, action], -1))


def nets_from_make_nn(alg: str, make_nn, state_dim: int, action_dim: int, kwargs: dict):
    """Call a reference-style make_nn hook (state_dim / action_dim passed as keywords, as
    annotate_make_nn does) and return (hidden width, net shape, {net name: numpy state_dict}) for
    the engine.  Only this module's classes (the reference's default net types) are accepted, with
    one shape across the agent's nets: (hdim, zs_dim) of the SALE nets, hidden_sizes of the MLPs
    (the shape is {"zs_dim": ...} or {"hidden_sizes": [...]}, as rle_config takes them)."""
    import numpy as np

    kw = dict(kwargs)
    kw["state_dim"], kw["action_dim"] = state_dim, action_dim
    out = make_nn(**kw)
    names = {"td7": ("policy", "q1", "q2", "encoder"), "td3": ("policy", "q1", "q2"),
             "sac": ("policy", "q1", "q2")}[alg]
    kinds = {"td7": (SALEActor, SALECritic, SALECritic, SALEEncoder),
             "td3": (MLPActor, MLPCritic, MLPCritic), "sac": (MLPActor, MLPCritic, MLPCritic)}[alg]
    if not isinstance(out, (tuple, list)) or len(out) != len(names):
        raise TypeError(f"make_nn must return {len(names)} nets {names}")
    widths = set()
    nets = {}
    for name, kind, m in zip(names, kinds, out):
        if type(m) is not kind:
            raise NotImplementedError(f"make_nn returned {type(m).__name__} for {name}; the engine builds "
                                      f"rl.nn.{kind.__name__} nets only")
        if isinstance(m, (SALEActor, SALECritic, SALEEncoder)):
            want = F.relu if isinstance(m, SALEActor) else F.elu  # (the engine's fixed activations)
            if m.activ is not want:
                raise NotImplementedError(f"{name}: activation {getattr(m.activ, '__name__', m.activ)}, the engine "
                                          f"runs {want.__name__}")
            widths.add((m.hdim, m.zs_dim))
        else:
            widths.add(tuple(m.hidden_sizes))
        want_out = 2 * action_dim if (alg == "sac" and name == "policy") else (action_dim if name == "policy" else None)
        if want_out is not None and getattr(m, "action_dim", want_out) != want_out:
            raise ValueError(f"{name}: output width {m.action_dim}, expected {want_out}")
        nets[name] = {k: v.detach().cpu().numpy().astype(np.float32) for k, v in m.state_dict().items()}
    if len(widths) != 1:
        raise NotImplementedError(f"one net shape across the agent's nets (got {sorted(widths)})")
    w = widths.pop()
    if alg == "td7":
        return w[0], {"zs_dim": w[1]}, nets
    return w[-1], {"hidden_sizes": list(w)}, nets
