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


# hidden activations the engine runs (rle_config act_*, include/rle.h RLE_ACT_*), by name
def _act_name(fn) -> str:
    """A SALE `activ` callable (sale.py:25,67,97) or a make_mlp action_fn module (mlp.py:23) -> "relu" /
    "elu" / "identity"; NotImplementedError for anything the engine does not run."""
    if fn in (F.relu, torch.relu) or isinstance(fn, nn.ReLU):
        return "relu"
    if fn is F.elu or (isinstance(fn, nn.ELU) and fn.alpha == 1.0):
        return "elu"
    if isinstance(fn, nn.Identity):
        return "identity"
    raise NotImplementedError(f"activation {getattr(fn, '__name__', fn)!r}: the engine runs ReLU, ELU (alpha 1) "
                              "and Identity")


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


def _mlp(fin: int, fout: int, hidden_sizes, action_fn="ReLU", init_weight=None, init_bias=None):
    """make_mlp (mlp.py:10-35): Linear-act-...-Linear (indices 0, 2, 4, ...); weights by nn.init.<init_weight>
    (default xavier_normal_), biases by nn.init.<init_bias> (default zeros_).  Returns (Sequential, activation
    name).  action_fn=None is refused: make_mlp then pops the output Linear (mlp.py:34), not an activation."""
    if action_fn is None:
        raise NotImplementedError("make_mlp(action_fn=None) drops the output layer (mlp.py:34 pops the last Linear); "
                                  "use action_fn='Identity' for a net without activations")
    act = getattr(nn, action_fn)() if isinstance(action_fn, str) else action_fn
    name = _act_name(act)
    init_w = nn.init.xavier_normal_ if init_weight is None else getattr(nn.init, init_weight)
    init_b = nn.init.zeros_ if init_bias is None else getattr(nn.init, init_bias)
    dims = [fin] + list(hidden_sizes) + [fout]
    mods = []
    for i in range(len(dims) - 1):
        lin = nn.Linear(dims[i], dims[i + 1])
        init_w(lin.weight.data)
        init_b(lin.bias.data)
        mods += [lin, act]
    return nn.Sequential(*mods[:-1]), name


def _sizes(hidden_sizes):
    sizes = [hidden_sizes] * 2 if isinstance(hidden_sizes, int) else list(hidden_sizes)
    if not 2 <= len(sizes) <= 6:  # (make_mlp takes any depth, mlp.py:10-35; the engine builds 2..6, rle.h)
        raise NotImplementedError(f"hidden_sizes {sizes}: the engine builds MLPs of 2 to 6 hidden layers")
    return sizes


class MLPActor(nn.Module):
    """mlp.py:38-72: mean = mlp(s); SAC heads chunk it into (mean, log_std)."""

    def __init__(self, state_dim: int, action_dim: int, hidden_sizes=256, **mlp_kwargs):
        super().__init__()
        self.state_dim, self.action_dim, self.hidden_sizes = state_dim, action_dim, _sizes(hidden_sizes)
        self.mlp, self.act = _mlp(state_dim, action_dim, self.hidden_sizes, **mlp_kwargs)

    def inference_mean(self, state):
        return self.mlp(state)

    def inference_mean_logvar(self, state):
        return self.mlp(state).chunk(2, -1)


class MLPCritic(nn.Module):
    """mlp.py:75-104: q = mlp([s, a])."""

    def __init__(self, state_dim: int, action_dim: int, hidden_sizes=256, **mlp_kwargs):
        super().__init__()
        self.state_dim, self.action_dim, self.hidden_sizes = state_dim, action_dim, _sizes(hidden_sizes)
        self.mlp, self.act = _mlp(state_dim + action_dim, 1, self.hidden_sizes, **mlp_kwargs)

    def estimate_q_value(self, state, action):
        return self.mlp(torch.cat([state, action], -1))


def nets_from_make_nn(alg: str, make_nn, state_dim: int, action_dim: int, kwargs: dict):
    """Call a reference-style make_nn hook (state_dim / action_dim passed as keywords, as
    annotate_make_nn does) and return (hidden width, net shape, {net name: numpy state_dict}, activations) for
    the engine.  Only this module's classes (the reference's default net types) are accepted, with
    one shape across the agent's nets: (hdim, zs_dim) of the SALE nets, hidden_sizes of the MLPs
    (the shape is {"zs_dim": ...} or {"hidden_sizes": [...]}, as rle_config takes them).  The
    activations are make_config's act_actor / act_critic / act_encoder ("relu" / "elu" / "identity"):
    the SALE nets' `activ`, make_mlp's action_fn; the two critics must agree."""
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
    acts = {}
    for name, kind, m in zip(names, kinds, out):
        if type(m) is not kind:
            raise NotImplementedError(f"make_nn returned {type(m).__name__} for {name}; the engine builds "
                                      f"rl.nn.{kind.__name__} nets only")
        role = "act_actor" if name == "policy" else "act_encoder" if name == "encoder" else "act_critic"
        act = _act_name(m.activ) if isinstance(m, (SALEActor, SALECritic, SALEEncoder)) else m.act
        if acts.setdefault(role, act) != act:
            raise NotImplementedError(f"one activation for both critics (got {acts[role]} and {act})")
        if isinstance(m, (SALEActor, SALECritic, SALEEncoder)):
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
        return w[0], {"zs_dim": w[1]}, nets, acts
    return w[-1], {"hidden_sizes": list(w)}, nets, acts
