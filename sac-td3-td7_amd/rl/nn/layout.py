"""Parameter layouts of the reference nets and their default initialisation.

Names/shapes follow the reference modules' state_dicts: ``SALEEncoder`` /
``SALEActor`` / ``SALECritic`` (rl/nn/sale.py:16-121) and ``make_mlp`` nets
(rl/nn/mlp.py:10-104, nn.Sequential indices 0/2/4).  Initialisation follows
torch: nn.Linear default (kaiming_uniform(a=sqrt(5)) => U(+-1/sqrt(fan_in)) for
weight and bias) for SALE nets; xavier_normal weights + zero bias for make_mlp
(mlp.py:19-31).
"""

from __future__ import annotations

import math

import numpy as np

SALE_ENCODER = (("zs1", "S", "H"), ("zs2", "H", "H"), ("zs3", "H", "Z"),
                ("zsa1", "Z+A", "H"), ("zsa2", "H", "H"), ("zsa3", "H", "Z"))
SALE_ACTOR = (("l0", "S", "H"), ("l1", "Z+H", "H"), ("l2", "H", "H"), ("l3", "H", "A"))
SALE_CRITIC = (("q01", "S+A", "H"), ("q1", "2*Z+H", "H"), ("q2", "H", "H"), ("q3", "H", "1"))


def _dim(expr, env):
    return int(eval(expr, {}, env))  # tiny closed vocabulary: S, A, H, Z, IN, OUT


def layers(kind: str, S: int, A: int, H: int, out: int | None = None, hidden_sizes=None, zs_dim=None):
    """[(prefix, in_features, out_features)] of one net kind.  SALE nets: hdim H, zs_dim (default H,
    sale.py:19-26); make_mlp nets: hidden_sizes (default [H, H], mlp.py:45-47), Linear layers at
    nn.Sequential indices 0, 2, 4, ... (mlp.py:24-35)."""
    env = {"S": S, "A": A, "H": H, "Z": H if zs_dim is None else zs_dim}
    table = {"sale_encoder": SALE_ENCODER, "sale_actor": SALE_ACTOR, "sale_critic": SALE_CRITIC}
    if kind in table:
        return [(p, _dim(i, env), _dim(o, env)) for p, i, o in table[kind]]
    if kind == "mlp_actor":
        dims = [S, out if out is not None else A]
    elif kind == "mlp_critic":
        dims = [S + A, 1]
    else:
        raise ValueError(kind)
    dims[1:1] = [H, H] if hidden_sizes is None else list(hidden_sizes)
    return [(f"mlp.{2 * i}", dims[i], dims[i + 1]) for i in range(len(dims) - 1)]


def init_params(kind: str, S: int, A: int, H: int, rng: np.random.Generator, out: int | None = None, **shape):
    """state_dict-shaped numpy params with the reference's default initialisation."""
    params = {}
    for prefix, fin, fout in layers(kind, S, A, H, out, **shape):
        if kind.startswith("mlp"):
            std = math.sqrt(2.0 / (fin + fout))  # xavier_normal_, gain 1
            params[prefix + ".weight"] = (rng.standard_normal((fout, fin)) * std).astype(np.float32)
            params[prefix + ".bias"] = np.zeros(fout, np.float32)
        else:
            k = 1.0 / math.sqrt(fin)
            params[prefix + ".weight"] = rng.uniform(-k, k, (fout, fin)).astype(np.float32)
            params[prefix + ".bias"] = rng.uniform(-k, k, fout).astype(np.float32)
    return params


# net name -> kind, per algorithm (attribute names of the reference agents)
AGENT_NETS = {
    "td7": {"encoder": "sale_encoder", "policy": "sale_actor", "q1": "sale_critic", "q2": "sale_critic"},
    "td3": {"policy": "mlp_actor", "q1": "mlp_critic", "q2": "mlp_critic"},
    "sac": {"policy": "mlp_actor", "q1": "mlp_critic", "q2": "mlp_critic"},
}
# deep copies made at construction (td7.py:62-66, td3.py:57-58, sac.py:52)
AGENT_COPIES = {
    "td7": {"target_q1": "q1", "target_q2": "q2", "fixed_encoder": "encoder",
            "fixed_encoder_target": "encoder"},
    "td3": {"target_q1": "q1", "target_q2": "q2"},
    "sac": {"target_q1": "q1", "target_q2": "q2"},
}


def init_agent(alg: str, S: int, A: int, H: int, seed: int, **shape):
    """All nets of a freshly constructed agent: copies equal their sources (shape: hidden_sizes /
    zs_dim, as layers())."""
    rng = np.random.default_rng(seed)
    nets = {}
    for name, kind in AGENT_NETS[alg].items():
        out = 2 * A if (alg == "sac" and name == "policy") else None
        nets[name] = init_params(kind, S, A, H, rng, out, **shape)
    for name, src in AGENT_COPIES[alg].items():
        nets[name] = {k: v.copy() for k, v in nets[src].items()}
    return nets
