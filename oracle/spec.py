"""Parameter specs and deterministic weights — shared by the fixture generator,
the oracle, the tests and the bench.

Parameter names/orders follow the reference modules' ``named_parameters()``:
``SALEEncoder``/``SALEActor``/``SALECritic`` (``rl/nn/sale.py:16-121``) and
``MLPActor``/``MLPCritic`` built by ``make_mlp`` (``rl/nn/mlp.py:10-104``,
``nn.Sequential`` indices 0, 2, 4).
"""

from __future__ import annotations

import math

import numpy as np

# env_id -> (obs_dim, act_dim, action high bound); MuJoCo-v4 spaces as returned
# by get_state_action_dims / get_action_bias_scale (rl/utils/miscellaneous.py:50-66).
TASKS = {
    "Humanoid-v4": (376, 17, 0.4),
    "Ant-v4": (27, 8, 1.0),
    "HalfCheetah-v4": (17, 6, 1.0),
    "Hopper-v4": (11, 3, 1.0),
    "Walker2d-v4": (17, 6, 1.0),
    "Tiny-v0": (11, 3, 0.5),
}


def sale_encoder_spec(S, A, Z=256, H=256):
    """rl/nn/sale.py:16-38."""
    return [
        ("zs1.weight", (H, S)), ("zs1.bias", (H,)),
        ("zs2.weight", (H, H)), ("zs2.bias", (H,)),
        ("zs3.weight", (Z, H)), ("zs3.bias", (Z,)),
        ("zsa1.weight", (H, Z + A)), ("zsa1.bias", (H,)),
        ("zsa2.weight", (H, H)), ("zsa2.bias", (H,)),
        ("zsa3.weight", (Z, H)), ("zsa3.bias", (Z,)),
    ]


def sale_actor_spec(S, A, Z=256, H=256):
    """rl/nn/sale.py:58-75."""
    return [
        ("l0.weight", (H, S)), ("l0.bias", (H,)),
        ("l1.weight", (H, Z + H)), ("l1.bias", (H,)),
        ("l2.weight", (H, H)), ("l2.bias", (H,)),
        ("l3.weight", (A, H)), ("l3.bias", (A,)),
    ]


def sale_critic_spec(S, A, Z=256, H=256):
    """rl/nn/sale.py:86-103."""
    return [
        ("q01.weight", (H, S + A)), ("q01.bias", (H,)),
        ("q1.weight", (H, 2 * Z + H)), ("q1.bias", (H,)),
        ("q2.weight", (H, H)), ("q2.bias", (H,)),
        ("q3.weight", (1, H)), ("q3.bias", (1,)),
    ]


def mlp_spec(inp, out, H=256):
    """make_mlp (rl/nn/mlp.py:10-35): hidden_sizes H (an int: [H, H], mlp.py:45-47); Linear layers at
    nn.Sequential indices 0, 2, 4, ... (a ReLU after each but the last)."""
    hs = [H, H] if isinstance(H, int) else list(H)
    dims = [inp] + hs + [out]
    out_spec = []
    for i in range(len(dims) - 1):
        out_spec += [(f"mlp.{2 * i}.weight", (dims[i + 1], dims[i])), (f"mlp.{2 * i}.bias", (dims[i + 1],))]
    return out_spec


def agent_specs(alg: str, S: int, A: int, H: int = 256, hidden_sizes=None, zs_dim=None) -> dict:
    """Net name -> param spec for the trainable nets of one agent.  TD7: hdim H, zs_dim (default H,
    sale.py:19-26); TD3 / SAC: make_mlp's hidden_sizes (default [H, H])."""
    if alg == "td7":
        Z = H if zs_dim is None else zs_dim
        return {
            "encoder": sale_encoder_spec(S, A, Z, H),
            "policy": sale_actor_spec(S, A, Z, H),
            "q1": sale_critic_spec(S, A, Z, H),
            "q2": sale_critic_spec(S, A, Z, H),
        }
    hs = [H, H] if hidden_sizes is None else list(hidden_sizes)
    if alg == "td3":
        return {
            "policy": mlp_spec(S, A, hs),
            "q1": mlp_spec(S + A, 1, hs),
            "q2": mlp_spec(S + A, 1, hs),
        }
    if alg == "sac":
        return {
            "policy": mlp_spec(S, 2 * A, hs),
            "q1": mlp_spec(S + A, 1, hs),
            "q2": mlp_spec(S + A, 1, hs),
        }
    raise ValueError(alg)


# Extra (non-trainable-copy) nets that are deep copies in the reference and
# therefore get their own deterministic weights in the fixtures so that hard /
# Polyak updates are observable: name -> source spec name.
COPY_NETS = {
    "td7": {"target_q1": "q1", "target_q2": "q2",
            "fixed_encoder": "encoder", "fixed_encoder_target": "encoder"},
    "td3": {"target_q1": "q1", "target_q2": "q2"},
    "sac": {"target_q1": "q1", "target_q2": "q2"},
}


def gen_params(spec, seed: int, scale: float = 1.0) -> dict:
    """Deterministic fp32 params ~ U(-k, k), k = scale/sqrt(fan_in).

    (Same family as torch.nn.Linear's default init; the distribution only
    needs to be realistic, the values are injected, not RNG-matched.)
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    fan = None
    for name, shape in spec:
        if name.endswith("weight"):
            fan = shape[1]
        k = scale / math.sqrt(fan)
        out[name] = rng.uniform(-k, k, size=shape).astype(np.float32)
    return out


def agent_params(alg: str, S: int, A: int, H: int, seed: int, hidden_sizes=None, zs_dim=None) -> dict:
    """All nets (trainable + copies) of one agent: net -> {param: array}."""
    specs = agent_specs(alg, S, A, H, hidden_sizes, zs_dim)
    nets = {}
    for i, (name, spec) in enumerate(specs.items()):
        nets[name] = gen_params(spec, seed * 1000 + i)
    for j, (name, src) in enumerate(COPY_NETS[alg].items()):
        nets[name] = gen_params(specs[src], seed * 1000 + 100 + j)
    return nets


def replay_data(S: int, A: int, n: int, seed: int, act_high: float) -> dict:
    """Synthetic transitions (float64 like env outputs) for append()."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return {
        "state": rng.standard_normal((n, S)),
        "action": rng.uniform(-act_high, act_high, (n, A)).astype(np.float32),
        "reward": rng.standard_normal(n),
        "next_state": rng.standard_normal((n, S)),
        "done": (rng.random(n) > 0.1).astype(np.float64),  # not-done mask (Q4)
    }


def init_priorities(n: int, seed: int) -> np.ndarray:
    """Random LAP priorities >= 1 (like clamp(|d|,1)^0.4 outputs)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    p = (1.0 + np.abs(rng.standard_normal(n)) * 2.0) ** 0.4
    return p.astype(np.float32)


def tapes(alg: str, B: int, A: int, n_steps: int, seed: int) -> dict:
    """Noise tapes per step: u[B] (sampler), eps[B,A] (target smoothing / SAC)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    t = {
        "u": rng.random((n_steps, B), dtype=np.float32),
        "eps": rng.standard_normal((n_steps, B, A), dtype=np.float32),
    }
    if alg == "sac":
        t["eps_pi"] = rng.standard_normal((n_steps, B, A), dtype=np.float32)
    return t
