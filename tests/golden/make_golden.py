"""Generate golden fixtures by running the REFERENCE itself (build container only).

Usage (from the repo root, in the build container where /root/reference exists):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference (``/root/reference/rl``) is imported with an offline
``gymnasium`` stand-in (``gym_stub.py``: env shapes/bounds only — the gradient
step never steps an environment).  Weights, replay data, priorities and noise
tapes are generated deterministically (``oracle/spec.py``) and injected; the
reference then runs its own ``replay.sample`` + ``agent.train_ops`` loop
(``rl/runner/run.py:87-96``) and its outputs are written as ``.npz`` fixtures.
Randomness inside the reference (``torch.rand`` in ``lap.py:48``/``simple.py:47``,
``torch.randn_like`` in ``td7.py:188``/``td3.py:154``, ``Tensor.normal_`` inside
``Normal.rsample`` in ``sac.py:185,222``) is replaced by tape values.

Nothing here runs on the GPU box; only the .npz files travel.
"""

from __future__ import annotations

import os
import sys
from copy import deepcopy

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import gym_stub  # noqa: E402

gym_stub.install()
sys.path.insert(0, "/root/reference")

from rl.agent import SAC, TD3, TD7  # noqa: E402
from rl.nn import MLPActor, MLPCritic, SALEActor, SALECritic, SALEEncoder  # noqa: E402
from rl.replay_memory import LAPReplayMemory, SimpleReplayMemory  # noqa: E402

from oracle import spec  # noqa: E402

torch.set_num_threads(1)


class Tape:
    """Feeds tape values to the reference's RNG call sites."""

    def __init__(self):
        self.queue = []
        self._orig = (torch.rand, torch.randn_like, torch.Tensor.normal_)

    def __enter__(self):
        tape = self

        def rand(*size, **kw):
            v = tape.queue.pop(0)
            assert v[0] == "u", v[0]
            t = torch.from_numpy(v[1].copy())
            assert tuple(t.shape) == tuple(size if not isinstance(size[0], (tuple, list)) else size[0])
            return t

        def randn_like(x, **kw):
            v = tape.queue.pop(0)
            assert v[0] == "eps", v[0]
            t = torch.from_numpy(v[1].copy())
            assert t.shape == x.shape, (t.shape, x.shape)
            return t

        def normal_(self_, *a, **kw):
            v = tape.queue.pop(0)
            assert v[0] in ("eps", "eps_pi"), v[0]
            t = torch.from_numpy(v[1].copy())
            assert t.shape == self_.shape
            with torch.no_grad():
                self_.copy_(t)
            return self_

        torch.rand = rand
        torch.randn_like = randn_like
        torch.Tensor.normal_ = normal_
        return self

    def __exit__(self, *a):
        torch.rand, torch.randn_like, torch.Tensor.normal_ = self._orig


def load_net(module, params):
    sd = module.state_dict()
    assert list(sd.keys()) == list(params.keys()), (list(sd.keys()), list(params.keys()))
    for k in sd:
        assert tuple(sd[k].shape) == params[k].shape, (k, sd[k].shape, params[k].shape)
    module.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in params.items()})


def dump_net(module):
    return {k: v.detach().cpu().numpy().copy() for k, v in module.state_dict().items()}


# hidden activations by name (oracle/nets.py ACTS): SALE `activ` callables (sale.py:25,67,97) and make_mlp's
# action_fn names (mlp.py:13,23 getattr(nn, action_fn)())
SALE_ACTIV = {"relu": torch.nn.functional.relu, "elu": torch.nn.functional.elu, "identity": torch.nn.Identity()}
MLP_ACTION_FN = {"relu": "ReLU", "elu": "ELU", "identity": "Identity"}


def make_agent(alg, env_id, H, use_lap, extra, shape=None, acts=None):
    """The reference agent with its nets built through its own make_nn hook (td7.py:46-61,
    td3.py:44-58, sac.py:40-52): SALE nets with zs_dim / hdim and `activ`, MLPs with make_mlp's hidden_sizes
    and action_fn.  acts: {"actor", "critic", "encoder"} activation names (missing: the defaults)."""
    shape = shape or {}
    acts = acts or {}
    if alg == "td7":
        Z = shape.get("zs_dim", H)
        kw_a, kw_c, kw_e = ({"activ": SALE_ACTIV[acts[k]]} if k in acts else {} for k in ("actor", "critic", "encoder"))

        def mk(state_dim, action_dim, **kw):
            return (SALEActor(state_dim, action_dim, Z, H, **kw_a), SALECritic(state_dim, action_dim, Z, H, **kw_c),
                    SALECritic(state_dim, action_dim, Z, H, **kw_c), SALEEncoder(state_dim, action_dim, Z, H, **kw_e))
        return TD7(env_id, use_lap=use_lap, make_nn=mk, **extra)
    hs = shape.get("hidden_sizes", H)
    kw_a, kw_c = ({"action_fn": MLP_ACTION_FN[acts[k]]} if k in acts else {} for k in ("actor", "critic"))
    if alg == "td3":
        def mk(state_dim, action_dim, **kw):
            return (MLPActor(state_dim, action_dim, hs, **kw_a), MLPCritic(state_dim, action_dim, hs, **kw_c),
                    MLPCritic(state_dim, action_dim, hs, **kw_c))
        return TD3(env_id, use_lap=use_lap, make_nn=mk, **extra)
    if alg == "sac":
        def mk(state_dim, action_dim, **kw):
            return (MLPActor(state_dim, 2 * action_dim, hs, **kw_a), MLPCritic(state_dim, action_dim, hs, **kw_c),
                    MLPCritic(state_dim, action_dim, hs, **kw_c))
        return SAC(env_id, make_nn=mk, **extra)
    raise ValueError(alg)


def inject(agent, alg, nets):
    for name, params in nets.items():
        load_net(getattr(agent, name), params)
    if alg in ("td7", "td3"):
        assert agent.policy is agent.target_policy  # Q1 alias survives


def digest(arr, rng_seed=7, k=64):
    a = np.asarray(arr, dtype=np.float32).ravel()
    rng = np.random.Generator(np.random.PCG64(rng_seed + a.size))
    pos = rng.integers(0, a.size, size=min(k, a.size))
    return np.array([a.astype(np.float64).sum(), np.abs(a.astype(np.float64)).sum()]), pos, a[pos]


def optimizer_moments(agent, nets):
    """Adam first / second moments (exp_avg, exp_avg_sq) of every trained parameter, keyed
    "{net}.{param}" as in the engine's rle_get_adam (td7.py:127-133, td3.py:102-107,
    sac.py:109-123: optim_policy / optim_q_fns / optim_encoder / optim_tmp)."""
    owner = {}
    for net in nets:
        for name, p in getattr(agent, net).named_parameters():
            owner.setdefault(id(p), f"{net}.{name}")
    if getattr(agent, "tmp", None) is not None:
        owner[id(agent.tmp)] = "tmp.log_alpha"
    out = {}
    for attr in ("optim_policy", "optim_q_fns", "optim_encoder", "optim_tmp"):
        opt = getattr(agent, attr, None)
        if opt is None:
            continue
        for p, st in opt.state.items():
            if "exp_avg" not in st:
                continue
            key = owner[id(p)]
            out[key + ":m"] = st["exp_avg"].detach().numpy().copy()
            out[key + ":v"] = st["exp_avg_sq"].detach().numpy().copy()
    return out


def forward_outputs(agent, alg, batch):
    """Forward-only outputs of the nets on a fixed batch (before training)."""
    out = {}
    s, a = batch["state"], batch["action"]
    with torch.no_grad():
        if alg == "td7":
            zs = agent.fixed_encoder.encode_state(s)
            zsa = agent.fixed_encoder.encode_state_action(zs, a)
            out["fwd_zs"] = zs
            out["fwd_zsa"] = zsa
            out["fwd_pi"] = agent.policy.inference_mean(s, zs)
            out["fwd_q1"] = agent.q1.estimate_q_value(s, a, zsa, zs)
            out["fwd_q2"] = agent.q2.estimate_q_value(s, a, zsa, zs)
            ezs = agent.encoder.encode_state(s)
            out["fwd_enc_zs"] = ezs
            out["fwd_enc_zsa"] = agent.encoder.encode_state_action(ezs, a)
        elif alg == "td3":
            out["fwd_pi"] = torch.tanh(agent.policy.inference_mean(s))
            out["fwd_q1"] = agent.q1.estimate_q_value(s, a)
            out["fwd_q2"] = agent.q2.estimate_q_value(s, a)
        else:
            mean, log_std = agent.policy.inference_mean_logvar(s)
            out["fwd_mean"] = mean
            out["fwd_log_std"] = log_std
            out["fwd_q1"] = agent.q1.estimate_q_value(s, a)
            out["fwd_q2"] = agent.q2.estimate_q_value(s, a)
    return {k: v.numpy().copy() for k, v in out.items()}


INFO_KEYS = {
    "td7": ["train/encoder", "train/q_fn", "train/policy"],
    "td3": ["train/q_fn", "train/policy", "norm/policy"],
    "sac": ["train/q_fn", "tmp", "norm/tmp", "train/policy", "train/tmp", "entropy"],
    "sac_fixed": ["train/q_fn", "train/policy", "entropy"],  # tmp >= 0 (sac.py:268-290)
}


ONLY = set(sys.argv[1:])  # optional fixture names to (re)generate; default: all


def run_config(name, alg, env_id, H, B, N, n_fill, n_steps, use_lap, seed, extra=None,
               full=True, sparse_prio=False, adam_steps=2, shape=None, acts=None):
    if ONLY and name not in ONLY:
        return
    extra = dict(extra or {})
    shape = dict(shape or {})
    S, A, hi = spec.TASKS[env_id]
    nets = spec.agent_params(alg, S, A, H, seed, **shape)
    agent = make_agent(alg, env_id, H, use_lap, extra, shape, acts)
    inject(agent, alg, nets)
    lap = use_lap
    replay = (LAPReplayMemory if lap else SimpleReplayMemory)(N, env_id)
    data = spec.replay_data(S, A, n_fill, seed + 1, hi)
    for i in range(n_fill):
        replay.append([data["state"][i], data["action"][i], float(data["reward"][i]),
                       data["next_state"][i], float(data["done"][i])])
    if lap:
        p0 = spec.init_priorities(N, seed + 2)
        p0[replay.size:] = 0.0
        replay.priority[:] = torch.from_numpy(p0)
        replay.max_priority = float(p0.max())
    tp = spec.tapes(alg, B, A, n_steps, seed + 3)

    res = {"meta_alg": np.array(alg), "meta_env": np.array(env_id),
           "meta": np.array([H, B, N, n_fill, n_steps, int(use_lap), seed]),
           "meta_extra_keys": np.array(list(extra.keys()), dtype=object).astype(str),
           "meta_extra_vals": np.array([float(v) for v in extra.values()])}
    if "hidden_sizes" in shape:  # (net shapes beyond the defaults: tests/conftest.py shape_of)
        res["meta_hidden"] = np.array(shape["hidden_sizes"], dtype=np.int64)
    if "zs_dim" in shape:
        res["meta_zs"] = np.array(shape["zs_dim"], dtype=np.int64)
    if acts:  # (hidden activations beyond the defaults: tests/conftest.py acts_of)
        res["meta_acts"] = np.array([acts.get(k, "default") for k in ("actor", "critic", "encoder")])
    for k, v in tp.items():
        res["tape_" + k] = v

    # forward goldens on the first batch indices (deterministic: first B rows)
    fb = {"state": torch.Tensor(replay.state[:B]), "action": torch.Tensor(replay.action[:B])}
    fwd = forward_outputs(agent, alg, fb)
    res.update(fwd if full else {k: v[:32] for k, v in fwd.items()})

    infos, inds = [], []
    for t in range(n_steps):
        with Tape() as tape:
            tape.queue.append(("u", tp["u"][t]))
            batch = replay.sample(B)
            if alg in ("td7", "td3"):
                tape.queue.append(("eps", tp["eps"][t]))
            else:
                tape.queue.append(("eps", tp["eps"][t]))
                tape.queue.append(("eps_pi", tp["eps_pi"][t]))
            ind = np.asarray(replay.ind).copy()
            info = agent.train_ops(batch, replay_buffer=replay)
            assert not tape.queue, "tape not fully consumed"
        inds.append(ind)
        ikeys = INFO_KEYS["sac_fixed" if alg == "sac" and extra.get("tmp", -1.0) >= 0 else alg]
        infos.append([np.nan if info.get(k) is None else float(info[k]) for k in ikeys])
        if lap:
            if sparse_prio:  # only rows ind_t change at step t (lap.py:66-69): their new values
                res[f"prioi_{t}"] = replay.priority.numpy()[ind].copy()
            else:
                res[f"prio_{t}"] = replay.priority.numpy().copy()
            res[f"maxprio_{t}"] = np.array(replay.max_priority, dtype=np.float64)
        if t < adam_steps:  # optimizer moments after steps 1 and 2 (m = 0.1 g after an optimizer's 1st step)
            for key, arr in optimizer_moments(agent, nets).items():
                if full:
                    res[f"adam{t}_{key}"] = arr
                else:
                    d, pos, vals = digest(arr, k=512)
                    res[f"adam{t}_{key}:digest"] = d
                    res[f"adam{t}_{key}:pos"] = pos.astype(np.int32)
                    res[f"adam{t}_{key}:vals"] = vals
        if alg == "td7":
            res[f"vbounds_{t}"] = np.array([float(agent.value_max), float(agent.value_min),
                                            float(agent.value_target_max), float(agent.value_target_min)])
    res["ind"] = np.stack(inds)
    res["info"] = np.array(infos)
    res["info_keys"] = np.array(ikeys)
    names = list(nets.keys())
    for net in names:
        for k, v in dump_net(getattr(agent, net)).items():
            key = f"out_{net}.{k}"
            if full:
                res[key] = v
            else:
                d, pos, vals = digest(v)
                res[key + ":digest"] = d
                res[key + ":pos"] = pos
                res[key + ":vals"] = vals
    if alg == "sac" and agent.auto_tmp_mode:
        res["out_log_alpha"] = agent.tmp.detach().numpy().copy()
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **res)
    print(f"wrote {path} ({os.path.getsize(path)} bytes)")


def lap_sampler_fixture():
    """LAP sample (lap.py:45-64): cumsum/rand*total/searchsorted, plus edge cases."""
    res = {}
    for n, seed in ((65536, 11), (1000000, 12), (1, 13), (4097, 14)):
        p = spec.init_priorities(n, seed)
        rng = np.random.Generator(np.random.PCG64(seed + 100))
        u = rng.random(256, dtype=np.float32)
        u[:4] = [0.0, np.float32(1 - 2**-24), 0.5, np.float32(2**-24)]
        c = torch.cumsum(torch.from_numpy(p), 0)
        v = torch.from_numpy(u) * c[-1]
        ind = torch.searchsorted(c, v).numpy()
        res[f"n{n}_u"] = u
        res[f"n{n}_ind"] = ind
        res[f"n{n}_total"] = c[-1].numpy()
    # priority scatter with duplicates (lap.py:66-69): last occurrence wins (Q9)
    rng = np.random.Generator(np.random.PCG64(21))
    ind = rng.integers(0, 64, size=256)
    pr = (1.0 + rng.random(256)).astype(np.float32)
    base = spec.init_priorities(64, 22)
    t = torch.from_numpy(base.copy())
    t[ind] = torch.from_numpy(pr)
    res["scatter_ind"] = ind
    res["scatter_new"] = pr
    res["scatter_base"] = base
    res["scatter_out"] = t.numpy()
    np.savez_compressed(os.path.join(HERE, "lap_sampler.npz"), **res)


def uniform_sampler_fixture():
    """SimpleReplayMemory.sample (simple.py:42-62) index law."""
    res = {}
    for size in (1, 7, 25000, 1000000):
        rng = np.random.Generator(np.random.PCG64(size))
        u = rng.random(256, dtype=np.float32)
        u[:4] = [0.0, np.float32(1 - 2**-24), 0.5, np.float32(2**-24)]
        c = torch.cumsum(torch.ones(size), 0)
        ind = torch.searchsorted(c, torch.from_numpy(u) * c[-1]).numpy()
        res[f"s{size}_u"] = u
        res[f"s{size}_ind"] = ind
    np.savez_compressed(os.path.join(HERE, "uniform_sampler.npz"), **res)


def sac_rsample_fixture():
    """SAC._inference/_rsample (sac.py:154-172) incl. saturated tanh and log_std clamp."""
    rng = np.random.Generator(np.random.PCG64(31))
    B, A = 64, 6
    mean = (rng.standard_normal((B, A)) * 3).astype(np.float32)
    log_std = (rng.standard_normal((B, A)) * 8).astype(np.float32)
    mean[0, :] = [25.0, -25.0, 10.0, -10.0, 0.0, 1e-3]
    log_std[1, :] = [-30.0, 5.0, -20.0, 2.0, 0.0, -1.0]
    eps = rng.standard_normal((B, A), dtype=np.float32)
    m, ls = torch.from_numpy(mean), torch.from_numpy(log_std)
    ls_c = torch.clamp(ls, -20.0, 2.0)
    dist = torch.distributions.Normal(m, ls_c.exp())
    with Tape() as tape:
        tape.queue.append(("eps", eps))
        a, logp = SAC._rsample(dist)
    np.savez_compressed(os.path.join(HERE, "sac_rsample.npz"), mean=mean, log_std=log_std,
                        eps=eps, action=a.numpy(), log_pi=logp.numpy())


def main():
    if not ONLY:
        lap_sampler_fixture()
        uniform_sampler_fixture()
        sac_rsample_fixture()
    # Tiny full dumps (H=32): multi-step trajectories incl. hard updates.
    run_config("td7_tiny", "td7", "Tiny-v0", 32, 16, 64, 50, 10, True, 5,
               extra={"target_update_rate": 4})
    run_config("td7_tiny_nolap", "td7", "Tiny-v0", 32, 16, 64, 64, 6, False, 6,
               extra={"target_update_rate": 3})
    run_config("td3_tiny", "td3", "Tiny-v0", 32, 16, 64, 50, 6, False, 7)
    run_config("td3_tiny_lap", "td3", "Tiny-v0", 32, 16, 64, 64, 4, True, 8)
    run_config("sac_tiny", "sac", "Tiny-v0", 32, 16, 64, 50, 6, False, 9)
    # fixed temperature (sac.py:55-60: tmp >= 0 is a float; no temperature loss or optimizer)
    run_config("sac_tiny_fixed", "sac", "Tiny-v0", 32, 16, 64, 50, 6, False, 10, extra={"tmp": 0.2})
    # Net shapes beyond the defaults, through make_nn: make_mlp with three hidden layers of unequal
    # widths (mlp.py:10-35; H = the last width), SALE nets with zs_dim != hdim (sale.py:19-26)
    run_config("td3_tiny_deep", "td3", "Tiny-v0", 32, 16, 64, 50, 6, False, 14,
               shape={"hidden_sizes": [32, 48, 32]})
    run_config("sac_tiny_deep", "sac", "Tiny-v0", 32, 16, 64, 50, 6, False, 15,
               shape={"hidden_sizes": [48, 32, 32]})
    run_config("td7_tiny_zs", "td7", "Tiny-v0", 256, 16, 64, 50, 8, True, 16,
               extra={"target_update_rate": 4}, shape={"zs_dim": 128}, full=False)
    # A batch that is not a multiple of 16 (the reference's --batch-size takes any int, cli_utils.py:83):
    # B = 100, the engine pads it to 112 rows and counts 100
    run_config("td7_tiny_b100", "td7", "Tiny-v0", 32, 100, 256, 200, 8, True, 17, extra={"target_update_rate": 4})
    run_config("td3_tiny_b100", "td3", "Tiny-v0", 32, 100, 256, 200, 6, False, 18)
    run_config("sac_tiny_b100", "sac", "Tiny-v0", 32, 100, 256, 200, 6, False, 19)
    # Hidden activations beyond the defaults, through make_nn: SALE nets' `activ` (sale.py:25,67,97) swapped
    # (actor ELU, critics and encoder ReLU), make_mlp's action_fn (mlp.py:13,23) as ELU / Identity
    # Hyper-parameters beyond the defaults (the agents' constructor arguments, td7.py:34-43, td3.py:33-43,
    # sac.py:27-37): policy_freq 3 (single-step graphs), discount, learning rates, smoothing noise, tau, log-std bounds
    run_config("td7_tiny_hp", "td7", "Tiny-v0", 32, 16, 64, 50, 9, True, 24,
               extra={"target_update_rate": 4, "policy_freq": 3, "discount_factor": 0.95, "policy_lr": 1e-3,
                      "critic_lr": 5e-4, "target_policy_noise": 0.3, "noise_clip": 0.4})
    run_config("td3_tiny_hp", "td3", "Tiny-v0", 32, 16, 64, 50, 7, False, 25,
               extra={"policy_freq": 3, "discount_factor": 0.9, "policy_lr": 1e-3, "critic_lr": 5e-4,
                      "target_policy_noise": 0.1, "noise_clip": 0.25, "tau": 0.02})
    run_config("sac_tiny_hp", "sac", "Tiny-v0", 32, 16, 64, 50, 6, False, 26,
               extra={"discount_factor": 0.9, "policy_lr": 1e-3, "critic_lr": 5e-4, "tau": 0.02, "min_log_std": -5.0,
                      "max_log_std": 1.0})
    run_config("td7_tiny_act", "td7", "Tiny-v0", 32, 16, 64, 50, 8, True, 20, extra={"target_update_rate": 4},
               acts={"actor": "elu", "critic": "relu", "encoder": "relu"})
    run_config("td7_tiny_act_id", "td7", "Tiny-v0", 32, 16, 64, 50, 6, False, 23, extra={"target_update_rate": 3},
               acts={"critic": "identity"})
    run_config("td3_tiny_act", "td3", "Tiny-v0", 32, 16, 64, 50, 6, True, 21,
               acts={"actor": "elu", "critic": "identity"})
    run_config("sac_tiny_act", "sac", "Tiny-v0", 32, 16, 64, 50, 6, False, 22,
               acts={"actor": "identity", "critic": "elu"}, shape={"hidden_sizes": [32, 48, 32]})
    # Full-size digests at the BASELINE configs' shapes.
    run_config("td7_humanoid", "td7", "Humanoid-v4", 256, 256, 2048, 2048, 3, True, 41,
               full=False)
    run_config("td7_ant", "td7", "Ant-v4", 256, 256, 2048, 2048, 2, True, 42, full=False)
    run_config("td3_halfcheetah", "td3", "HalfCheetah-v4", 256, 256, 2048, 2048, 3, False, 43,
               full=False)
    run_config("sac_humanoid", "sac", "Humanoid-v4", 256, 256, 2048, 2048, 2, False, 44,
               full=False)
    # Many-block LAP trajectory at full width: 65,536 rows (16 block sums of 4,096), 12 steps,
    # hard updates at steps 5 and 10 (td7.py:278-285, 325-331), a 4-step graph at steps 6-9.
    run_config("td7_humanoid_64k", "td7", "Humanoid-v4", 256, 256, 65536, 65536, 12, True, 45,
               extra={"target_update_rate": 5}, full=False, sparse_prio=True)


if __name__ == "__main__":
    main()
