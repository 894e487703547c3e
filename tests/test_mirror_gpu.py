"""The reference-interface mirror (sac-td3-td7_amd/rl) on the HIP engine.

Drives agents exactly like the reference's runner does — ``replay.sample(B)`` then
``agent.train_ops(batch, replay)`` (rl/runner/run.py:87-96) — and checks against the
oracle on the same batches.  Target-smoothing noise is a Philox stream on the device,
so the explicit-batch parity cases use target_policy_noise = 0 (TD7/TD3: the noise term
is then exactly 0 in the reference too, td7.py:188-190, td3.py:158-160).
"""

import copy
import pickle

import numpy as np
import pytest
import torch

from oracle import agents as OA
from oracle import replay as OR
from harness import LOSS_RTOL  # noqa: E402
from rl import _engine as E
from rl.agent import SAC, TD3, TD7
from rl.replay_memory import LAPReplayMemory, SimpleReplayMemory
from rl.runner.run import run_train_ops
from rl.utils import register_env

pytestmark = pytest.mark.gpu

register_env("Tiny-v0", 11, 3, -0.5, 0.5)
S, A, HI = 11, 3, 0.5


def _transitions(n, seed):
    rng = np.random.default_rng(seed)
    return [(rng.standard_normal(S), rng.uniform(-HI, HI, A), float(rng.standard_normal()),
             rng.standard_normal(S), float(rng.random() > 0.1)) for _ in range(n)]


def _fill(rep, trans):
    for t in trans:
        rep.append(list(t))


def _oracle_replay(cap, lap, trans):
    r = OR.Replay(cap, S, A, np.full(A, HI, np.float32), np.zeros(A, np.float32), lap)
    for t in trans:
        r.append(*t)
    return r


def _close(a, b, tol):
    if a is None or b is None:
        assert a is None and b is None
    else:
        assert abs(a - b) <= tol * (1 + abs(b)), (a, b)


@pytest.mark.parametrize("alg,lap,B", [("td7", True, 32), ("td7", False, 32), ("td3", False, 32), ("td3", True, 32),
                                       ("td7", True, 20), ("td3", False, 20), ("td7", True, 1), ("td3", True, 17)])
# (B = 20 / 1 / 17: padded to 32 / 16 / 32 rows inside; the padded rows count in nothing)
def test_train_ops_on_sampled_batches_matches_oracle(alg, lap, B):
    cap, H, steps = 512, 32, 6
    trans = _transitions(300, 1)
    Agent = TD7 if alg == "td7" else TD3
    ag = Agent("Tiny-v0", use_lap=lap, target_policy_noise=0.0, hidden=H, batch_size=B, seed=5)
    rep = (LAPReplayMemory if lap else SimpleReplayMemory)(cap, "Tiny-v0")
    _fill(rep, trans)
    assert len(rep) == 300 and rep.size == 300
    nets = {k: dict(v) for k, v in ag.state_dict().items()}
    orc = OA.make_oracle(alg, nets, A, lap, target_policy_noise=0.0)
    orep = _oracle_replay(cap, lap, trans)
    torch.manual_seed(0)
    for t in range(steps):
        u_ref = torch.rand(B, generator=torch.Generator().manual_seed(1000 + t)).numpy()
        torch.manual_seed(1000 + t)
        batch = rep.sample(B)
        ind_ref = orep.sample_indices(u_ref)
        np.testing.assert_array_equal(batch.ind, ind_ref)
        ob = orep.gather(ind_ref)
        for k in ("state", "action", "reward", "next_state", "done"):
            np.testing.assert_array_equal(batch[k].numpy(), ob[k])
        info = ag.train_ops(batch, rep)
        ref = orc.step(ob, orep, np.zeros((B, A), np.float32))
        assert list(info) == list(ref)
        for k in ref:
            _close(info[k], ref[k], LOSS_RTOL)
        if lap:
            np.testing.assert_allclose(rep.priority.numpy()[:300], orep.priority[:300], rtol=1e-4, atol=1e-5)
            assert abs(rep.max_priority - orep.max_priority) <= 1e-4 * orep.max_priority
    # parameters: every element within the Adam sign-flip bound 2 lr t, and (the criterion that
    # catches a wrong gradient) >= 99% of each tensor within 1e-5 (H = 32 tensors)
    got = ag.state_dict()
    for net, d in orc.nets().items():
        for name, v in d.items():
            ref = v.detach().numpy()
            np.testing.assert_allclose(got[net][name], ref, rtol=0, atol=2 * 3e-4 * steps + 1e-4)
            close = np.abs(got[net][name] - ref) <= 1e-5 + 1e-5 * np.abs(ref)
            assert close.mean() >= 0.99, (net, name, float(close.mean()))


def test_sac_train_ops_info_keys_and_fused_loop():
    cap, B, H = 512, 32, 32
    ag = SAC("Tiny-v0", hidden=H, batch_size=B, seed=3)
    rep = SimpleReplayMemory(cap, "Tiny-v0")
    _fill(rep, _transitions(200, 2))
    info = ag.train_ops(rep.sample(B), rep)
    assert list(info) == ["train/q_fn", "tmp", "norm/tmp", "train/policy", "train/tmp", "entropy"]
    assert all(np.isfinite(v) for v in info.values())
    infos = run_train_ops(type("R", (), {"replay_buffer": rep})(), ag, B, n_ops=5)
    assert len(infos) == 5 and ag.n_runs == 6
    assert rep.ind.shape == (B,) and rep.ind.max() < 200
    fixed = SAC("Tiny-v0", tmp=0.2, hidden=H, batch_size=B, seed=3)
    info = fixed.train_ops(rep.sample(B), rep)
    assert list(info) == ["train/q_fn", "train/policy", "entropy"]


def test_pickle_roundtrip_continues_identically(tmp_path):
    cap, B, H = 512, 32, 32
    ag = TD7("Tiny-v0", use_lap=True, hidden=H, batch_size=B, seed=9)
    rep = LAPReplayMemory(cap, "Tiny-v0")
    _fill(rep, _transitions(300, 3))
    run_train_ops(type("R", (), {"replay_buffer": rep})(), ag, B, n_ops=3)
    path = tmp_path / "agent.pkl"
    ag.save(path)
    ag2 = TD7.load(path)
    ag3 = copy.deepcopy(ag)
    assert ag2.n_runs == ag.n_runs == 3
    for net, d in ag.state_dict().items():
        for name, v in d.items():
            np.testing.assert_array_equal(ag2.state_dict()[net][name], v)
    # same explicit batch -> bit-identical steps (same Philox stream position, same state)
    p0, m0 = rep.priority.numpy().copy(), rep.max_priority
    torch.manual_seed(7)
    batch = rep.sample(B)
    i1 = ag.train_ops(batch, rep)
    rep.dev.set_priority(p0, m0)
    i2 = ag2.train_ops(batch, rep)
    rep.dev.set_priority(p0, m0)
    i3 = ag3.train_ops(batch, rep)
    assert i1 == i2 == i3
    pickle.loads(pickle.dumps(ag))  # in-memory too


def test_load_state_dict_copies_networks_only():
    B, H = 32, 32
    a = TD3("Tiny-v0", hidden=H, batch_size=B, seed=1)
    b = TD3("Tiny-v0", hidden=H, batch_size=B, seed=2)
    rep = SimpleReplayMemory(256, "Tiny-v0")
    _fill(rep, _transitions(100, 4))
    run_train_ops(type("R", (), {"replay_buffer": rep})(), a, B, n_ops=2)
    b.load_state_dict(a)
    for net, d in a.state_dict().items():
        for name, v in d.items():
            np.testing.assert_array_equal(b.state_dict()[net][name], v)
    assert b.n_runs == 0  # optimiser state / counters are not part of load_state_dict (td3.py:94-100)


def test_sample_actions_match_oracle_forward():
    from oracle import nets as N

    for Agent in (TD7, TD3, SAC):
        ag = Agent("Tiny-v0", hidden=32, batch_size=32, seed=4)
        obs = np.random.default_rng(0).standard_normal(S).astype(np.float32)
        sd = {k: {n: torch.from_numpy(v) for n, v in d.items()} for k, d in ag.state_dict().items()}
        x = torch.from_numpy(obs)[None]
        with torch.no_grad():
            if Agent is TD7:
                ref = N.sale_actor(sd["policy"], x, N.sale_zs(sd["fixed_encoder"], x))
            elif Agent is TD3:
                ref = torch.tanh(N.mlp(sd["policy"], x))
            else:
                ref = torch.tanh(N.mlp(sd["policy"], x).chunk(2, -1)[0])
        got = ag.sample(obs, deterministic=True)
        np.testing.assert_allclose(got, ref.numpy()[0] * HI, rtol=1e-5, atol=1e-6)
        stoch = ag.sample(obs)
        assert stoch.shape == (A,) and np.all(np.abs(stoch) <= HI + 1e-6)


def _oracle_env_action(Agent, ag, obs, eps):
    """The reference's sample() (td7.py:141-156, td3.py:114-129, sac.py:132-152) on the oracle
    nets with the exploration draw eps in place of torch.randn_like: float32 throughout."""
    from oracle import nets as N

    sd = {k: {n: torch.from_numpy(v) for n, v in d.items()} for k, d in ag.state_dict().items()}
    x = torch.from_numpy(np.asarray(obs, np.float32))[None]
    e = torch.from_numpy(np.asarray(eps, np.float32))[None]
    with torch.no_grad():
        if Agent is SAC:
            mean, log_std = N.mlp(sd["policy"], x).chunk(2, -1)
            log_std = torch.clamp(log_std, ag.min_log_std, ag.max_log_std)
            a = torch.tanh(mean + e * log_std.exp()).numpy()[0]
        else:
            if Agent is TD7:
                a = N.sale_actor(sd["policy"], x, N.sale_zs(sd["fixed_encoder"], x))
            else:
                a = torch.tanh(N.mlp(sd["policy"], x))
            a = a + e * ag.exploration_noise
            a = np.clip(a.numpy()[0], -1.0, 1.0)
    return a * ag.action_scale + ag.action_bias


@pytest.mark.parametrize("Agent", [TD7, TD3, SAC])
def test_fused_act_sample_matches_oracle_with_noise_tape(Agent):
    """agent.sample as one device program (forward + exploration noise +
    clip + action map, rle_act_sample) equals the reference's sample() on the same draw:
    |d| <= 2e-6 + 1e-5 |ref| (fp32 tanh / exp ulps)."""
    ag = Agent("Tiny-v0", hidden=32, batch_size=32, seed=7)
    rng = np.random.default_rng(3)
    for k in range(4):
        obs = rng.standard_normal(S).astype(np.float32) * (1 + 2 * k)  # k = 3: saturated outputs
        eps = rng.standard_normal(A).astype(np.float32) * (1 + 4 * (k == 2))  # k = 2: clipping
        ref = _oracle_env_action(Agent, ag, obs, eps)
        got = ag.sample(obs, eps=eps)
        assert got.dtype == np.float32 and got.shape == (A,)
        assert (np.abs(got - ref) <= 2e-6 + 1e-5 * np.abs(ref)).all(), (k, got, ref)
        det = ag.sample(obs, deterministic=True)
        ref0 = _oracle_env_action(Agent, ag, obs, np.zeros(A, np.float32))
        assert (np.abs(det - ref0) <= 2e-6 + 1e-5 * np.abs(ref0)).all(), (k, det, ref0)


def test_fused_act_sample_humanoid_and_batches():
    """Full-size TD7 Humanoid (S 376, A 17, scale 0.4): the taped draw against the oracle, and a
    batch of n = 5 observations (the act graph) agrees with five single calls (n = 1: the
    one-launch act chain, its own summation order) to fp32 rounding."""
    ag = TD7("Humanoid-v4", batch_size=256, seed=11)
    rng = np.random.default_rng(5)
    obs = rng.standard_normal(376).astype(np.float32)
    eps = rng.standard_normal(17).astype(np.float32)
    ref = _oracle_env_action(TD7, ag, obs, eps)
    got = ag.sample(obs, eps=eps)
    assert (np.abs(got - ref) <= 2e-6 + 1e-5 * np.abs(ref)).all(), np.abs(got - ref).max()
    xs = rng.standard_normal((5, 376)).astype(np.float32)
    es = rng.standard_normal((5, 17)).astype(np.float32)
    batch = ag.engine.act_sample(xs, 2, es).copy()
    for i in range(5):
        one = ag.sample(xs[i], eps=es[i])
        assert (np.abs(batch[i] - one) <= 2e-6 + 1e-5 * np.abs(one)).all(), (i, np.abs(batch[i] - one).max())
        ref = _oracle_env_action(TD7, ag, xs[i], es[i])
        assert (np.abs(one - ref) <= 2e-6 + 1e-5 * np.abs(ref)).all(), (i, np.abs(one - ref).max())


def test_fused_act_sample_philox_noise_statistics():
    """Device exploration draws (mode 1): (stochastic - deterministic) / (scale * sigma) is
    N(0, 1) per action dimension where unclipped, and consecutive calls draw fresh noise."""
    ag = TD3("Tiny-v0", hidden=32, batch_size=32, seed=2)
    obs = np.zeros(S, np.float32)
    det = ag.sample(obs, deterministic=True)
    z = np.stack([ag.sample(obs) for _ in range(3000)])
    z = (z - det) / (HI * ag.exploration_noise)
    assert len({tuple(r) for r in z[:50]}) == 50
    assert np.abs(z.mean(0)).max() < 0.08 and np.abs(z.std(0) - 1).max() < 0.06, (z.mean(0), z.std(0))


def test_batch_size_change_rebuilds_engine():
    ag = TD3("Tiny-v0", hidden=32, batch_size=32, seed=1)
    rep = SimpleReplayMemory(256, "Tiny-v0")
    _fill(rep, _transitions(100, 5))
    before = ag.state_dict()["q1"]["mlp.0.weight"].copy()
    info = ag.train_ops(rep.sample(48), rep)
    assert ag.batch_size == 48 and np.isfinite(info["train/q_fn"])
    assert not np.array_equal(before, ag.state_dict()["q1"]["mlp.0.weight"])


def test_act_sample_rejects_misshaped_observations():
    """A wrong observation width or rank raises (the reference's first Linear would), instead of
    the kernel reading past the caller's buffer."""
    ag = TD3("Tiny-v0", hidden=32, batch_size=32, seed=2)
    for bad in (np.zeros(S - 1, np.float32), np.zeros((2, S + 1), np.float32), np.zeros((1, 1, S), np.float32)):
        with pytest.raises(ValueError):
            ag.sample(bad)
    assert ag.sample(np.zeros(S, np.float32)).shape == (A,)


def test_act_map_and_exploration_stream_follow_the_agent():
    """action_scale / exploration_noise changes apply to the next sample() (the reference reads
    them per call), and a rebuilt engine (batch-size change) continues the Philox exploration
    stream instead of repeating its first draws."""
    ag = TD7("Tiny-v0", hidden=32, batch_size=32, seed=4)
    obs = np.linspace(-1, 1, S).astype(np.float32)
    det = ag.sample(obs, deterministic=True)
    ag.action_scale = ag.action_scale * 2
    assert np.allclose(ag.sample(obs, deterministic=True), 2 * det, rtol=1e-6, atol=1e-7)
    ag.action_scale = ag.action_scale / 2
    ag.exploration_noise = 0.0
    assert np.array_equal(ag.sample(obs), det)  # sigma 0: the exploration draw adds exactly 0
    ag.exploration_noise = 0.1
    first = [ag.sample(obs).copy() for _ in range(3)]
    rep = LAPReplayMemory(256, "Tiny-v0")
    _fill(rep, _transitions(100, 5))
    ag.train_ops(rep.sample(48), rep)  # batch 32 -> 48: a new engine
    after = [ag.sample(obs).copy() for _ in range(3)]
    assert all(not np.array_equal(a, b) for a in first for b in after)


def test_act_chain_failed_hand_off_is_reported(monkeypatch):
    """The one-launch act chain's failure path: a workgroup that withholds its granules
    (RLE_ACT_FAIL_WG, first call only) makes every consumer time out and poison its own
    granules, the head reports the failure before its completion tag, the call raises, and
    the next call on the same engine succeeds (the error flag is per call)."""
    monkeypatch.setenv("RLE_ACT_FAIL_WG", "1")
    ag = TD3("Tiny-v0", hidden=32, batch_size=32, seed=2)
    obs = np.zeros(S, np.float32)
    with pytest.raises(RuntimeError, match="hand-off"):
        ag.sample(obs, deterministic=True)
    monkeypatch.delenv("RLE_ACT_FAIL_WG")
    ref = TD3("Tiny-v0", hidden=32, batch_size=32, seed=2).sample(obs, deterministic=True)
    assert np.array_equal(ag.sample(obs, deterministic=True), ref)


def test_make_nn_hook_with_reference_net_types():
    """td7.py:56-61 / td3.py:53-56 / sac.py:47-50: a make_nn callable returning the reference's
    default net types (rl.nn.SALEActor / SALECritic / SALEEncoder, MLPActor / MLPCritic) at one
    width builds the engine at that width with the hook's initial weights (targets and fixed
    encoders copies of them); other types or mixed widths are rejected."""
    from rl.nn import MLPActor, MLPCritic, SALEActor, SALECritic, SALEEncoder

    torch.manual_seed(0)
    made = {}

    def mk7(state_dim, action_dim, **kw):
        made["td7"] = (SALEActor(state_dim, action_dim, 32, 32), SALECritic(state_dim, action_dim, 32, 32),
                       SALECritic(state_dim, action_dim, 32, 32), SALEEncoder(state_dim, action_dim, 32, 32))
        return made["td7"]

    ag = TD7("Tiny-v0", make_nn=mk7, batch_size=16, seed=1)
    assert ag.hidden == 32
    sd = ag.state_dict()
    for name, m in zip(("policy", "q1", "q2", "encoder"), made["td7"]):
        for k, v in m.state_dict().items():
            np.testing.assert_array_equal(sd[name][k], v.numpy())
    for k, v in made["td7"][3].state_dict().items():
        np.testing.assert_array_equal(sd["fixed_encoder_target"][k], v.numpy())
    # forward parity with the hook's own torch modules (the device act path)
    obs = np.linspace(-1, 1, S).astype(np.float32)
    pol, enc = made["td7"][0], made["td7"][3]
    with torch.no_grad():
        x = torch.from_numpy(obs)[None]
        ref = pol.inference_mean(x, enc.encode_state(x)).numpy()[0] * ag.action_scale + ag.action_bias
    got = ag.sample(obs, deterministic=True)
    assert np.abs(got - ref).max() <= 2e-6 + 1e-5 * np.abs(ref).max()

    def mk3(state_dim, action_dim, **kw):
        return MLPActor(state_dim, action_dim, 64), MLPCritic(state_dim, action_dim, 64), MLPCritic(state_dim, action_dim, 64)

    assert TD3("Tiny-v0", make_nn=mk3, batch_size=16, seed=1).hidden == 64

    def mks(state_dim, action_dim, **kw):
        return (MLPActor(state_dim, 2 * action_dim, [48, 48]), MLPCritic(state_dim, action_dim, 48),
                MLPCritic(state_dim, action_dim, 48))

    assert SAC("Tiny-v0", make_nn=mks, batch_size=16, seed=1).hidden == 48

    def mixed(state_dim, action_dim, **kw):
        return MLPActor(state_dim, action_dim, 64), MLPCritic(state_dim, action_dim, 32), MLPCritic(state_dim, action_dim, 32)

    with pytest.raises(NotImplementedError):
        TD3("Tiny-v0", make_nn=mixed, batch_size=16, seed=1)

    def other(state_dim, action_dim, **kw):
        return torch.nn.Linear(state_dim, action_dim), MLPCritic(state_dim, action_dim), MLPCritic(state_dim, action_dim)

    with pytest.raises(NotImplementedError):
        TD3("Tiny-v0", make_nn=other, batch_size=16, seed=1)


def test_make_nn_hook_with_other_net_shapes():
    """make_nn hooks with the shapes make_mlp / the SALE nets take beyond the defaults
    (mlp.py:10-35 any depth and widths, sale.py:19-26 zs_dim != hdim): the engine builds those
    nets with the hook's weights, acts as the hook's torch modules do, trains, and pickles back to
    the same state (the trajectories themselves: td3_tiny_deep / sac_tiny_deep / td7_tiny_zs)."""
    from rl.nn import MLPActor, MLPCritic, SALEActor, SALECritic, SALEEncoder

    torch.manual_seed(3)
    made = {}

    def mk3(state_dim, action_dim, **kw):
        hs = [32, 48, 32]
        made["td3"] = (MLPActor(state_dim, action_dim, hs), MLPCritic(state_dim, action_dim, hs),
                       MLPCritic(state_dim, action_dim, hs))
        return made["td3"]

    def mks(state_dim, action_dim, **kw):
        hs = [48, 32, 32, 16]
        made["sac"] = (MLPActor(state_dim, 2 * action_dim, hs), MLPCritic(state_dim, action_dim, hs),
                       MLPCritic(state_dim, action_dim, hs))
        return made["sac"]

    def mk7(state_dim, action_dim, **kw):
        made["td7"] = (SALEActor(state_dim, action_dim, 16, 64), SALECritic(state_dim, action_dim, 16, 64),
                       SALECritic(state_dim, action_dim, 16, 64), SALEEncoder(state_dim, action_dim, 16, 64))
        return made["td7"]

    obs = np.linspace(-1, 1, S).astype(np.float32)
    x = torch.from_numpy(obs)[None]
    trans = _transitions(200, 5)
    for cls, mk, alg in ((TD3, mk3, "td3"), (SAC, mks, "sac"), (TD7, mk7, "td7")):
        ag = cls("Tiny-v0", make_nn=mk, batch_size=16, seed=4)
        sd = ag.state_dict()
        for name, m in zip(("policy", "q1", "q2", "encoder"), made[alg]):
            for k, v in m.state_dict().items():
                np.testing.assert_array_equal(sd[name][k], v.numpy())
        with torch.no_grad():
            if alg == "td7":
                pol, enc = made["td7"][0], made["td7"][3]
                ref = pol.inference_mean(x, enc.encode_state(x)).numpy()[0]
            elif alg == "td3":
                ref = torch.tanh(made["td3"][0].inference_mean(x)).numpy()[0]
            else:
                ref = torch.tanh(made["sac"][0].inference_mean_logvar(x)[0]).numpy()[0]
        ref = ref * ag.action_scale + ag.action_bias
        got = ag.sample(obs, deterministic=True)
        assert np.abs(got - ref).max() <= 2e-6 + 1e-5 * np.abs(ref).max(), alg
        rep = (LAPReplayMemory if alg == "td7" else SimpleReplayMemory)(256, "Tiny-v0")
        _fill(rep, trans)
        run_train_ops(rep, ag, 16, 5)
        ag2 = pickle.loads(pickle.dumps(ag))
        sd, sd2 = ag.state_dict(), ag2.state_dict()
        for name in sd:
            for k in sd[name]:
                np.testing.assert_array_equal(sd[name][k], sd2[name][k])
        assert ag2.shape == ag.shape and ag.shape


def test_make_nn_hook_with_other_activations():
    """make_nn hooks whose nets use other hidden activations (sale.py:25,67,97 `activ`; mlp.py:13,23 action_fn,
    with make_mlp's init_weight / init_bias): the engine runs them (rle_config act_*), acts as the hook's torch
    modules do, trains, and pickles back with the same activations (the trajectories themselves: the
    td7_tiny_act / td3_tiny_act / sac_tiny_act goldens)."""
    from torch.nn import functional as F

    from rl.nn import MLPActor, MLPCritic, SALEActor, SALECritic, SALEEncoder

    torch.manual_seed(5)
    made = {}

    def mk3(state_dim, action_dim, **kw):
        made["td3"] = (MLPActor(state_dim, action_dim, 32, action_fn="ELU", init_weight="orthogonal_"),
                       MLPCritic(state_dim, action_dim, 32, action_fn="Identity", init_bias="normal_"),
                       MLPCritic(state_dim, action_dim, 32, action_fn="Identity", init_bias="normal_"))
        return made["td3"]

    def mks(state_dim, action_dim, **kw):
        made["sac"] = (MLPActor(state_dim, 2 * action_dim, [48, 32], action_fn=torch.nn.Identity()),
                       MLPCritic(state_dim, action_dim, [48, 32], action_fn=torch.nn.ELU()),
                       MLPCritic(state_dim, action_dim, [48, 32], action_fn=torch.nn.ELU()))
        return made["sac"]

    def mk7(state_dim, action_dim, **kw):
        made["td7"] = (SALEActor(state_dim, action_dim, 32, 32, activ=F.elu),
                       SALECritic(state_dim, action_dim, 32, 32, activ=F.relu),
                       SALECritic(state_dim, action_dim, 32, 32, activ=F.relu),
                       SALEEncoder(state_dim, action_dim, 32, 32, activ=F.relu))
        return made["td7"]

    want = {"td3": {"act_actor": "elu", "act_critic": "identity"}, "sac": {"act_actor": "identity", "act_critic": "elu"},
            "td7": {"act_actor": "elu", "act_critic": "relu", "act_encoder": "relu"}}
    obs = np.linspace(-1, 1, S).astype(np.float32)
    x = torch.from_numpy(obs)[None]
    trans = _transitions(200, 6)
    for cls, mk, alg in ((TD3, mk3, "td3"), (SAC, mks, "sac"), (TD7, mk7, "td7")):
        ag = cls("Tiny-v0", make_nn=mk, batch_size=16, seed=4)
        assert {k: v for k, v in ag.acts.items() if k in want[alg]} == want[alg], ag.acts
        codes = {k: getattr(ag.engine.cfg, k) for k in want[alg]}
        assert codes == {k: E.ACT_CODES[v] for k, v in want[alg].items()}
        sd = ag.state_dict()
        for name, m in zip(("policy", "q1", "q2", "encoder"), made[alg]):
            for k, v in m.state_dict().items():
                np.testing.assert_array_equal(sd[name][k], v.numpy())
        with torch.no_grad():
            if alg == "td7":
                pol, enc = made["td7"][0], made["td7"][3]
                ref = pol.inference_mean(x, enc.encode_state(x)).numpy()[0]
            elif alg == "td3":
                ref = torch.tanh(made["td3"][0].inference_mean(x)).numpy()[0]
            else:
                ref = torch.tanh(made["sac"][0].inference_mean_logvar(x)[0]).numpy()[0]
        ref = ref * ag.action_scale + ag.action_bias
        got = ag.sample(obs, deterministic=True)
        assert np.abs(got - ref).max() <= 2e-6 + 1e-5 * np.abs(ref).max(), alg
        rep = (LAPReplayMemory if alg == "td7" else SimpleReplayMemory)(256, "Tiny-v0")
        _fill(rep, trans)
        run_train_ops(rep, ag, 16, 5)
        ag2 = pickle.loads(pickle.dumps(ag))
        assert ag2.acts == ag.acts
        assert {k: getattr(ag2.engine.cfg, k) for k in want[alg]} == codes
        sd, sd2 = ag.state_dict(), ag2.state_dict()
        for name in sd:
            for k in sd[name]:
                np.testing.assert_array_equal(sd[name][k], sd2[name][k])


def test_train_ops_on_a_host_batch_dict():
    """abc.py:23-28: train_ops on a plain BATCH dict (here the oracle replay's gather, as a host
    replay would hand it over) trains exactly as on the same rows drawn from a device replay, and
    a LAP host replay receives the step's priorities through its own update_priority."""
    cap, B, H, steps = 512, 32, 32, 3
    trans = _transitions(300, 11)
    for lap in (True, False):
        dev = TD7("Tiny-v0", use_lap=lap, target_policy_noise=0.0, hidden=H, batch_size=B, seed=21)
        host = TD7("Tiny-v0", use_lap=lap, target_policy_noise=0.0, hidden=H, batch_size=B, seed=21)
        rep = (LAPReplayMemory if lap else SimpleReplayMemory)(cap, "Tiny-v0")
        _fill(rep, trans)
        orep = _oracle_replay(cap, lap, trans)
        for t in range(steps):
            torch.manual_seed(500 + t)
            batch = rep.sample(B)
            orep.ind = np.asarray(batch.ind)
            hb = {k: torch.from_numpy(v) for k, v in orep.gather(batch.ind).items()}
            i_dev = dev.train_ops(batch, rep)
            i_host = host.train_ops(hb, orep)
            for k in i_dev:
                _close(i_host[k], i_dev[k], 1e-6)
            if lap:
                np.testing.assert_allclose(orep.priority[batch.ind], rep.priority.numpy()[batch.ind], rtol=1e-6)
        for net, d in dev.state_dict().items():
            for name, v in d.items():
                np.testing.assert_array_equal(host.state_dict()[net][name], v)


def test_lap_agent_host_batch_needs_its_lap_replay():
    """A LAP agent's train_ops on a host BATCH dict with no LAP replay to send the priorities to fails
    as the reference's assert does (td7.py:310, td3.py:221), instead of skipping the update."""
    ag = TD7("Tiny-v0", use_lap=True, hidden=32, batch_size=32, seed=3)
    t = _transitions(32, 9)
    batch = {k: np.array([r[i] for r in t], np.float32) for i, k in enumerate(("state", "action", "reward",
                                                                               "next_state", "done"))}
    with pytest.raises(AssertionError):
        ag.train_ops(batch, None)
    with pytest.raises(AssertionError):
        ag.train_ops(batch, SimpleReplayMemory(64, "Tiny-v0"))
