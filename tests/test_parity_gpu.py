"""Device parity beyond the loss scalars: Q-values / embeddings of every net the step trains,
Adam moments (the step's gradients), SAC rsample, independent seeds stepped asynchronously,
and replay operations ordered after asynchronous steps.  All through the C ABI.

Tolerances (stated per check):
* forward outputs (Q, zs, zsa): |d| <= 1e-5 + 1e-5 |ref|  (fp32, different reduction order);
* Adam moments after an optimizer's first steps (m = 0.1 g, v = 0.001 g^2 at step 1):
  |d| <= 1e-4 |ref| + 1e-4 max|ref of that tensor| (gradients at rel 1e-4; the
  floor scales with the tensor because a sum of B = 256 products that cancels to ~0 has an
  absolute, not relative, fp32 error);
* SAC rsample: action |d| <= 2e-6, log_pi |d| <= 1e-4 + 1e-5 |ref| (a sum of A logs).
"""

import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

E = pytest.importorskip("rl._engine")
from harness import LOSS_RTOL, engine_from_golden, parse, shape_of  # noqa: E402
from oracle import spec  # noqa: E402
from test_oracle import expected_priorities, golden_moments  # noqa: E402

ALL = ["td7_tiny", "td7_tiny_nolap", "td3_tiny", "td3_tiny_lap", "sac_tiny", "sac_tiny_fixed", "td7_humanoid", "td7_ant",
       "td3_halfcheetah", "sac_humanoid", "td7_humanoid_64k", "td3_tiny_deep", "sac_tiny_deep", "td7_tiny_zs",
       "td7_tiny_b100", "td3_tiny_b100", "sac_tiny_b100",  # (b100: a batch of 100 -- not a multiple of 16)
       "td7_tiny_act", "td7_tiny_act_id", "td3_tiny_act", "sac_tiny_act",  # (act: hidden activations beyond the defaults)
        "td7_tiny_hp", "td3_tiny_hp", "sac_tiny_hp"]  # (hp: constructor hyper-parameters beyond the defaults)


def _fwd_close(got, ref, what):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    d = np.abs(got - ref)
    lim = 1e-5 + 1e-5 * np.abs(ref)
    assert (d <= lim).all(), (what, float(d.max()), float((d / lim).max()))


@pytest.mark.parametrize("name", ALL)
def test_eval_matches_reference(name):
    """estimate_q_value / encode_state / encode_state_action on the golden's fixed batch
    (make_golden.forward_outputs: first B replay rows, weights before any step)."""
    g = load_golden(name)
    alg, env, H, B, *_ = parse(g)
    S, A, _ = spec.TASKS[env]
    eng, rep, _ = engine_from_golden(g)
    n = g["fwd_q1"].shape[0]
    s, a, *_ = rep.gather(np.arange(n))
    params = spec.agent_params(alg, S, A, H, int(g["meta"][6]), **shape_of(g))
    same = lambda x, y: all(np.array_equal(params[x][k], params[y][k]) for k in params[x])  # noqa: E731
    if alg == "td7":
        for q in ("q1", "q2"):
            _fwd_close(eng.eval_q(q, s, a, "fixed_encoder"), g[f"fwd_{q}"][:, 0], q)
            if same(q, "target_" + q) and same("fixed_encoder", "fixed_encoder_target"):
                _fwd_close(eng.eval_q("target_" + q, s, a, "fixed_encoder_target"), g[f"fwd_{q}"][:, 0], "t" + q)
        _fwd_close(eng.eval_zs("fixed_encoder", s), g["fwd_zs"], "zs")
        _fwd_close(eng.eval_zsa("fixed_encoder", s, a), g["fwd_zsa"], "zsa")
        _fwd_close(eng.eval_zs("encoder", s), g["fwd_enc_zs"], "enc_zs")
        _fwd_close(eng.eval_zsa("encoder", s, a), g["fwd_enc_zsa"], "enc_zsa")
    else:
        for q in ("q1", "q2"):
            _fwd_close(eng.eval_q(q, s, a), g[f"fwd_{q}"][:, 0], q)
            if same(q, "target_" + q):
                _fwd_close(eng.eval_q("target_" + q, s, a), g[f"fwd_{q}"][:, 0], "t" + q)


def assert_moments(eng, g, t):
    ref = golden_moments(g, t)
    assert ref, "golden has no moments for step %d" % t
    for key, (pos, vals) in ref.items():
        base, which = key.rsplit(":", 1)
        net, pname = base.split(".", 1)
        got = eng.get_adam(net, pname, 0 if which == "m" else 1).ravel()
        got = got if pos is None else got[pos]
        got, r = np.asarray(got, np.float64), np.asarray(vals, np.float64).ravel()
        scale = max(np.abs(r).max(), 1e-30)
        d = np.abs(got - r)
        lim = 1e-4 * np.abs(r) + 1e-4 * scale
        assert (d <= lim).all(), (t, key, float(d.max()), float((d / lim).max()), scale)


@pytest.mark.parametrize("name", ALL)
def test_adam_moments_match_reference(name):
    """After steps 1 and 2 (single-step graphs), every optimizer's exp_avg / exp_avg_sq equals
    the reference's: the step's gradients (critics, encoder, actor, SAC log_alpha) pinned
    element-wise, not through losses."""
    g = load_golden(name)
    eng, rep, tp = engine_from_golden(g)
    eng.set_tapes(u=tp["u"][:2], eps=tp["eps"][:2], eps_pi=tp.get("eps_pi", None) if "eps_pi" in tp else None)
    for t in range(2):
        eng.step(1)
        assert_moments(eng, g, t)
    eng.set_tapes()


def test_sac_rsample_device():
    """sac_rsample.npz (SAC._rsample on fixed mean / log_std / eps, saturated tanh and clamped
    log_std rows included) through OP_SAC_ACTOR."""
    g = load_golden("sac_rsample")
    n, A = g["mean"].shape
    cfg = E.make_config(E.RLE_SAC, 17, A, 32, 16, seed=1, device=0)
    eng = E.Engine(cfg)
    act, lp = eng.sac_rsample(g["mean"], g["log_std"], g["eps"])
    assert np.abs(act - g["action"]).max() <= 2e-6
    ref = g["log_pi"].reshape(-1).astype(np.float64)
    assert (np.abs(lp - ref) <= 1e-4 + 1e-5 * np.abs(ref)).all(), np.abs(lp - ref).max()


def test_uniform_sampler_device_1m():
    """SimpleReplayMemory.sample index law at size 1M (uniform_sampler.npz s1000000)."""
    g = load_golden("uniform_sampler")
    n = 1_000_000
    rep = E.Replay(n, 3, 2, False)
    rep.fill_random(n, seed=0)
    assert rep.state()[1] == n
    np.testing.assert_array_equal(rep.sample_indices(g["s1000000_u"]), g["s1000000_ind"])
    rep.close()


def test_many_block_lap_trajectory_per_step():
    """TD7 Humanoid B=256 on a 65,536-row LAP replay (16 block sums), 12 steps, hard updates at
    steps 5 and 10: indices bit-exact, priorities rtol 1e-4 and value bounds after EVERY step
    (single-step graphs: the incremental fp64 block sums over many blocks)."""
    g = load_golden("td7_humanoid_64k")
    alg, env, H, B, Ncap, n_fill, n_steps, use_lap, seed, extra = parse(g)
    eng, rep, tp = engine_from_golden(g)
    eng.set_tapes(u=tp["u"][:n_steps], eps=tp["eps"][:n_steps])
    for t in range(n_steps):
        info = eng.step(1)[0]
        np.testing.assert_array_equal(eng.last_indices(), g["ind"][t])
        np.testing.assert_allclose(rep.get_priority(Ncap), expected_priorities(g, Ncap, t), rtol=1e-4, atol=1e-5)
        assert rep.state()[2] == pytest.approx(float(g[f"maxprio_{t}"]), rel=1e-4)
        np.testing.assert_allclose(eng.value_bounds(), g[f"vbounds_{t}"].astype(np.float32), rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(info[:3], g["info"][t], rtol=LOSS_RTOL, atol=1e-4, equal_nan=True)
    eng.set_tapes()


def _tiny_end_state_matches(eng, rep, g, infos):
    alg, env, H, B, Ncap, n_fill, n_steps, use_lap, seed, extra = parse(g)
    np.testing.assert_array_equal(eng.last_indices(), g["ind"][n_steps - 1])
    ref = g["info"]
    np.testing.assert_allclose(infos[:, :ref.shape[1]], ref, rtol=LOSS_RTOL, atol=1e-4, equal_nan=True)
    if use_lap:
        np.testing.assert_allclose(rep.get_priority(Ncap), g[f"prio_{n_steps - 1}"], rtol=1e-4, atol=1e-5)
    for key in g:
        if not key.startswith("out_") or key == "out_log_alpha" or ":" in key:
            continue
        net, pname = key[4:].split(".", 1)
        d = np.abs(eng.get_param(net, pname, g[key].shape) - g[key])
        assert (d <= 1e-5).mean() >= 0.99 and d.max() <= 2 * 3e-4 * n_steps + 1e-4, (key, d.max())


def test_async_seeds_each_match_their_golden():
    """three independent agents (TD7 LAP, TD3, SAC) enqueued with
    rle_step_async on their own streams, overlapping on one GPU; each ends on ITS OWN
    reference trajectory (indices, infos, priorities, parameters)."""
    runs = []
    for name in ("td7_tiny", "td3_tiny", "sac_tiny"):
        g = load_golden(name)
        eng, rep, tp = engine_from_golden(g)
        n = parse(g)[6]
        eng.set_tapes(u=tp["u"][:n], eps=tp["eps"][:n], eps_pi=tp.get("eps_pi", None) if "eps_pi" in tp else None)
        runs.append((g, eng, rep, n))
    for g, eng, rep, n in runs:  # all three enqueued before any sync
        eng.step_async(n)
    for g, eng, rep, n in runs:
        infos = eng.get_info(n)
        eng.set_tapes()
        _tiny_end_state_matches(eng, rep, g, infos)


def test_append_after_async_step_is_ordered():
    """A replay append issued right after rle_step_async waits for the enqueued steps (their
    priority scatter and block sums): the end state equals the synchronous sequence."""
    g = load_golden("td7_tiny")
    alg, env, H, B, Ncap, n_fill, n_steps, use_lap, seed, extra = parse(g)
    S, A, hi = spec.TASKS[env]
    rng = np.random.default_rng(5)
    k = 6
    new = (rng.standard_normal((k, S)), rng.uniform(-1, 1, (k, A)), rng.standard_normal(k),
           rng.standard_normal((k, S)), np.ones(k))
    ends = []
    for mode in ("sync", "async"):
        eng, rep, _ = engine_from_golden(g)
        if mode == "sync":
            eng.step(3)
        else:
            eng.step_async(3)
        rep.append(*new)
        eng.step(3)
        params = {(n, p): eng.get_param(n, p) for n, d in spec.agent_params(alg, S, A, H, 0).items() for p in d}
        ends.append((eng.last_indices(), rep.get_priority(), rep.state(), params))
    np.testing.assert_array_equal(ends[0][0], ends[1][0])
    np.testing.assert_array_equal(ends[0][1], ends[1][1])
    assert ends[0][2] == ends[1][2]
    for key in ends[0][3]:
        np.testing.assert_array_equal(ends[0][3][key], ends[1][3][key])


def test_host_reads_after_async_step_see_the_whole_burst():
    """rle_step_async leaves its levels in flight on the engine's own dispatch queue (direct AQL
    dispatch, which no HIP stream or device synchronize covers): the replay's host reads
    (priorities, max priority) and the engine's parameter reads issued right after it retire the
    burst first and see the same state as after a synchronous rle_step."""
    g = load_golden("td7_tiny")
    alg, env, H, B, Ncap, n_fill, n_steps, use_lap, seed, extra = parse(g)
    S, A, hi = spec.TASKS[env]
    ends = []
    for mode in ("sync", "async"):
        eng, rep, _ = engine_from_golden(g)
        if mode == "sync":
            eng.step(12)
        else:
            eng.step_async(12)
        prio = rep.get_priority()
        mx = rep.state()[2]
        eng.step_async(7)
        params = {(n, p): eng.get_param(n, p) for n, d in spec.agent_params(alg, S, A, H, 0).items() for p in d}
        eng.step_async(5)
        idx = eng.last_indices()
        ends.append((prio, mx, params, idx))
    np.testing.assert_array_equal(ends[0][0], ends[1][0])
    assert ends[0][1] == ends[1][1]
    for key in ends[0][2]:
        np.testing.assert_array_equal(ends[0][2][key], ends[1][2][key])
    np.testing.assert_array_equal(ends[0][3], ends[1][3])


def test_update_priority_below_one_keeps_sampling_exact():
    """Priorities < 1 written through update_priority (allowed by lap.py:66-69) recompute the
    block sums: the sampler then agrees with the searchsorted law on the new vector."""
    from oracle import replay as R

    n = 10000
    rep = E.Replay(n, 3, 2, True)
    rep.append(np.zeros((n, 3)), np.zeros((n, 2)), np.zeros(n), np.zeros((n, 3)), np.ones(n))
    p = spec.init_priorities(n, 3)
    rep.set_priority(p, float(p.max()))
    rng = np.random.default_rng(1)
    ind = rng.integers(0, n, 512)
    newp = rng.uniform(0.01, 0.5, 512).astype(np.float32)
    for i0 in range(0, 512, 256):
        rep.update_priority(ind[i0:i0 + 256], newp[i0:i0 + 256])
    exp = p.copy()
    exp[ind] = newp  # last writer wins within each call; calls in order
    np.testing.assert_array_equal(rep.get_priority(n), exp)
    u = rng.random(256, dtype=np.float32)
    np.testing.assert_array_equal(rep.sample_indices(u), R.lap_indices(exp, n, u))
    rep.close()
