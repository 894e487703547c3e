"""Parity of the HIP engine (through the C ABI) against reference goldens + the oracle.

Tolerances (SURVEY.md §4 evidence: fp32 reference vs fp64 of the same math):
forward outputs |d| <= 1e-5 + 1e-5 |ref|; per-step losses rel 1e-3 (harness.LOSS_RTOL) over <= 18 steps on identical
batches; parameters after k Adam steps: >= 99.9% of the elements (full size; 99% of each H=32
tensor) within 1e-5 of the reference, and every element within 2*lr*k + 1e-4 (Adam's first steps
are ~lr*sign(g): a gradient that rounds to the other sign in another summation order moves its
parameter 2*lr away, so the bulk criterion is what catches a wrong gradient).  Gradients
themselves are pinned through the Adam moments in test_parity_gpu.py.
"""

import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

E = pytest.importorskip("rl._engine")
from harness import LOSS_RTOL, engine_from_golden, parse, run_with_tapes  # noqa: E402
from oracle import spec  # noqa: E402
from test_oracle import expected_priorities  # noqa: E402

BULK = 0.999  # fraction of parameter elements within 1e-5 of the reference (full size)


def assert_params_close(got, ref, tol, what, bulk=BULK):
    d = np.abs(np.asarray(got, np.float64) - np.asarray(ref, np.float64))
    assert d.max() <= tol, (what, float(d.max()))
    assert (d <= 1e-5).mean() >= bulk, (what, float((d <= 1e-5).mean()))
    return int((d <= 1e-5).sum()), d.size


def test_lap_sampler_device():
    g = load_golden("lap_sampler")
    for n, seed in ((65536, 11), (1000000, 12), (1, 13), (4097, 14)):
        rep = E.Replay(n, 3, 2, True)
        rep.append(np.zeros((n, 3)), np.zeros((n, 2)), np.zeros(n), np.zeros((n, 3)), np.ones(n))
        p = spec.init_priorities(n, seed)
        rep.set_priority(p, float(p.max()))
        ind = rep.sample_indices(g[f"n{n}_u"])
        np.testing.assert_array_equal(ind, g[f"n{n}_ind"])
        rep.close()


def test_uniform_sampler_device():
    g = load_golden("uniform_sampler")
    for size in (1, 7, 25000):
        rep = E.Replay(size, 3, 2, False)
        rep.append(np.zeros((size, 3)), np.zeros((size, 2)), np.zeros(size), np.zeros((size, 3)),
                   np.ones(size))
        ind = rep.sample_indices(g[f"s{size}_u"])
        np.testing.assert_array_equal(ind, g[f"s{size}_ind"])
        rep.close()


def test_priority_scatter_last_writer_wins():
    g = load_golden("lap_sampler")
    rep = E.Replay(64, 3, 2, True)
    rep.append(np.zeros((64, 3)), np.zeros((64, 2)), np.zeros(64), np.zeros((64, 3)), np.ones(64))
    rep.set_priority(g["scatter_base"], 1.0)
    rep.update_priority(g["scatter_ind"], g["scatter_new"])
    np.testing.assert_array_equal(rep.get_priority(64), g["scatter_out"])
    assert rep.state()[2] == max(1.0, float(g["scatter_new"].max()))
    rep.reset_max_priority()
    assert rep.state()[2] == float(g["scatter_out"].max())


def test_replay_gather_roundtrip():
    rng = np.random.default_rng(0)
    n, S, A = 100, 17, 6
    rep = E.Replay(64, S, A, False)  # wraps around: rows 64..99 overwrite 0..35
    s = rng.standard_normal((n, S)).astype(np.float32)
    a = rng.standard_normal((n, A)).astype(np.float32)
    r = rng.standard_normal(n).astype(np.float32)
    s2 = rng.standard_normal((n, S)).astype(np.float32)
    d = (rng.random(n) > 0.5).astype(np.float32)
    rep.append(s, a, r, s2, d)
    ptr, size, _ = rep.state()
    assert (ptr, size) == (36, 64)
    ind = np.array([0, 35, 36, 63])
    gs, ga, gr, gs2, gd = rep.gather(ind)
    src = np.array([64, 99, 36, 63])
    np.testing.assert_array_equal(gs, s[src])
    np.testing.assert_array_equal(ga, a[src])
    np.testing.assert_array_equal(gr, r[src])
    np.testing.assert_array_equal(gs2, s2[src])
    np.testing.assert_array_equal(gd, d[src])


def _fwd_check(name):
    g = load_golden(name)
    alg, env, H, B, *_ = parse(g)
    S, A, hi = spec.TASKS[env]
    eng, rep, tp = engine_from_golden(g)
    s, a, *_ = rep.gather(np.arange(B))
    if alg == "td7":
        out = eng.act(s, A)
        ref = g["fwd_pi"]
    elif alg == "td3":
        out = np.tanh(eng.act(s, A))
        ref = g["fwd_pi"]
    else:
        out = eng.act(s, 2 * A)
        ref = np.concatenate([g["fwd_mean"], g["fwd_log_std"]], 1)
    n = ref.shape[0]
    np.testing.assert_allclose(out[:n], ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("name", ["td7_tiny", "td3_tiny", "sac_tiny", "td7_humanoid", "sac_humanoid",
                                  "td3_halfcheetah", "td3_tiny_deep", "sac_tiny_deep", "td7_tiny_zs", "td7_tiny_act",
                                  "td7_tiny_act_id", "td3_tiny_act", "sac_tiny_act"])
def test_forward_matches_reference(name):
    _fwd_check(name)


TINY = ["td7_tiny", "td7_tiny_nolap", "td3_tiny", "td3_tiny_lap", "sac_tiny", "sac_tiny_fixed", "td3_tiny_deep",
        "sac_tiny_deep", "td7_tiny_b100", "td3_tiny_b100", "sac_tiny_b100",  # (b100: a batch of 100, padded to 112)
        "td7_tiny_act", "td7_tiny_act_id", "td3_tiny_act", "sac_tiny_act",  # (act: hidden activations beyond the defaults)
        "td7_tiny_hp", "td3_tiny_hp", "sac_tiny_hp"]  # (hp: constructor hyper-parameters beyond the defaults)
FULL = ["td7_humanoid", "td7_ant", "td3_halfcheetah", "sac_humanoid", "td7_humanoid_64k", "td7_tiny_zs"]


@pytest.mark.parametrize("burst", [False, True], ids=["per_step", "burst"])
@pytest.mark.parametrize("name", TINY + FULL)
def test_step_trajectory_matches_reference(name, burst):
    """per_step: one rle_step(1) per step (single-step graphs), checked after every step.
    burst: the whole taped trajectory in one rle_step(n) (two-step graphs g_pair wherever a
    policy step is followed by a plain step, or any two SAC steps), checked at the end."""
    _trajectory(name, burst)


@pytest.mark.parametrize("variant", ["headdx", "qdot"])
@pytest.mark.parametrize("name", ["td7_tiny", "td7_tiny_nolap", "td7_humanoid"])
def test_td7_head_variants_match_reference(name, variant):
    """The TD7 critic loss head's alternative schedules (rle_plan fuse_off): without HEADDX the
    head runs as its own op (q from the EPI_QDOT row partials), without QDOT (implies no fusion)
    from the critics' last hidden activations with row dot products."""
    _trajectory(name, False, E.make_plan(fuse_off=[variant]))


@pytest.mark.parametrize("name", ["td7_tiny", "td3_tiny_lap", "sac_tiny", "td7_humanoid", "td3_halfcheetah",
                                  "sac_humanoid", "td7_tiny_act", "td7_tiny_act_id", "td3_tiny_act", "sac_tiny_act"])
def test_level_hazards(name, monkeypatch):
    """RLE_HAZARD=1: no byte that one op of a level stores is read or stored by another op of the
    same level (engine.cpp level_hazards: each op's accesses replayed from its descriptor) in any
    program the engine builds -- single-step, multi-step, hard-update and eval graphs; then one
    step runs."""
    monkeypatch.setenv("RLE_HAZARD", "1")
    g = load_golden(name)
    eng, rep, tp = engine_from_golden(g)
    run_with_tapes(eng, tp, 1, lambda t: None)


@pytest.mark.parametrize("name", ["td7_tiny", "td3_tiny_lap", "sac_tiny", "td7_humanoid", "td3_halfcheetah", "sac_humanoid",
                                  "td7_tiny_act", "td7_tiny_act_id", "td3_tiny_act", "sac_tiny_act"])
def test_gemm_address_audit(name, monkeypatch):
    """RLE_AUDIT=1: every byte range each GEMM op's workgroups can load or store (the kernel's
    address arithmetic replayed on the host, engine.cpp audit_gemm) lies inside one live device
    allocation, for every program the engine builds; then one step runs."""
    monkeypatch.setenv("RLE_AUDIT", "1")
    g = load_golden(name)
    eng, rep, tp = engine_from_golden(g)
    run_with_tapes(eng, tp, 1, lambda t: None)


def _trajectory(name, burst, plan=None):
    g = load_golden(name)
    alg, env, H, B, Ncap, n_fill, n_steps, use_lap, seed, extra = parse(g)
    eng, rep, tp = engine_from_golden(g, plan=plan)

    def check(t):
        np.testing.assert_array_equal(eng.last_indices(), g["ind"][t])
        if use_lap:
            exp = g[f"prio_{t}"] if f"prio_{t}" in g else expected_priorities(g, Ncap, t)
            np.testing.assert_allclose(rep.get_priority(Ncap), exp, rtol=1e-4, atol=1e-5)
        if f"vbounds_{t}" in g:
            np.testing.assert_allclose(eng.value_bounds(), g[f"vbounds_{t}"].astype(np.float32),
                                       rtol=1e-4, atol=1e-4)

    if burst:
        eng.set_tapes(u=tp["u"][:n_steps], eps=tp["eps"][:n_steps],
                      eps_pi=tp.get("eps_pi", None) if "eps_pi" in tp else None)
        infos = np.array(eng.step(n_steps))
        eng.set_tapes()
        check(n_steps - 1)
    else:
        infos = run_with_tapes(eng, tp, n_steps, check)
    ref = g["info"]
    k = ref.shape[1]
    np.testing.assert_array_equal(np.isnan(infos[:, :k]), np.isnan(ref))
    np.testing.assert_allclose(infos[:, :k], ref, rtol=LOSS_RTOL, atol=1e-4, equal_nan=True)
    # parameters after the trajectory
    tol = 2 * 3e-4 * n_steps + 1e-4
    within = total = 0
    for key in g:
        if not key.startswith("out_") or key == "out_log_alpha":
            continue
        net, rest = key[4:].split(".", 1)
        if rest.endswith(":digest"):  # full size: 64 sampled elements per tensor, pooled
            pname = rest[: -len(":digest")]
            v = eng.get_param(net, pname)
            base = key[: -len(":digest")]
            w, n = assert_params_close(v[g[base + ":pos"]], g[base + ":vals"], tol, key, bulk=0.0)
            within, total = within + w, total + n
        elif ":" not in rest:
            assert_params_close(eng.get_param(net, rest, g[key].shape), g[key], tol, key, bulk=0.99)
    if total:
        assert within / total >= BULK, (name, within / total)
    if "out_log_alpha" in g:  # SAC temperature (sac.py:55-60, 271-284)
        np.testing.assert_allclose(eng.get_param("tmp", "log_alpha"), g["out_log_alpha"].reshape(-1),
                                   rtol=1e-5, atol=1e-7)


def _synthetic_golden(alg, env, H, B, ncap, n_fill, n_steps, use_lap, seed, **extra):
    S, A, _ = spec.TASKS[env]
    g = {"meta_alg": np.array(alg), "meta_env": np.array(env),
         "meta": np.array([H, B, ncap, n_fill, n_steps, int(use_lap), seed]),
         "meta_extra_keys": np.array(list(extra), dtype="<U32"),
         "meta_extra_vals": np.array(list(extra.values()), np.float64)}
    for k, v in spec.tapes(alg, B, A, n_steps, seed + 3).items():
        g["tape_" + k] = v
    return g


def test_td7_humanoid_b1024_matches_oracle():
    """BASELINE config 4 (TD7 Humanoid, LAP, B=1024): the oracle (pinned at B=256 by the
    goldens) runs the same tapes on the host; the engine must agree step by step."""
    from oracle import agents
    from test_oracle import build_from_golden

    g = _synthetic_golden("td7", "Humanoid-v4", 256, 1024, 8192, 8192, 2, True, 77)
    alg, orc, orep, tp, n_steps, B = build_from_golden(g)
    eng, rep, tp2 = engine_from_golden(g)
    infos_ref, inds_ref = [], []
    prios = []

    def per_step(t):
        np.testing.assert_array_equal(eng.last_indices(), inds_ref[t])
        np.testing.assert_allclose(rep.get_priority(8192), prios[t], rtol=1e-4, atol=1e-5)

    for t in range(n_steps):
        i1, n1 = agents.run_steps(orc, alg, orep, {k: v[t:t + 1] for k, v in tp.items()}, 1, B)
        infos_ref += i1
        inds_ref += n1
        prios.append(orep.priority.copy())
    infos = run_with_tapes(eng, tp2, n_steps, per_step)
    keys = ["train/encoder", "train/q_fn", "train/policy"]
    ref = np.array([[np.nan if i[k] is None else i[k] for k in keys] for i in infos_ref])
    np.testing.assert_allclose(infos[:, :3], ref, rtol=LOSS_RTOL, atol=1e-4, equal_nan=True)
    tol = 2 * 3e-4 * n_steps + 1e-4
    for net, d in orc.nets().items():
        for name, v in d.items():
            assert_params_close(eng.get_param(net, name, tuple(v.shape)), v.detach().numpy(), tol, (net, name))


@pytest.mark.parametrize("name", ["td7_tiny", "td3_tiny_lap", "sac_tiny"])
def test_prefetched_batches_equal_fresh_draws(name):
    """Each step's graph prefetches the next step's batch (after its priority update);
    a run that re-draws every batch from scratch must be bit-identical."""
    g = load_golden(name)
    n = 6
    e1, r1, _ = engine_from_golden(g)
    e2, r2, _ = engine_from_golden(g)
    info1 = e1.step(n)
    info2 = []
    for _ in range(n):
        e2.set_counters(e2.counters())  # invalidates the prefetched batch
        info2.append(e2.step(1)[0])
    np.testing.assert_array_equal(info1, np.array(info2))
    np.testing.assert_array_equal(e1.last_indices(), e2.last_indices())
    np.testing.assert_array_equal(r1.get_priority(), r2.get_priority())
    alg = parse(g)[0]
    for net, params in spec.agent_params(alg, *spec.TASKS[parse(g)[1]][:2], parse(g)[2], 0).items():
        for pname in params:
            np.testing.assert_array_equal(e1.get_param(net, pname), e2.get_param(net, pname))


@pytest.mark.gpu
def test_step_async_equals_step_and_seeds_overlap():
    """rle_step_async (several seeds per GPU, one stream each) enqueues the
    same steps as rle_step: two engines stepped concurrently end bit-identical to a
    synchronous run of each."""
    g = load_golden("td7_tiny")
    runs = []
    for mode in ("sync", "async"):
        pair = [engine_from_golden(g) for _ in range(2)]
        if mode == "sync":
            for eng, _, _ in pair:
                eng.step(5)
        else:
            for _ in range(5):
                for eng, _, _ in pair:
                    eng.step_async(1)
            for eng, _, _ in pair:
                eng.synchronize()
        runs.append(pair)
    alg = parse(g)[0]
    for (e1, r1, _), (e2, r2, _) in zip(runs[0], runs[1]):
        np.testing.assert_array_equal(e1.last_indices(), e2.last_indices())
        np.testing.assert_array_equal(r1.get_priority(), r2.get_priority())
        for net, params in spec.agent_params(alg, *spec.TASKS[parse(g)[1]][:2], parse(g)[2], 0).items():
            for pname in params:
                np.testing.assert_array_equal(e1.get_param(net, pname), e2.get_param(net, pname))


# (td7_tiny hard-updates every 4 steps, so its bursts run single-step graphs around the hard
# updates; with target_update_rate 250 it replays the 6-step graph, LAP included)
@pytest.mark.parametrize("name", ["td7_tiny", "td7_tiny@tur250", "td7_tiny_nolap", "td3_tiny", "sac_tiny"])
def test_multistep_graphs_equal_single_steps(name):
    """rle_step(20) replays the K-step graphs (TD7 K=6, SAC K=8, TD3 K=16, plus single-step
    graphs around them); twenty rle_step(1) calls replay single-step graphs only.  Same ops on
    the same data, only grouped into other levels: bit-identical end state."""
    g = dict(load_golden(name.split("@")[0]))
    if name.endswith("@tur250"):
        g["meta_extra_vals"] = np.array([250.0])
    n = 20
    e1, r1, _ = engine_from_golden(g)
    e2, r2, _ = engine_from_golden(g)
    info1 = e1.step(n)
    info2 = np.array([e2.step(1)[0] for _ in range(n)])
    np.testing.assert_array_equal(info1, info2)
    np.testing.assert_array_equal(e1.last_indices(), e2.last_indices())
    np.testing.assert_array_equal(r1.get_priority(), r2.get_priority())
    np.testing.assert_array_equal(e1.counters(), e2.counters())
    alg, env, H = parse(g)[:3]
    for net, params in spec.agent_params(alg, *spec.TASKS[env][:2], H, 0).items():
        for pname in params:
            np.testing.assert_array_equal(e1.get_param(net, pname), e2.get_param(net, pname))


@pytest.mark.parametrize("name", ["td3_tiny", "td3_tiny_lap", "td3_halfcheetah"])
def test_td3_fused_policy_polyak_bitwise(name):
    """TD3's self-aliased target-policy Polyak (td3.py:200-204) applied in the actor's
    Adam epilogues (AdamArgs::ptau) is bit-identical to the standalone OP_POLYAK over the policy
    (plan fuse_off pipolyak), through single-step and 16-step graphs."""
    g = load_golden(name)
    n = 20
    e1, r1, _ = engine_from_golden(g)
    info1 = e1.step(n)
    e2, r2, _ = engine_from_golden(g, plan=E.make_plan(fuse_off=["pipolyak"]))
    info2 = e2.step(n)
    np.testing.assert_array_equal(info1, info2)
    np.testing.assert_array_equal(r1.get_priority(), r2.get_priority())
    alg, env, H = parse(g)[:3]
    for net, params in spec.agent_params(alg, *spec.TASKS[env][:2], H, 0).items():
        for pname in params:
            np.testing.assert_array_equal(e1.get_param(net, pname), e2.get_param(net, pname))


@pytest.mark.parametrize("name", ["td3_tiny", "td3_tiny_lap", "td3_halfcheetah", "sac_tiny", "sac_humanoid"])
def test_prelayer_bitwise(name):
    """The small-K first layers (TD3 actor and critics, K <= 48) recomputed in-tile by the layer
    after them, and SAC's gradient through the actor's raw head (K = 2A <= 48) recomputed in-tile by
    the next input-gradient GEMM (GemmArgs::has_pre 3, kernels.hip prelayer_fwd), give the same
    floats as reading the standalone op's output (plan fuse_off prelayer): chunk sums in the standalone
    op's split-K order, consumer chunks on ring_run's two accumulators, and the consumer ordered
    before the Adam update of the weights it recomputes with.  Tile widening off in both (level_cap), so
    the standalone first layers keep 16-wide tiles, and the consumers take the same 16-wide tiles
    (pl_tn 16; production widens them to 64, covered by the golden trajectories)."""
    g = load_golden(name)
    n = 20
    e1, r1, _ = engine_from_golden(g, plan=E.make_plan(level_cap=100000, pl_tn=16))
    info1 = e1.step(n)
    e2, r2, _ = engine_from_golden(g, plan=E.make_plan(["prelayer"], level_cap=100000, pl_tn=16))
    info2 = e2.step(n)
    np.testing.assert_array_equal(info1, info2)
    np.testing.assert_array_equal(r1.get_priority(), r2.get_priority())
    alg, env, H = parse(g)[:3]
    for net, params in spec.agent_params(alg, *spec.TASKS[env][:2], H, 0).items():
        for pname in params:
            np.testing.assert_array_equal(e1.get_param(net, pname), e2.get_param(net, pname))


@pytest.mark.parametrize("name", ["td3_tiny", "td3_tiny_lap", "td3_halfcheetah"])
def test_td3_twostage_bitwise(name):
    """TD3's target critics: their first layer, behind the pre-GEMM target action, recomputed in-tile by
    their second layer with the action segment computed in-tile first (GemmArgs::has_pre 4, kernels.hip
    PK 4), gives the floats of the standalone first layer (plan fuse_off twostage: a level of its own, in
    at most 32-wide tiles so that its split-K order is the pre-layer's chunk order).  Tile widening off
    in both and the consumers 16 wide (pl_tn 16), as test_prelayer_bitwise."""
    g = load_golden(name)
    n = 20
    e1, r1, _ = engine_from_golden(g, plan=E.make_plan(level_cap=100000, pl_tn=16))
    info1 = e1.step(n)
    e2, r2, _ = engine_from_golden(g, plan=E.make_plan(["twostage"], level_cap=100000, pl_tn=16))
    info2 = e2.step(n)
    assert "qdot+pl2" in e1.describe() and "qdot+pl2" not in e2.describe()
    np.testing.assert_array_equal(info1, info2)
    np.testing.assert_array_equal(r1.get_priority(), r2.get_priority())
    alg, env, H = parse(g)[:3]
    for net, params in spec.agent_params(alg, *spec.TASKS[env][:2], H, 0).items():
        for pname in params:
            np.testing.assert_array_equal(e1.get_param(net, pname), e2.get_param(net, pname))


@pytest.mark.parametrize("name", ["sac_tiny", "sac_tiny_fixed", "sac_humanoid"])
def test_sac_target_pre_bitwise(name):
    """SAC's target critics: their first layer recomputes the raw head and the target rsample a' for
    its rows in-tile (GemmArgs::has_pre 5, kernels.hip PK 5), in the standalone EPI_SACFWD op's reduction
    order (sacraw_*) and arithmetic, and sums a' on ring_run's two accumulators: the floats of reading
    the standalone op's output (plan fuse_off sacpre).  Equal tile widths in both (level_cap; pre_tn and
    pl_tn 16: on the tiny shapes, K <= 48, the unfused target critics take the pre-layer instead, whose
    consumer must keep the q partials' 16-wide tiles)."""
    g = load_golden(name)
    n = 20
    e1, r1, _ = engine_from_golden(g, plan=E.make_plan(level_cap=100000, pre_tn=16, pl_tn=16))
    info1 = e1.step(n)
    e2, r2, _ = engine_from_golden(g, plan=E.make_plan(["sacpre"], level_cap=100000, pre_tn=16, pl_tn=16))
    info2 = e2.step(n)
    assert "st+sacpre" in e1.describe() and "st+sacpre" not in e2.describe()
    np.testing.assert_array_equal(info1, info2)
    alg, env, H = parse(g)[:3]
    for net, params in spec.agent_params(alg, *spec.TASKS[env][:2], H, 0).items():
        for pname in params:
            np.testing.assert_array_equal(e1.get_param(net, pname), e2.get_param(net, pname))


# (TD7 with policy_freq 2 starts a 6-step graph at every odd step count n_runs whose window holds no
# hard update: n_runs = 1 -> steps 2..7 as one graph.  Humanoid 13: 1 + 6 + 6 steps, the headline
# program (B = 256, default planner, LAP over 4096 rows); B = 1024: 1 + 6 + 1, BASELINE config 4;
# target_update_rate 8, 16 steps: 1 + 6 + 1 (hard update) + 1 + 6 + 1 (hard update), so both
# 6-step graphs run on either side of a hard update)
BURSTS = [("td3", "HalfCheetah-v4", 18, 256, {}), ("sac", "Humanoid-v4", 9, 256, {}),
          ("td7", "Ant-v4", 8, 256, {}), ("td7", "Humanoid-v4", 13, 256, {}),
          ("td7", "Humanoid-v4", 8, 1024, {}), ("td7", "Humanoid-v4", 16, 256, {"target_update_rate": 8}),
          ("td7", "Humanoid-v4", 8, 512, {})]


@pytest.mark.parametrize("alg,env,n,B,extra", BURSTS,
                         ids=[f"{a}-{e.split('-')[0]}-n{n}-B{b}" + ("-tur8" if x else "") for a, e, n, b, x in BURSTS])
def test_multistep_burst_matches_oracle(alg, env, n, B, extra):
    """Full-size burst through the multi-step graphs (TD3: one 16-step graph + 2 single steps;
    SAC: one 8-step graph + 1; TD7: single steps + 6-step graphs, with the production tile planner)
    against the oracle stepped one taped step at a time on the same draws."""
    _burst_vs_oracle(alg, env, n, B, extra)


OPT_PLANS = {"priosample": dict(fuse_on=["priosample"]), "rb": dict(rb=1),
             "priosample+rb": dict(fuse_on=["priosample"], rb=1)}


@pytest.mark.parametrize("plan", list(OPT_PLANS))
@pytest.mark.parametrize("alg,env,n,B", [("td7", "Humanoid-v4", 13, 256), ("td7", "Humanoid-v4", 8, 1024),
                                         ("td3", "HalfCheetah-v4", 18, 256), ("sac", "Humanoid-v4", 9, 256)])
def test_opt_in_plans_match_oracle(alg, env, n, B, plan):
    """The opt-in plan choices on full-size bursts against the oracle: the LAP priority update applied by
    the next batch's sampler (RLE_FUSE_PRIOSAMPLE, exact: the same indices) and the register-blocked
    weight-gradient tiles (rle_plan rb)."""
    _burst_vs_oracle(alg, env, n, B, {}, E.make_plan(**OPT_PLANS[plan]))


@pytest.mark.parametrize("burst", [False, True], ids=["per_step", "burst"])
@pytest.mark.parametrize("name", ["td7_tiny", "td3_tiny_lap", "td7_humanoid", "td7_humanoid_64k"])
def test_fused_priority_sampler_matches_reference(name, burst):
    """RLE_FUSE_PRIOSAMPLE against the reference goldens: the sampler applies the step's priority
    update (duplicates: last writer wins) to the block sums, sub-block sums and priorities it reads,
    so every drawn index is the reference's (lap.py:45-69); the persisted priorities follow."""
    _trajectory(name, burst, E.make_plan(fuse_on=["priosample"]))


@pytest.mark.parametrize("alg,env,H", [("sac", "Humanoid-v4", 512), ("td3", "HalfCheetah-v4", 512)])
def test_wide_hidden_steps_match_oracle(alg, env, H):
    """Hidden width 512 (rle_create accepts H <= 512): the fusions whose kernels bound H (SAC's raw head
    + rsample in one GEMM epilogue, kernels.hip sacraw_*, R <= 256) fall back to their standalone ops
    instead of failing the program build.  Step 1's gradients (the Adam first moments) agree with the
    oracle's at 1e-5 of each tensor's max |g| (measured <= 5e-7), then 3 more steps' losses and parameters.
    (The parameters' bulk criterion is 0.98 here: at H = 512 SAC's critic input layers carry more
    near-zero gradients whose sign the fp32 summation order decides, and Adam's first steps move those
    elements by ~2 lr: measured 0.989 for q2.mlp.0 after 3 steps while step 1's gradients agree to 4.8e-7
    of the tensor max, tools/diag_wide.py.)"""
    from oracle import agents
    from test_oracle import build_from_golden

    n, B, ncap = 4, 256, 4096
    g = _synthetic_golden(alg, env, H, B, ncap, ncap, n, False, 91)
    _, orc, orep, tp, n_steps, B = build_from_golden(g)
    eng, rep, tp2 = engine_from_golden(g)
    eng.set_tapes(u=tp2["u"][:n], eps=tp2["eps"][:n], eps_pi=tp2.get("eps_pi", None))
    infos = [eng.step(1)[0]]
    i1, _ = agents.run_steps(orc, alg, orep, {k: v[0:1] for k, v in tp.items()}, 1, B)
    infos_ref = list(i1)
    for key, ref in agents.moments(orc).items():
        if not key.endswith(":m") or key.startswith("tmp."):
            continue
        net, pname = key[:-2].split(".", 1)
        got = eng.get_adam(net, pname, 0, ref.shape)
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-5 * float(np.abs(ref).max()), err_msg=key)
    infos += list(eng.step(n - 1))
    eng.set_tapes()
    for t in range(1, n):
        i1, _ = agents.run_steps(orc, alg, orep, {k: v[t:t + 1] for k, v in tp.items()}, 1, B)
        infos_ref += i1
    keys = {"td3": ["train/q_fn", "train/policy", "norm/policy"],
            "sac": ["train/q_fn", "tmp", "norm/tmp", "train/policy", "train/tmp", "entropy"]}[alg]
    ref = np.array([[np.nan if i[k] is None else i[k] for k in keys] for i in infos_ref], np.float64)
    np.testing.assert_allclose(np.array(infos)[:, :len(keys)], ref, rtol=LOSS_RTOL, atol=1e-4, equal_nan=True)
    tol = 2 * 3e-4 * n + 1e-4
    for net, d in orc.nets().items():
        for name, v in d.items():
            assert_params_close(eng.get_param(net, name, tuple(v.shape)), v.detach().numpy(), tol, (net, name),
                                bulk=0.98)


def _burst_vs_oracle(alg, env, n, B, extra, plan=None, H=256):
    from oracle import agents
    from test_oracle import build_from_golden

    ncap = 8192 if B > 256 else 4096
    g = _synthetic_golden(alg, env, H, B, ncap, ncap, n, alg == "td7", 91, **extra)
    _, orc, orep, tp, n_steps, B = build_from_golden(g)
    eng, rep, tp2 = engine_from_golden(g, plan=plan)
    launches0 = eng.launch_count()
    infos_ref = []
    for t in range(n_steps):
        i1, n1 = agents.run_steps(orc, alg, orep, {k: v[t:t + 1] for k, v in tp.items()}, 1, B)
        infos_ref += i1
    eng.set_tapes(u=tp2["u"][:n_steps], eps=tp2["eps"][:n_steps],
                  eps_pi=tp2.get("eps_pi", None) if "eps_pi" in tp2 else None)
    infos = np.array(eng.step(n_steps))
    eng.set_tapes()
    if alg == "td7":  # the multi-step graphs ran: fewer launches than single-step graphs would take (plain first)
        lp, lpl = eng.graph_stats()
        assert eng.launch_count() - launches0 < (n_steps + 1) // 2 * lpl + n_steps // 2 * lp, "no multi-step graph ran"
    np.testing.assert_array_equal(eng.last_indices(), n1[-1])
    keys = {"td7": ["train/encoder", "train/q_fn", "train/policy"],
            "td3": ["train/q_fn", "train/policy", "norm/policy"],
            "sac": ["train/q_fn", "tmp", "norm/tmp", "train/policy", "train/tmp", "entropy"]}[alg]
    ref = np.array([[np.nan if i[k] is None else i[k] for k in keys] for i in infos_ref], np.float64)
    k = ref.shape[1]
    np.testing.assert_allclose(infos[:, :k], ref, rtol=LOSS_RTOL, atol=1e-4, equal_nan=True)
    if alg == "td7":
        np.testing.assert_allclose(rep.get_priority(ncap), orep.priority, rtol=1e-4, atol=1e-5)
        vb = np.array([orc.value_max, orc.value_min, orc.vt_max, orc.vt_min], np.float32)  # td7.py:325-331
        np.testing.assert_allclose(eng.value_bounds(), vb, rtol=1e-4, atol=1e-4)
    tol = 2 * 3e-4 * n_steps + 1e-4
    for net, d in orc.nets().items():
        for name, v in d.items():
            assert_params_close(eng.get_param(net, name, tuple(v.shape)), v.detach().numpy(), tol, (net, name))


def _burst_launches(alg, env, n, plan=None):
    """rle_level launches of one n-step burst from the synthetic golden's start state."""
    g = _synthetic_golden(alg, env, 256, 256, 4096, 4096, n, alg == "td7", 91)
    eng, rep, tp = engine_from_golden(g, plan=plan)
    l0 = eng.launch_count()
    eng.set_tapes(u=tp["u"][:n], eps=tp["eps"][:n], eps_pi=tp.get("eps_pi", None) if "eps_pi" in tp else None)
    eng.step(n)
    return eng.launch_count() - l0


# (a burst's tail shorter than the multi-step graph runs as a 4- or 2-step program, engine.cpp kRemK:
# TD7 1 + 6 + 2 and 1 + 6 + 4 steps, TD3 16 + 4 (16 + 2: BURSTS' n = 18), SAC 8 + 4 + 2.  TD3 stops at 20: at
# step 22 this synthetic trajectory's first policy layer leaves the bulk criterion with single-step graphs too,
# bit for bit the same floats as the multi-step path -- tools/diag_wide.py -- the oracle's own drift)
REMAINDERS = [("td7", "Humanoid-v4", 9, 7), ("td7", "Humanoid-v4", 11, 7), ("td3", "HalfCheetah-v4", 20, 16),
              ("sac", "Humanoid-v4", 14, 8)]


@pytest.mark.parametrize("alg,env,n,n0", REMAINDERS, ids=[f"{a}-{e.split('-')[0]}-n{n}" for a, e, n, _ in REMAINDERS])
def test_remainder_programs_match_oracle(alg, env, n, n0):
    """A burst whose tail (n - n0 steps after the multi-step graphs) is shorter than the multi-step graph:
    the tail runs as one 4- / 2-step program (TD7 / TD3: fewer launches than the same steps as single-step
    graphs), and
    the whole burst matches the oracle stepped one taped step at a time."""
    _burst_vs_oracle(alg, env, n, 256, {})
    tail = _burst_launches(alg, env, n) - _burst_launches(alg, env, n0)
    single = E.make_plan(steps_per_graph=0)
    tail_single = _burst_launches(alg, env, n, single) - _burst_launches(alg, env, n0, single)
    # (SAC's multi-step programs run 12 levels per step, as its single-step graph: equal counts there)
    assert 0 < tail <= tail_single if alg == "sac" else 0 < tail < tail_single, (tail, tail_single)


@pytest.mark.parametrize("name", ["td7_humanoid", "td3_halfcheetah"])
def test_plan_is_explicit_and_env_free(name, monkeypatch):
    """The step program's plan (tile plan, schedule, fusions: everything that sets the fp32 summation
    order) comes only from rle_plan: the old environment switches change nothing, the plan given as
    fields or as bench.py's --plan text builds the same program bitwise, and a different level
    capacity builds a different one."""
    g = load_golden(name)
    n = 18

    def run(plan=None):
        e, r, _ = engine_from_golden(g, plan=plan)
        info = np.array(e.step(n))
        params = {(net, p): e.get_param(net, p) for net, ps in spec.agent_params(*_alg_dims(g)).items() for p in ps}
        return e, info, params

    def same(a, b):
        np.testing.assert_array_equal(a[1], b[1])
        for k in a[2]:
            np.testing.assert_array_equal(a[2][k], b[2][k], str(k))

    base = run()
    for var, val in (("RLE_LEVEL_CAP", "512"), ("RLE_PL_TN", "16"), ("RLE_PRE_TN", "16"), ("RLE_PAIR", "2"),
                     ("RLE_NO_HEADDX", "1"), ("RLE_FLAT_DIV", "1"), ("RLE_TN_MIN", "64"), ("RLE_AQL", "0"),
                     ("RLE_AQL_ACQ", "0"), ("RLE_AQL_REL", "0"), ("RLE_EAGER", "1"), ("RLE_NO_DPF", "1"),
                     ("RLE_XCD", "0")):
        monkeypatch.setenv(var, val)
    env = run()
    assert env[0].plan() == base[0].plan()
    same(base, env)
    monkeypatch.undo()
    fields = run(E.make_plan(level_cap=512))
    text = run(E.parse_plan("level_cap=512"))
    assert fields[0].plan()["level_cap"] == 512 and fields[0].plan() == text[0].plan()
    same(fields, text)
    assert fields[0].describe(0) != base[0].describe(0)  # (a narrower level capacity widens other tiles)
    # the launch choices (rle_plan dispatch / dpf / xcd) change how the levels reach the device, not a float
    for launch in (dict(dispatch=0, dpf=0, xcd=0), dict(dispatch=2)):
        other = run(E.make_plan(**launch))
        assert all(other[0].plan()[k] == v for k, v in launch.items())
        same(base, other)


def _alg_dims(g):
    alg, env, H = parse(g)[:3]
    return (alg, *spec.TASKS[env][:2], H, 0)


def _bench_program_run(n=13, plan=None):
    """TD7 Humanoid B=256, LAP over a 1,000,000-row replay, n taped steps on the engine (one burst, default plan)
    and on the oracle: (eng, rep, infos, orc, orep, infos_ref, inds, launches)."""
    from oracle import agents, replay

    S, A, hi = spec.TASKS["Humanoid-v4"]
    N, blk, B, H, seed = 1_000_000, 4096, 256, 256, 93
    data = spec.replay_data(S, A, blk, seed + 1, hi)
    scale = np.full(A, hi, np.float32)
    scale = (scale - (-scale)) / 2.0
    pat = {"state": data["state"].astype(np.float32), "next_state": data["next_state"].astype(np.float32),
           "action": (np.asarray(data["action"]) / scale - np.zeros(A, np.float32)).astype(np.float32),
           "reward": data["reward"].astype(np.float32), "done": data["done"].astype(np.float32)}
    p0 = spec.init_priorities(N, seed + 2)
    # engine side: the pattern appended in 64K-row chunks (the replay stores the normalised action)
    cfg = E.make_config(E.RLE_TD7, S, A, H, B, use_lap=True, seed=seed)
    eng = E.Engine(cfg, plan)
    nets = spec.agent_params("td7", S, A, H, seed)
    for net, params in nets.items():
        for name, v in params.items():
            eng.set_param(net, name, v)
    rep = E.Replay(N, S, A, True)
    chunk = 16 * blk
    tiled = {k: np.tile(v, (16,) + (1,) * (v.ndim - 1)) for k, v in pat.items()}
    for i in range(0, N, chunk):
        m = min(chunk, N - i)
        rep.append(tiled["state"][:m], tiled["action"][:m], tiled["reward"][:m], tiled["next_state"][:m],
                   tiled["done"][:m])
    del tiled
    rep.set_priority(p0, float(p0.max()))
    eng.bind(rep)
    # oracle side: the same rows written in place (Replay.append row by row would take minutes)
    orc = agents.make_oracle("td7", nets, A, True)
    orep = replay.Replay(N, S, A, scale, np.zeros(A, np.float32), True)
    for i in range(0, N, blk):
        m = min(blk, N - i)
        orep.state[i:i + m] = pat["state"][:m]
        orep.next_state[i:i + m] = pat["next_state"][:m]
        orep.action[i:i + m] = pat["action"][:m]
        orep.reward[i:i + m, 0] = pat["reward"][:m]
        orep.done[i:i + m, 0] = pat["done"][:m]
    orep.priority[:] = p0
    orep.max_priority = float(p0.max())
    orep.size, orep.ptr = N, 0
    tp = spec.tapes("td7", B, A, n, seed + 3)
    infos_ref, inds = [], []
    amb = {"q1": set(), "q2": set()}  # q01 outputs whose sign fp32 rounding decides (see the test)
    for t in range(n):
        ind = orep.sample_indices(tp["u"][t][:B])
        sa = np.concatenate([orep.state[ind], orep.action[ind]], 1).astype(np.float64)
        for qn, qp in (("q1", orc.q1), ("q2", orc.q2)):
            w, b = qp["q01.weight"].detach().numpy(), qp["q01.bias"].detach().numpy()
            x = sa @ w.T.astype(np.float64) + b
            amb[qn].update(np.nonzero((np.abs(x) < 1e-5).any(0))[0].tolist())
        i1, n1 = agents.run_steps(orc, "td7", orep, {k: v[t:t + 1] for k, v in tp.items()}, 1, B)
        infos_ref += i1
        inds += n1
    launches0 = eng.launch_count()
    eng.set_tapes(u=tp["u"], eps=tp["eps"])
    infos = np.array(eng.step(n))
    eng.set_tapes()
    return eng, rep, infos, orc, orep, infos_ref, inds, eng.launch_count() - launches0, amb


def test_bench_program_1m_lap_replay_matches_oracle():
    """The exact bench program (bench.py's default line): TD7 Humanoid B=256, LAP over a 1,000,000-row
    replay (245 priority blocks of 4096 in the sampler's block-sum scan), 13 steps = 1 single step + two
    6-step graphs with the default plan, against the oracle stepped one taped step at a time on the same
    draws.  Rows are a 4096-row pattern repeated over the replay (bench.py's fill shape, small host
    memory); the priorities are distinct over all 1M rows.  Indices bit-exact, every priority of the 1M
    rows (which records every index drawn) at rtol 1e-4, parameters at the module's bulk criterion.
    One exclusion, measured (tools/diag_bench1m.py): a critic's first-layer output x = q01([s, a]) that lies
    within fp32 rounding of zero (|x| < 1e-5; step 1 here has x = 2.0e-7 in q1's unit 55) gets its sign --
    which the AvgL1Norm backward's d|x|/dx = sign(x) uses -- from the summation order, so that unit's row of
    the q01 weight gradient differs from torch's (step-1 gradients elsewhere agree to < 1e-6 of each tensor's
    max), and the rows of such units are left out of the q01 bulk fraction (their max bound still holds)."""
    n, N = 13, 1_000_000
    eng, rep, infos, orc, orep, infos_ref, inds, launches, amb = _bench_program_run(n)
    lp, lpl = eng.graph_stats()
    assert launches < (n // 2) * (lp + lpl), "no multi-step graph ran"
    np.testing.assert_array_equal(eng.last_indices(), inds[-1])
    keys = ["train/encoder", "train/q_fn", "train/policy"]
    ref = np.array([[np.nan if i[k] is None else i[k] for k in keys] for i in infos_ref], np.float64)
    np.testing.assert_allclose(infos[:, :3], ref, rtol=LOSS_RTOL, atol=1e-4, equal_nan=True)
    np.testing.assert_allclose(rep.get_priority(N), orep.priority, rtol=1e-4, atol=1e-5)
    vb = np.array([orc.value_max, orc.value_min, orc.vt_max, orc.vt_min], np.float32)
    np.testing.assert_allclose(eng.value_bounds(), vb, rtol=1e-4, atol=1e-4)
    tol = 2 * 3e-4 * n + 1e-4
    for net, d in orc.nets().items():
        for name, v in d.items():
            got, ref = eng.get_param(net, name, tuple(v.shape)), v.detach().numpy()
            if net in amb and name.startswith("q01.") and amb[net]:
                keep = np.setdiff1d(np.arange(ref.shape[0]), sorted(amb[net]))
                assert_params_close(got, ref, tol, (net, name), bulk=0.0)
                got, ref = got[keep], ref[keep]
            assert_params_close(got, ref, tol, (net, name))


def _wide_run(B, n, plan, env="Humanoid-v4"):
    g = _synthetic_golden("td7", env, 256, B, 8192, 8192, n, True, 95)
    eng, rep, tp = engine_from_golden(g, plan=plan)
    eng.set_tapes(u=tp["u"][:n], eps=tp["eps"][:n])
    info = np.array(eng.step(n))
    eng.set_tapes()
    S, A, _ = spec.TASKS[env]
    params = {(net, p): eng.get_param(net, p) for net, ps in spec.agent_params("td7", S, A, 256, 0).items() for p in ps}
    return eng, rep, info, params


@pytest.mark.parametrize("B", [512, 1024])
def test_wide_tiles_bitwise_equal_16_row_tiles(B):
    """The 64-row LDS-staged tiles (rle_plan wide, kernels.hip gemm_wide) against the 16-row tiles at the same tile
    width (tn_min 64: every 16-row tile reduces all of K in one wave, on ring_run's two parity accumulators, as
    each wave of a wide tile does for each of its 4 column blocks): 8 TD7 Humanoid steps (single step + a 6-step
    graph + 1) end with bit-identical parameters, indices and priorities.  (The loss values may differ in the
    last bits: the 16-row tiles write their MSE / q-head loss partials in XCD tile order, the wide tiles in row
    order, and only the info row sums them.)"""
    e1, r1, i1, p1 = _wide_run(B, 8, E.make_plan(tn_min=64, wide=1, rb=1))
    e0, r0, i0, p0 = _wide_run(B, 8, E.make_plan(tn_min=64, wide=0, rb=1))
    assert ".w]" in e1.describe(0) and ".w]" not in e0.describe(0)
    np.testing.assert_array_equal(e1.last_indices(), e0.last_indices())
    np.testing.assert_array_equal(r1.get_priority(), r0.get_priority())
    for k in p1:
        np.testing.assert_array_equal(p1[k], p0[k], err_msg=str(k))
    np.testing.assert_allclose(i1, i0, rtol=1e-5, atol=1e-7, equal_nan=True)


@pytest.mark.parametrize("check", ["RLE_AUDIT", "RLE_HAZARD"])
def test_wide_tiles_audit_and_hazards(check, monkeypatch):
    """RLE_AUDIT / RLE_HAZARD over every program of a B = 512 TD7 engine with the 64-row tiles (the address replay
    covers a wide tile as the four 16-row tn-64 tiles it computes), then steps run."""
    monkeypatch.setenv(check, "1")
    e, r, info, _ = _wide_run(512, 3, E.make_plan(wide=1))
    assert ".w]" in e.describe(0)
    assert np.isfinite(info[:, :2]).all()
