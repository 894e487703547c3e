"""Pin the CPU oracle against golden vectors produced by the reference itself."""

import numpy as np
import pytest
import torch

from conftest import acts_of, load_golden, shape_of
from oracle import agents, replay, spec
from oracle import nets as N

torch.set_num_threads(1)


def _close(a, b, rtol=1e-5, atol=1e-6):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


def test_lap_sampler_law():
    g = load_golden("lap_sampler")
    for n, seed in ((65536, 11), (1000000, 12), (1, 13), (4097, 14)):
        p = spec.init_priorities(n, seed)
        ind = replay.lap_indices(p, n, g[f"n{n}_u"])
        np.testing.assert_array_equal(ind, g[f"n{n}_ind"])


def test_lap_scatter_last_writer_wins():
    g = load_golden("lap_sampler")
    r = replay.Replay(64, 1, 1, np.ones(1, np.float32), np.zeros(1, np.float32), True)
    r.priority[:] = g["scatter_base"]
    r.size = 64
    r.ind = g["scatter_ind"]
    r.update_priority(g["scatter_new"])
    np.testing.assert_array_equal(r.priority, g["scatter_out"])
    assert r.max_priority == max(1.0, float(g["scatter_new"].max()))


def test_uniform_sampler_law():
    g = load_golden("uniform_sampler")
    for size in (1, 7, 25000, 1000000):
        ind = replay.uniform_indices(size, g[f"s{size}_u"])
        np.testing.assert_array_equal(ind, g[f"s{size}_ind"])
        assert ind.min() >= 0 and ind.max() <= size - 1


def test_sac_rsample():
    g = load_golden("sac_rsample")
    a, lp = N.gaussian_tanh(torch.from_numpy(g["mean"]), torch.from_numpy(g["log_std"]),
                            torch.from_numpy(g["eps"]))
    np.testing.assert_array_equal(a.numpy(), g["action"])
    np.testing.assert_array_equal(lp.numpy(), g["log_pi"])


def build_from_golden(g):
    alg = str(g["meta_alg"])
    env = str(g["meta_env"])
    H, B, Ncap, n_fill, n_steps, use_lap, seed = (int(x) for x in g["meta"])
    S, A, hi = spec.TASKS[env]
    extra = dict(zip([str(k) for k in g["meta_extra_keys"]], g["meta_extra_vals"].tolist()))
    extra = {("discount" if k == "discount_factor" else k): (int(v) if k in ("target_update_rate", "policy_freq") else v)
             for k, v in extra.items()}  # (the reference's constructor names -> the oracle's)
    nets = spec.agent_params(alg, S, A, H, seed, **shape_of(g))
    orc = agents.make_oracle(alg, nets, A, bool(use_lap), acts=acts_of(g), **extra)
    scale = np.full(A, hi, np.float32)
    bias = np.zeros(A, np.float32)
    rep = replay.Replay(Ncap, S, A, (scale - (-scale)) / 2.0, bias, bool(use_lap))
    data = spec.replay_data(S, A, n_fill, seed + 1, hi)
    for i in range(n_fill):
        rep.append(data["state"][i], data["action"][i], float(data["reward"][i]),
                   data["next_state"][i], float(data["done"][i]))
    if use_lap:
        p0 = spec.init_priorities(Ncap, seed + 2)
        p0[rep.size:] = 0.0
        rep.priority[:] = p0
        rep.max_priority = float(p0.max())
    tp = {k[5:]: v for k, v in g.items() if k.startswith("tape_")}
    return alg, orc, rep, tp, n_steps, B


TINY = ["td7_tiny", "td7_tiny_nolap", "td3_tiny", "td3_tiny_lap", "sac_tiny", "sac_tiny_fixed", "td3_tiny_deep",
        "sac_tiny_deep", "td7_tiny_b100", "td3_tiny_b100", "sac_tiny_b100",  # (b100: a batch of 100, padded to 112)
        "td7_tiny_act", "td7_tiny_act_id", "td3_tiny_act", "sac_tiny_act",  # (act: hidden activations beyond the defaults)
        "td7_tiny_hp", "td3_tiny_hp", "sac_tiny_hp"]  # (hp: constructor hyper-parameters beyond the defaults)
FULL = ["td7_humanoid", "td7_ant", "td3_halfcheetah", "sac_humanoid", "td7_humanoid_64k", "td7_tiny_zs"]


def golden_moments(g, t):
    """{key: (positions or None, values)} of the reference's Adam moments after step t."""
    out = {}
    pre = f"adam{t}_"
    for k in g:
        if not k.startswith(pre) or k.endswith(":digest") or k.endswith(":pos"):
            continue
        if k.endswith(":vals"):
            key = k[len(pre):-len(":vals")]
            out[key] = (g[pre + key + ":pos"], g[k])
        else:
            out[k[len(pre):]] = (None, g[k])
    return out


def expected_priorities(g, ncap, t_last):
    """Full priority vector after step t_last from a golden that stores only the rows each step
    wrote (prioi_t = priority[ind_t] after step t; other rows keep their values, lap.py:66-69)."""
    H, B, Ncap, n_fill, n_steps, use_lap, seed = (int(x) for x in g["meta"])
    p = spec.init_priorities(Ncap, seed + 2)
    p[n_fill:] = 0.0
    for t in range(t_last + 1):
        p[g["ind"][t]] = g[f"prioi_{t}"]
    return p[:ncap]


def assert_moments_close(got, ref, what, rtol=1e-4):
    """|d| <= rtol |ref| + rtol * max|ref| of the tensor (m, v of one parameter)."""
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    scale = max(np.abs(ref).max(), 1e-30)
    d = np.abs(got - ref)
    assert (d <= rtol * np.abs(ref) + rtol * scale).all(), (what, d.max(), scale)


@pytest.mark.parametrize("name", TINY + FULL)
def test_oracle_matches_reference(name):
    g = load_golden(name)
    alg, orc, rep, tp, n_steps, B = build_from_golden(g)
    keys = [str(k) for k in g["info_keys"]]
    infos, inds = [], []
    for t in range(n_steps):
        i1, n1 = agents.run_steps(orc, alg, rep, {k: v[t:t + 1] for k, v in tp.items()}, 1, B)
        infos += i1
        inds += n1
        np.testing.assert_array_equal(inds[t], g["ind"][t])
        got = [np.nan if infos[t][k] is None else infos[t][k] for k in keys]
        _close(got, g["info"][t], rtol=1e-5, atol=1e-6)
        if f"prio_{t}" in g:
            _close(rep.priority, g[f"prio_{t}"], rtol=1e-6, atol=0)
        if f"prioi_{t}" in g:
            _close(rep.priority, expected_priorities(g, rep.priority.size, t), rtol=1e-6, atol=0)
            assert rep.max_priority == pytest.approx(float(g[f"maxprio_{t}"]), rel=1e-6)
        ref_m = golden_moments(g, t)
        if ref_m:
            mom = agents.moments(orc)
            assert set(ref_m) == set(mom), sorted(set(ref_m) ^ set(mom))
            for key, (pos, vals) in ref_m.items():
                got = mom[key].ravel() if pos is None else mom[key].ravel()[pos]
                assert_moments_close(got, np.ravel(vals), (t, key), rtol=1e-5)
        if f"vbounds_{t}" in g:
            _close([orc.value_max, orc.value_min, orc.vt_max, orc.vt_min], g[f"vbounds_{t}"])
    nets = orc.nets()
    for key in g:
        if not key.startswith("out_") or key == "out_log_alpha":
            continue
        net, rest = key[4:].split(".", 1)
        if rest.endswith(":digest"):
            pname = rest[: -len(":digest")]
            v = nets[net][pname].detach().numpy().ravel()
            _close(v[g[key[: -len(':digest')] + ':pos']], g[key[: -len(':digest')] + ':vals'],
                   rtol=1e-5, atol=1e-6)
        elif ":" not in rest:
            _close(nets[net][rest].detach().numpy(), g[key], rtol=1e-5, atol=1e-6)
    if "out_log_alpha" in g:
        _close(orc.log_alpha.detach().numpy(), g["out_log_alpha"])


@pytest.mark.parametrize("name", TINY)
def test_oracle_bitwise_on_this_host(name):
    """Same torch-CPU ops in the same order => bitwise equal infos/params here."""
    g = load_golden(name)
    alg, orc, rep, tp, n_steps, B = build_from_golden(g)
    infos, _ = agents.run_steps(orc, alg, rep, tp, n_steps, B)
    keys = [str(k) for k in g["info_keys"]]
    got = np.array([[np.nan if infos[t][k] is None else infos[t][k] for k in keys]
                    for t in range(n_steps)])
    np.testing.assert_array_equal(got, g["info"])
