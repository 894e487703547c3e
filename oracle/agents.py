"""Functional restatement of the three agents' gradient step (TEST INFRASTRUCTURE ONLY).

Each ``*Oracle.step(batch, replay, eps...)`` reproduces one
``Agent.train_ops`` call of the reference in the same order:

* TD7: ``rl/agent/td7.py:287-332`` (encoder -> critics (+LAP priority) ->
  policy every ``policy_freq`` -> hard update every ``target_update_rate``).
* TD3: ``rl/agent/td3.py:206-242`` (critics -> policy + Polyak when
  ``n_runs % policy_freq == 0`` *before* incrementing).
* SAC: ``rl/agent/sac.py:251-295`` (critics -> policy + temperature ->
  Polyak on critics).

Adam is restated from torch 2.x ``_single_tensor_adam`` (non-capturable path;
the reference pins torch 2.0.1, same update law): m.lerp_(g, 1-b1);
v = v*b2 + (1-b2) g^2; p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps).

Reference quirks kept: target policy aliases the online policy (Q1), TD3
"Polyak" on the aliased policy (Q2), TD7 value clipping starting at [0, 0]
(Q3), not-done masks (Q4), TD7 actor loss over both critics (Q11), LAP
Huber/priority (Q12), cadence (Q10), SAC logged policy loss includes the
temperature loss (Q15).
"""

from __future__ import annotations

import numpy as np
import torch

from . import nets as N


class Adam:
    """torch.optim.Adam defaults (betas 0.9/0.999, eps 1e-8, no decay)."""

    def __init__(self, params, lr=3e-4, betas=(0.9, 0.999), eps=1e-8):
        self.params = list(params)
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.t = 0

    @torch.no_grad()
    def step(self, grads):
        self.t += 1
        bc1 = 1 - self.b1 ** self.t
        bc2 = 1 - self.b2 ** self.t
        step_size = self.lr / bc1
        bc2_sqrt = bc2 ** 0.5
        for p, g, m, v in zip(self.params, grads, self.m, self.v):
            m.lerp_(g, 1 - self.b1)
            v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            denom = (v.sqrt() / bc2_sqrt).add_(self.eps)
            p.addcdiv_(m, denom, value=-step_size)


def _params(d):
    return {k: torch.tensor(np.asarray(v), dtype=torch.float32).requires_grad_(True)
            for k, v in d.items()}


def _grads(loss, params: dict):
    keys = list(params.keys())
    gs = torch.autograd.grad(loss, [params[k] for k in keys])
    return gs


def _tt(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))


def _acts(acts, defaults):
    """{"actor", "critic", "encoder"} -> activation functions (nets.ACTS names; missing: the reference
    defaults, sale.py:25,67,97 / mlp.py:13)."""
    acts = dict(acts or {})
    return {k: N.ACTS[acts.get(k) or d] for k, d in defaults.items()}


class TD7Oracle:
    def __init__(self, nets, discount=0.99, policy_lr=3e-4, critic_lr=3e-4,
                 target_update_rate=250, target_policy_noise=0.2, noise_clip=0.5,
                 policy_freq=2, use_lap=True, acts=None):
        a = _acts(acts, {"actor": "relu", "critic": "elu", "encoder": "elu"})
        self.ap, self.ac, self.ae = a["actor"], a["critic"], a["encoder"]
        self.enc = _params(nets["encoder"])
        self.pi = _params(nets["policy"])
        self.q1 = _params(nets["q1"])
        self.q2 = _params(nets["q2"])
        self.tq1 = _params(nets["target_q1"])
        self.tq2 = _params(nets["target_q2"])
        self.fe = _params(nets["fixed_encoder"])
        self.fet = _params(nets["fixed_encoder_target"])
        self.gamma, self.tr = discount, target_update_rate
        self.noise, self.clip, self.pf, self.lap = target_policy_noise, noise_clip, policy_freq, use_lap
        self.opt_pi = Adam(self.pi.values(), lr=policy_lr)
        self.opt_q = Adam(list(self.q1.values()) + list(self.q2.values()), lr=critic_lr)
        self.opt_enc = Adam(self.enc.values(), lr=policy_lr)
        self.value_max, self.value_min = -1e8, 1e8
        self.vt_max, self.vt_min = 0.0, 0.0
        self.n_runs = 0

    def step(self, batch, replay, eps):
        """td7.py:287-332 with target-smoothing noise ``eps`` (randn, [B, A])."""
        self.n_runs += 1
        info = {}
        s, a, s2 = _tt(batch["state"]), _tt(batch["action"]), _tt(batch["next_state"])
        r, nd = _tt(batch["reward"]), _tt(batch["done"])
        # encoder (td7.py:246-257, 299-303)
        zs_, zsa_, actor, critic = self._fns()
        with torch.no_grad():
            zs_next = zs_(self.enc, s2)
        zsa = zsa_(self.enc, zs_(self.enc, s), a)
        loss_e = (zsa - zs_next).pow(2.0).mean()
        self.opt_enc.step(_grads(loss_e, self.enc))
        info["train/encoder"] = float(loss_e.detach())
        # critics (td7.py:175-244)
        with torch.no_grad():
            zs2 = zs_(self.fet, s2)
            noise = (_tt(eps) * self.noise).clamp(-self.clip, self.clip)
            a2 = (actor(self.pi, s2, zs2) + noise).clamp(-1.0, 1.0)
            zsa2 = zsa_(self.fet, zs2, a2)
            nq1 = critic(self.tq1, s2, a2, zsa2, zs2)
            nq2 = critic(self.tq2, s2, a2, zsa2, zs2)
            nv = torch.cat([nq1, nq2], -1).min(1, keepdim=True)[0].clamp(self.vt_min, self.vt_max)
            y = r + self.gamma * nv * nd
            self.value_max = max(self.value_max, float(y.max()))
            self.value_min = min(self.value_min, float(y.min()))
            zs = zs_(self.fe, s)
            zsa_f = zsa_(self.fe, zs, a)
        q1 = critic(self.q1, s, a, zsa_f, zs)
        q2 = critic(self.q2, s, a, zsa_f, zs)
        if self.lap:
            td = torch.cat([(q1 - y).abs(), (q2 - y).abs()], 1)
            loss_q = torch.where(td < 1.0, 0.5 * td.pow(2), 1.0 * td).sum(1).mean()
            prio = td.max(1)[0].clamp(1.0).pow(0.4).view(-1)
            replay.update_priority(prio.detach().numpy())
        else:
            loss_q = torch.mean((y - q1) ** 2.0) * 0.5 + torch.mean((y - q2) ** 2.0) * 0.5
        g = _grads(loss_q, {**{"a" + k: v for k, v in self.q1.items()},
                            **{"b" + k: v for k, v in self.q2.items()}})
        self.opt_q.step(g)
        info["train/q_fn"] = float(loss_q.detach())
        # policy (td7.py:259-276, 319-324)
        info["train/policy"] = None
        if self.n_runs % self.pf == 0:
            zs = zs_(self.fe, s)
            act = actor(self.pi, s, zs)
            zsa_p = zsa_(self.fe, zs, act)
            qa = critic(self.q1, s, act, zsa_p, zs)
            qb = critic(self.q2, s, act, zsa_p, zs)
            loss_p = -torch.cat([qa, qb], -1).mean()
            self.opt_pi.step(_grads(loss_p, self.pi))
            info["train/policy"] = float(loss_p.detach())
        # hard update (td7.py:278-285, 325-331)
        if self.n_runs % self.tr == 0:
            with torch.no_grad():
                for dst, src in ((self.tq1, self.q1), (self.tq2, self.q2),
                                 (self.fet, self.fe), (self.fe, self.enc)):
                    for k in dst:
                        dst[k].copy_(src[k])
            self.vt_max, self.vt_min = self.value_max, self.value_min
            if self.lap:
                replay.reset_max_priority()
        return info

    def _fns(self):
        """The four SALE forwards with this agent's activations."""
        ae, ap, ac = self.ae, self.ap, self.ac
        return (lambda p, s: N.sale_zs(p, s, ae), lambda p, zs, a: N.sale_zsa(p, zs, a, ae),
                lambda p, s, zs: N.sale_actor(p, s, zs, ap),
                lambda p, s, a, zsa, zs: N.sale_critic(p, s, a, zsa, zs, ac))


class TD3Oracle:
    def __init__(self, nets, discount=0.99, policy_lr=3e-4, critic_lr=3e-4,
                 target_policy_noise=0.2, noise_clip=0.5, policy_freq=2, tau=0.005,
                 use_lap=False, acts=None):
        a = _acts(acts, {"actor": "relu", "critic": "relu"})
        self.ap, self.ac = a["actor"], a["critic"]
        self.pi = _params(nets["policy"])
        self.q1 = _params(nets["q1"])
        self.q2 = _params(nets["q2"])
        self.tq1 = _params(nets["target_q1"])
        self.tq2 = _params(nets["target_q2"])
        self.gamma, self.noise, self.clip, self.pf, self.tau = (
            discount, target_policy_noise, noise_clip, policy_freq, tau)
        self.lap = use_lap
        self.opt_pi = Adam(self.pi.values(), lr=policy_lr)
        self.opt_q = Adam(list(self.q1.values()) + list(self.q2.values()), lr=critic_lr)
        self.n_runs = 0

    def step(self, batch, replay, eps):
        """td3.py:206-242."""
        info = {}
        s, a, s2 = _tt(batch["state"]), _tt(batch["action"]), _tt(batch["next_state"])
        r, nd = _tt(batch["reward"]), _tt(batch["done"])
        with torch.no_grad():
            noise = (_tt(eps) * self.noise).clamp(-self.clip, self.clip)
            a2 = (torch.tanh(N.mlp(self.pi, s2, self.ap)) + noise).clamp(-1.0, 1.0)
            nv = torch.min(N.mlp_critic(self.tq1, s2, a2, self.ac), N.mlp_critic(self.tq2, s2, a2, self.ac))
            y = r + self.gamma * nv * nd
        q1, q2 = N.mlp_critic(self.q1, s, a, self.ac), N.mlp_critic(self.q2, s, a, self.ac)
        if self.lap:
            d1, d2 = (q1 - y).abs(), (q2 - y).abs()

            def hub(d):
                return torch.where(d < 1.0, 0.5 * d.pow(2), 1.0 * d).mean()

            loss_q = hub(d1) + hub(d2)
            prio = torch.max(d1, d2).clamp(1.0).pow(0.4).view(-1)
            replay.update_priority(prio.detach().numpy())
        else:
            loss_q = torch.mean((y - q1) ** 2.0) * 0.5 + torch.mean((y - q2) ** 2.0) * 0.5
        g = _grads(loss_q, {**{"a" + k: v for k, v in self.q1.items()},
                            **{"b" + k: v for k, v in self.q2.items()}})
        self.opt_q.step(g)
        info["train/q_fn"] = float(loss_q.detach())
        info["train/policy"] = None
        info["norm/policy"] = None
        if self.n_runs % self.pf == 0:
            act = torch.tanh(N.mlp(self.pi, s, self.ap))
            loss_p = -torch.min(N.mlp_critic(self.q1, s, act, self.ac), N.mlp_critic(self.q2, s, act, self.ac)).mean()
            gp = _grads(loss_p, self.pi)
            info["train/policy"] = float(loss_p.detach())
            tot = 0.0
            for gg in gp:  # nn/utils.py:13-19: sum of per-tensor L2 norms
                tot += torch.norm(gg, p=2)
            info["norm/policy"] = float(tot)
            self.opt_pi.step(gp)
            with torch.no_grad():  # td3.py:194-204 (policy term aliases itself, Q2)
                for src, dst in ((self.q1, self.tq1), (self.q2, self.tq2), (self.pi, self.pi)):
                    for k in src:
                        dst[k].copy_(self.tau * src[k] + dst[k] * (1 - self.tau))
        self.n_runs += 1
        return info


class SACOracle:
    def __init__(self, nets, A, discount=0.99, policy_lr=3e-4, critic_lr=3e-4, tau=0.005,
                 min_log_std=-20.0, max_log_std=2.0, tmp=-1.0, acts=None):
        a = _acts(acts, {"actor": "relu", "critic": "relu"})
        self.ap, self.ac = a["actor"], a["critic"]
        self.pi = _params(nets["policy"])
        self.q1 = _params(nets["q1"])
        self.q2 = _params(nets["q2"])
        self.tq1 = _params(nets["target_q1"])
        self.tq2 = _params(nets["target_q2"])
        self.log_alpha = torch.zeros(1, requires_grad=True)
        self.A = A
        self.target_entropy = -A
        self.gamma, self.tau = discount, tau
        self.lo, self.hi = min_log_std, max_log_std
        self.opt_pi = Adam(self.pi.values(), lr=policy_lr)
        self.opt_q = Adam(list(self.q1.values()) + list(self.q2.values()), lr=critic_lr)
        self.opt_t = Adam([self.log_alpha], lr=policy_lr)
        # sac.py:55-60: tmp >= 0 is a fixed temperature, a plain Python float (no optimizer,
        # no temperature loss); multiplying an fp32 tensor by it rounds it to fp32 (Q of torch)
        self.auto = tmp < 0.0
        self.tmp = None if self.auto else float(tmp)
        self.n_runs = 0

    def _dist(self, s, eps):
        out = N.mlp(self.pi, s, self.ap)
        mean, log_std = out.chunk(2, -1)
        return N.gaussian_tanh(mean, log_std, _tt(eps), self.lo, self.hi)

    def step(self, batch, replay, eps, eps_pi):
        """sac.py:251-295."""
        info = {}
        s, a, s2 = _tt(batch["state"]), _tt(batch["action"]), _tt(batch["next_state"])
        r, nd = _tt(batch["reward"]), _tt(batch["done"])
        with torch.no_grad():
            a2, lp2 = self._dist(s2, eps)
            nq = torch.min(N.mlp_critic(self.tq1, s2, a2, self.ac), N.mlp_critic(self.tq2, s2, a2, self.ac))
            alpha = self.log_alpha.exp() if self.auto else self.tmp  # sac.py:189
            y = r + self.gamma * (nq - alpha * lp2) * nd
        q1, q2 = N.mlp_critic(self.q1, s, a, self.ac), N.mlp_critic(self.q2, s, a, self.ac)
        loss_q = torch.mean((y - q1) ** 2.0) * 0.5 + torch.mean((y - q2) ** 2.0) * 0.5
        g = _grads(loss_q, {**{"a" + k: v for k, v in self.q1.items()},
                            **{"b" + k: v for k, v in self.q2.items()}})
        self.opt_q.step(g)
        info["train/q_fn"] = float(loss_q.detach())
        act, lp = self._dist(s, eps_pi)
        qv = torch.min(N.mlp_critic(self.q1, s, act, self.ac), N.mlp_critic(self.q2, s, act, self.ac))
        alpha_d = self.log_alpha.exp().detach() if self.auto else self.tmp  # sac.py:227-228
        policy_obj = torch.mean(-qv + lp * alpha_d)
        entropy = -(lp.mean().detach())
        if not self.auto:  # sac.py:228-236, 271-290 without the temperature terms
            keys = list(self.pi.keys())
            gs = torch.autograd.grad(policy_obj, [self.pi[k] for k in keys])
            self.opt_pi.step(gs)
            info["train/policy"] = float(policy_obj.detach())
            info["entropy"] = float(entropy)
            self._polyak()
            self.n_runs += 1
            return info
        tmp_obj = torch.mean(self.log_alpha.exp() * (-lp.detach() - self.target_entropy))
        obj = policy_obj
        obj += tmp_obj  # in place: logged policy loss includes the temperature loss (Q15)
        keys = list(self.pi.keys())
        gs = torch.autograd.grad(obj, [self.pi[k] for k in keys] + [self.log_alpha])
        info["tmp"] = float(self.log_alpha.detach().exp())
        info["norm/tmp"] = float(gs[-1])
        self.opt_pi.step(gs[:-1])
        self.opt_t.step([gs[-1]])
        info["train/policy"] = float(policy_obj.detach())
        info["train/tmp"] = float(tmp_obj.detach())
        info["entropy"] = float(entropy)
        self._polyak()
        self.n_runs += 1
        return info

    def _polyak(self):
        with torch.no_grad():  # sac.py:243-249
            for src, dst in ((self.q1, self.tq1), (self.q2, self.tq2)):
                for k in src:
                    dst[k].copy_(self.tau * src[k] + dst[k] * (1 - self.tau))

    def nets(self):
        return {"policy": self.pi, "q1": self.q1, "q2": self.q2,
                "target_q1": self.tq1, "target_q2": self.tq2}


def _nets(self):
    out = {}
    for name, attr in (("encoder", "enc"), ("policy", "pi"), ("q1", "q1"), ("q2", "q2"),
                       ("target_q1", "tq1"), ("target_q2", "tq2"), ("fixed_encoder", "fe"),
                       ("fixed_encoder_target", "fet")):
        if hasattr(self, attr):
            out[name] = getattr(self, attr)
    return out


TD7Oracle.nets = _nets
TD3Oracle.nets = _nets

# optimizer -> the nets whose parameters it holds, in parameter order (td7.py:127-133,
# td3.py:102-107, sac.py:109-123)
_OPT_NETS = {"opt_pi": ("policy",), "opt_q": ("q1", "q2"), "opt_enc": ("encoder",)}


def moments(oracle):
    """Adam exp_avg / exp_avg_sq keyed "{net}.{param}:m|v" (the engine's rle_get_adam layout);
    only optimizers that have stepped (torch creates the state at the first step)."""
    out = {}
    nets = oracle.nets()
    for attr, owners in _OPT_NETS.items():
        opt = getattr(oracle, attr, None)
        if opt is None or opt.t == 0:
            continue
        keys = [f"{n}.{k}" for n in owners for k in nets[n]]
        for key, m, v in zip(keys, opt.m, opt.v):
            out[key + ":m"] = m.detach().numpy().copy()
            out[key + ":v"] = v.detach().numpy().copy()
    if isinstance(oracle, SACOracle) and oracle.opt_t.t:
        out["tmp.log_alpha:m"] = oracle.opt_t.m[0].detach().numpy().copy()
        out["tmp.log_alpha:v"] = oracle.opt_t.v[0].detach().numpy().copy()
    return out


def make_oracle(alg, nets, A, use_lap, acts=None, **hp):
    """acts: hidden activations {"actor", "critic", "encoder" (TD7)} by nets.ACTS name (None: defaults)."""
    if alg == "td7":
        return TD7Oracle(nets, use_lap=use_lap, acts=acts, **hp)
    if alg == "td3":
        return TD3Oracle(nets, use_lap=use_lap, acts=acts, **hp)
    return SACOracle(nets, A, acts=acts, **hp)


def run_steps(oracle, alg, replay, tapes, n_steps, B):
    """run_train_ops (run.py:87-96) with tape-driven sampling/noise."""
    infos, inds = [], []
    for t in range(n_steps):
        ind = replay.sample_indices(tapes["u"][t][:B])
        batch = replay.gather(ind)
        if alg == "sac":
            info = oracle.step(batch, replay, tapes["eps"][t], tapes["eps_pi"][t])
        else:
            info = oracle.step(batch, replay, tapes["eps"][t])
        infos.append(info)
        inds.append(ind)
    return infos, inds
