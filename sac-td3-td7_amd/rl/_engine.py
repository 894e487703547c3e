"""ctypes binding of ``librle.so`` (C ABI in ``include/rle.h``).

This is the only bridge between the Python mirror of the reference interface
and the HIP engine.  There is no CPU fallback: if the library is missing or
fails to load, every engine-backed object raises.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

RLE_TD7, RLE_TD3, RLE_SAC = 0, 1, 2
RLE_EVAL_Q, RLE_EVAL_ZS, RLE_EVAL_ZSA = 0, 1, 2
INFO_MAX = 8

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RLE_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "librle.so")  # RLE_LIB: experiment builds

_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)
_i64p = ctypes.POINTER(ctypes.c_longlong)
_vp = ctypes.c_void_p
_cs = ctypes.c_char_p
_int = ctypes.c_int
_ll = ctypes.c_longlong


class Config(ctypes.Structure):
    """Mirror of ``rle_config`` (include/rle.h)."""

    _fields_ = [
        ("algo", _int), ("state_dim", _int), ("action_dim", _int), ("hidden", _int),
        ("batch", _int), ("use_lap", _int), ("discount", ctypes.c_float),
        ("policy_lr", ctypes.c_float), ("critic_lr", ctypes.c_float), ("tau", ctypes.c_float),
        ("target_policy_noise", ctypes.c_float), ("noise_clip", ctypes.c_float),
        ("policy_freq", _int), ("target_update_rate", _int), ("min_log_std", ctypes.c_float),
        ("max_log_std", ctypes.c_float), ("tmp", ctypes.c_float), ("seed", ctypes.c_ulonglong),
        ("device", _int), ("zs_dim", _int), ("n_hidden", _int), ("hidden_sizes", _int * 8),
        ("act_actor", _int), ("act_critic", _int), ("act_encoder", _int),
    ]


# rle_config act_* codes (include/rle.h RLE_ACT_*): 0 = the reference default of that net
ACT_CODES = {"default": 0, "relu": 1, "elu": 2, "identity": 3}


class Plan(ctypes.Structure):
    """Mirror of ``rle_plan`` (include/rle.h): the schedule / tile-plan / fusion choices that
    decide the step's fp32 summation order.  No environment variable changes it."""

    _fields_ = [
        ("level_cap", _int), ("steps_per_graph", _int), ("pre_tn", _int), ("pl_tn", _int), ("tn_min", _int),
        ("flat_div", _int), ("balance", _int), ("tiny_w", _int), ("uni_w", _int), ("tiny_wg", _int),
        ("sched_cap", _int), ("fuse_off", ctypes.c_uint), ("fuse_on", ctypes.c_uint), ("rb", _int),
        ("pl_w", _int), ("lap_w", _int), ("head_w", _int), ("adam_w", _int), ("wide", _int), ("lpt", _int),
        ("dispatch", _int), ("dpf", _int), ("xcd", _int),
    ]


# RLE_FUSE_* bits of rle_plan.fuse_off
FUSE = {"prelayer": 1 << 0, "pre": 1 << 1, "qdot": 1 << 2, "headdx": 1 << 3, "nbdefer": 1 << 4, "sacfwd": 1 << 5,
        "sacbwd": 1 << 6, "fold": 1 << 7, "pipolyak": 1 << 8, "endsplit": 1 << 9, "priosample": 1 << 10,
        "twostage": 1 << 11, "sacpre": 1 << 12, "normfin": 1 << 13}


def make_plan(fuse_off=(), fuse_on=(), **kw) -> Plan:
    """rle_plan_default() with the given fields changed; fuse_off / fuse_on: names of FUSE to switch off
    / on (fuse_on: the opt-in fusions, FUSE_OPT_IN)."""
    p = Plan()
    _check(lib().rle_plan_default(ctypes.byref(p)))
    for k, v in kw.items():
        if k not in dict(Plan._fields_):
            raise ValueError(f"unknown plan field {k!r}")
        setattr(p, k, int(v))
    def bits(names):
        b = 0
        for name in ([names] if isinstance(names, str) else names):
            b |= FUSE[name]
        return b

    p.fuse_off, p.fuse_on = bits(fuse_off), bits(fuse_on)
    return p


def parse_plan(text: str) -> Plan:
    """'level_cap=512,steps_per_graph=4,fuse_off=headdx+qdot' -> Plan (bench.py --plan, tools)."""
    kw, off, on = {}, (), ()
    for item in filter(None, (t.strip() for t in (text or "").split(","))):
        k, _, v = item.partition("=")
        if k == "fuse_off":
            off = tuple(filter(None, v.split("+")))
        elif k == "fuse_on":
            on = tuple(filter(None, v.split("+")))
        else:
            kw[k] = int(v)
    return make_plan(off, on, **kw)


def plan_dict(p: Plan) -> dict:
    d = {k: getattr(p, k) for k, _ in Plan._fields_}
    d["fuse_off"] = [n for n, b in FUSE.items() if p.fuse_off & b]
    d["fuse_on"] = [n for n, b in FUSE.items() if p.fuse_on & b]
    return d


# name -> (restype, argtypes)
SIGNATURES = {
    "rle_last_error": (_cs, []),
    "rle_replay_create": (_int, [_int, _ll, _int, _int, _int, ctypes.POINTER(_vp)]),
    "rle_replay_destroy": (_int, [_vp]),
    "rle_replay_append": (_int, [_vp, _f32p, _f32p, _f32p, _f32p, _f32p, _ll]),
    "rle_replay_state": (_int, [_vp, _i64p, _i64p, _f32p]),
    "rle_replay_fill_random": (_int, [_vp, _ll, ctypes.c_ulonglong]),
    "rle_replay_get_priority": (_int, [_vp, _f32p, _ll]),
    "rle_replay_set_priority": (_int, [_vp, _f32p, _ll, ctypes.c_float]),
    "rle_replay_sample_indices": (_int, [_vp, _int, _f32p, _i64p]),
    "rle_replay_update_priority": (_int, [_vp, _int, _i64p, _f32p]),
    "rle_replay_reset_max_priority": (_int, [_vp]),
    "rle_replay_gather": (_int, [_vp, _int, _i64p, _f32p, _f32p, _f32p, _f32p, _f32p]),
    "rle_create": (_int, [ctypes.POINTER(Config), ctypes.POINTER(_vp)]),
    "rle_destroy": (_int, [_vp]),
    "rle_plan_default": (_int, [ctypes.POINTER(Plan)]),
    "rle_set_plan": (_int, [_vp, ctypes.POINTER(Plan)]),
    "rle_get_plan": (_int, [_vp, ctypes.POINTER(Plan)]),
    "rle_bind_replay": (_int, [_vp, _vp]),
    "rle_param_numel": (_int, [_vp, _cs, _cs, _i64p]),
    "rle_get_param": (_int, [_vp, _cs, _cs, _f32p, _ll]),
    "rle_set_param": (_int, [_vp, _cs, _cs, _f32p, _ll]),
    "rle_get_adam": (_int, [_vp, _cs, _cs, _int, _f32p, _ll]),
    "rle_set_adam": (_int, [_vp, _cs, _cs, _int, _f32p, _ll]),
    "rle_get_counters": (_int, [_vp, _i64p]),
    "rle_set_counters": (_int, [_vp, _i64p]),
    "rle_get_act_counter": (_int, [_vp, ctypes.POINTER(ctypes.c_uint64)]),
    "rle_set_act_counter": (_int, [_vp, ctypes.c_uint64]),
    "rle_get_value_bounds": (_int, [_vp, _f32p]),
    "rle_set_value_bounds": (_int, [_vp, _f32p]),
    "rle_step": (_int, [_vp, _int, _f32p]),
    "rle_step_timed": (_int, [_vp, _int, _f32p]),
    "rle_step_async": (_int, [_vp, _int]),
    "rle_set_tapes": (_int, [_vp, _int, _f32p, _f32p, _f32p, _i64p]),
    "rle_last_indices": (_int, [_vp, _i64p]),
    "rle_act": (_int, [_vp, _f32p, _int, _f32p]),
    # (raw addresses: the per-env-step path skips ctypes pointer conversions)
    "rle_act_sample": (_int, [_vp, _vp, _int, _int, _vp, _vp]),
    "rle_set_action_map": (_int, [_vp, _f32p, _f32p, ctypes.c_float]),
    "rle_launch_count": (_int, [_vp, ctypes.POINTER(ctypes.c_longlong)]),
    "rle_graph_stats": (_int, [_vp, ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "rle_graph_describe": (_int, [_vp, _int, ctypes.c_char_p, _int]),
    "rle_graph_trace": (_int, [_vp, _int, ctypes.c_void_p, ctypes.c_longlong, ctypes.POINTER(ctypes.c_longlong)]),
    "rle_trace_stride": (_int, []),
    "rle_aql_wait_plan": (_int, [ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.POINTER(ctypes.c_double)]),
    "rle_aql_selftest": (_int, []),
    "rle_eval": (_int, [_vp, _int, _cs, _cs, _f32p, _f32p, _int, _f32p]),
    "rle_sac_rsample": (_int, [_vp, _f32p, _f32p, _f32p, _int, _f32p, _f32p]),
    "rle_get_info": (_int, [_vp, _int, _f32p]),
    "rle_copy_state": (_int, [_vp, _vp]),
    "rle_synchronize": (_int, [_vp]),
}


def lib():
    """Load librle.so (fails loudly: no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"HIP engine library not built: {LIB_PATH} (run __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        msg = lib().rle_last_error().decode(errors="replace")
        raise RuntimeError(f"rle error {rc}: {msg}")


def _fp(a):
    return None if a is None else a.ctypes.data_as(_f32p)


def _ip(a):
    return None if a is None else a.ctypes.data_as(_i64p)


def _f32(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a if shape is None else a.reshape(shape)


class Replay:
    """Device replay ring (HBM) with optional LAP priorities."""

    def __init__(self, capacity, state_dim, action_dim, lap, device=0):
        self.h = _vp()
        self.S, self.A, self.capacity, self.lap = state_dim, action_dim, capacity, bool(lap)
        _check(lib().rle_replay_create(device, capacity, state_dim, action_dim, int(lap), ctypes.byref(self.h)))

    def close(self):
        if self.h:
            _check(lib().rle_replay_destroy(self.h))
            self.h = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def append(self, state, action, reward, next_state, notdone):
        n = len(reward)
        s = _f32(state, (n, self.S))
        a = _f32(action, (n, self.A))
        r = _f32(reward, (n,))
        s2 = _f32(next_state, (n, self.S))
        d = _f32(notdone, (n,))
        _check(lib().rle_replay_append(self.h, _fp(s), _fp(a), _fp(r), _fp(s2), _fp(d), n))

    def state(self):
        p, s, m = _ll(), _ll(), ctypes.c_float()
        _check(lib().rle_replay_state(self.h, ctypes.byref(p), ctypes.byref(s), ctypes.byref(m)))
        return p.value, s.value, m.value

    def fill_random(self, count, seed):
        _check(lib().rle_replay_fill_random(self.h, count, seed))

    def get_priority(self, n=None):
        n = self.capacity if n is None else n
        out = np.empty(n, np.float32)
        _check(lib().rle_replay_get_priority(self.h, _fp(out), n))
        return out

    def set_priority(self, p, max_priority):
        p = _f32(p)
        _check(lib().rle_replay_set_priority(self.h, _fp(p), p.size, float(max_priority)))

    def sample_indices(self, u):
        u = _f32(u)
        out = np.empty(u.size, np.int64)
        _check(lib().rle_replay_sample_indices(self.h, u.size, _fp(u), _ip(out)))
        return out

    def update_priority(self, ind, p):
        ind = np.ascontiguousarray(ind, np.int64)
        p = _f32(p)
        _check(lib().rle_replay_update_priority(self.h, ind.size, _ip(ind), _fp(p)))

    def reset_max_priority(self):
        _check(lib().rle_replay_reset_max_priority(self.h))

    def gather(self, ind):
        ind = np.ascontiguousarray(ind, np.int64)
        n = ind.size
        s = np.empty((n, self.S), np.float32)
        a = np.empty((n, self.A), np.float32)
        r = np.empty(n, np.float32)
        s2 = np.empty((n, self.S), np.float32)
        d = np.empty(n, np.float32)
        _check(lib().rle_replay_gather(self.h, n, _ip(ind), _fp(s), _fp(a), _fp(r), _fp(s2), _fp(d)))
        return s, a, r, s2, d


class Engine:
    """One agent's device state + captured step graphs."""

    def __init__(self, cfg: Config, plan: Plan | None = None):
        self.cfg = cfg
        self.h = _vp()
        _check(lib().rle_create(ctypes.byref(cfg), ctypes.byref(self.h)))
        self.replay = None
        self._act_out = {}
        if plan is not None:
            self.set_plan(plan)

    def set_plan(self, plan: Plan):
        """Before the first step (the step programs are built with it)."""
        _check(lib().rle_set_plan(self.h, ctypes.byref(plan)))

    def plan(self) -> dict:
        """The plan in effect (defaults resolved)."""
        p = Plan()
        _check(lib().rle_get_plan(self.h, ctypes.byref(p)))
        return plan_dict(p)

    def close(self):
        if self.h:
            _check(lib().rle_destroy(self.h))
            self.h = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def bind(self, replay: Replay):
        _check(lib().rle_bind_replay(self.h, replay.h))
        self.replay = replay

    def numel(self, net, name):
        n = _ll()
        _check(lib().rle_param_numel(self.h, net.encode(), name.encode(), ctypes.byref(n)))
        return n.value

    def get_param(self, net, name, shape=None):
        n = self.numel(net, name)
        out = np.empty(n, np.float32)
        _check(lib().rle_get_param(self.h, net.encode(), name.encode(), _fp(out), n))
        return out if shape is None else out.reshape(shape)

    def set_param(self, net, name, value):
        v = _f32(value).ravel()
        _check(lib().rle_set_param(self.h, net.encode(), name.encode(), _fp(v), v.size))

    def get_adam(self, net, name, which, shape=None):
        n = self.numel(net, name)
        out = np.empty(n, np.float32)
        _check(lib().rle_get_adam(self.h, net.encode(), name.encode(), which, _fp(out), n))
        return out if shape is None else out.reshape(shape)

    def set_adam(self, net, name, which, value):
        v = _f32(value).ravel()
        _check(lib().rle_set_adam(self.h, net.encode(), name.encode(), which, _fp(v), v.size))

    def counters(self):
        out = np.zeros(6, np.int64)
        _check(lib().rle_get_counters(self.h, _ip(out)))
        return out

    def act_counter(self):
        v = ctypes.c_uint64(0)
        _check(lib().rle_get_act_counter(self.h, ctypes.byref(v)))
        return int(v.value)

    def set_act_counter(self, v):
        _check(lib().rle_set_act_counter(self.h, int(v)))

    def set_counters(self, c):
        c = np.ascontiguousarray(c, np.int64)
        _check(lib().rle_set_counters(self.h, _ip(c)))

    def value_bounds(self):
        out = np.zeros(4, np.float32)
        _check(lib().rle_get_value_bounds(self.h, _fp(out)))
        return out

    def set_value_bounds(self, v):
        v = _f32(v)
        _check(lib().rle_set_value_bounds(self.h, _fp(v)))

    def step(self, n, want_info=True):
        info = np.empty((max(n, 1), INFO_MAX), np.float32) if want_info else None
        _check(lib().rle_step(self.h, n, _fp(info)))
        return info[:n] if want_info else None

    def step_timed(self, n):
        """n steps, no info readback; returns GPU ms from HIP events on the engine stream."""
        ms = ctypes.c_float()
        _check(lib().rle_step_timed(self.h, n, ctypes.byref(ms)))
        return ms.value

    def step_async(self, n):
        """Enqueue n steps on the engine's stream; no host sync, no info readback."""
        _check(lib().rle_step_async(self.h, n))

    def set_tapes(self, u=None, eps=None, eps_pi=None, ind=None):
        if u is None and ind is None:
            _check(lib().rle_set_tapes(self.h, 0, None, None, None, None))
            return
        n = (u if u is not None else ind).shape[0]
        _check(lib().rle_set_tapes(
            self.h, n, _fp(None if u is None else _f32(u)), _fp(None if eps is None else _f32(eps)),
            _fp(None if eps_pi is None else _f32(eps_pi)),
            _ip(None if ind is None else np.ascontiguousarray(ind, np.int64))))

    def last_indices(self):
        out = np.empty(self.cfg.batch, np.int64)
        _check(lib().rle_last_indices(self.h, _ip(out)))
        return out

    def act(self, obs, width):
        obs = _f32(obs)
        if obs.ndim == 1:
            obs = obs[None]
        if obs.ndim != 2 or obs.shape[1] != self.cfg.state_dim:
            raise ValueError(f"act: observation shape {obs.shape}, expected (n, {self.cfg.state_dim})")
        n = obs.shape[0]
        out = np.empty((n, width), np.float32)
        _check(lib().rle_act(self.h, _fp(obs), n, _fp(out)))
        return out

    def set_action_map(self, scale, bias, exploration_noise=0.1):
        """Environment action map of act_sample: a * scale + bias, and the TD7 / TD3
        exploration noise std (rle_set_action_map)."""
        scale = _f32(np.broadcast_to(np.asarray(scale, np.float32), (self.cfg.action_dim,)))
        bias = _f32(np.broadcast_to(np.asarray(bias, np.float32), (self.cfg.action_dim,)))
        _check(lib().rle_set_action_map(self.h, _fp(scale), _fp(bias), float(exploration_noise)))

    def act_sample(self, obs, mode, eps=None):
        """Agent.sample on the device (rle_act_sample): obs [S] or [n][S] -> environment
        actions [n][A].  mode 0 deterministic, 1 Philox exploration noise, 2 noise tape eps."""
        x = obs if (type(obs) is np.ndarray and obs.dtype == np.float32 and obs.flags.c_contiguous) else _f32(obs)
        # the kernel reads n rows of state_dim floats from this address: shapes are checked here,
        # as the reference's first Linear would reject them
        if x.ndim not in (1, 2) or x.shape[-1] != self.cfg.state_dim:
            raise ValueError(f"act_sample: observation shape {x.shape}, expected ({self.cfg.state_dim},) "
                             f"or (n, {self.cfg.state_dim})")
        n = 1 if x.ndim == 1 else x.shape[0]
        if not 1 <= n <= 1024:
            raise ValueError(f"act_sample: {n} observations (1..1024)")
        out = self._act_out.get(n)
        if out is None:
            out = self._act_out[n] = np.empty((n, self.cfg.action_dim), np.float32)
        e = 0
        if mode == 2:
            eps = _f32(eps).reshape(n, self.cfg.action_dim)
            e = eps.ctypes.data
        rc = lib().rle_act_sample(self.h, x.ctypes.data, n, mode, e, out.ctypes.data)
        if rc:
            _check(rc)
        return out

    def eval_q(self, net, s, a, enc="fixed_encoder"):
        """estimate_q_value of critic `net` on (s, a) -> [n] (TD7: embeddings of encoder `enc`)."""
        s = _f32(s)
        n = s.shape[0]
        a = _f32(a, (n, self.cfg.action_dim))
        out = np.empty(n, np.float32)
        enc_b = enc.encode() if (enc and self.cfg.algo == RLE_TD7) else None
        _check(lib().rle_eval(self.h, RLE_EVAL_Q, net.encode(), enc_b, _fp(s), _fp(a), n, _fp(out)))
        return out

    def eval_zs(self, enc, s):
        """encode_state of encoder `enc` (TD7) -> [n][zs_dim]."""
        s = _f32(s)
        n = s.shape[0]
        out = np.empty((n, self.cfg.zs_dim or self.cfg.hidden), np.float32)
        _check(lib().rle_eval(self.h, RLE_EVAL_ZS, enc.encode(), None, _fp(s), None, n, _fp(out)))
        return out

    def eval_zsa(self, enc, s, a):
        """encode_state_action(encode_state(s), a) of encoder `enc` (TD7) -> [n][zs_dim]."""
        s = _f32(s)
        n = s.shape[0]
        a = _f32(a, (n, self.cfg.action_dim))
        out = np.empty((n, self.cfg.zs_dim or self.cfg.hidden), np.float32)
        _check(lib().rle_eval(self.h, RLE_EVAL_ZSA, enc.encode(), None, _fp(s), _fp(a), n, _fp(out)))
        return out

    def sac_rsample(self, mean, log_std, eps):
        """SAC._rsample through the device op: (tanh action [n][A], log_pi [n])."""
        mean = _f32(mean)
        n, A = mean.shape
        log_std, eps = _f32(log_std, (n, A)), _f32(eps, (n, A))
        act = np.empty((n, A), np.float32)
        lp = np.empty(n, np.float32)
        _check(lib().rle_sac_rsample(self.h, _fp(mean), _fp(log_std), _fp(eps), n, _fp(act), _fp(lp)))
        return act, lp

    def get_info(self, n):
        """Info rows of the last step / step_async call."""
        out = np.empty((max(n, 1), INFO_MAX), np.float32)
        _check(lib().rle_get_info(self.h, n, _fp(out)))
        return out[:n]

    def launch_count(self):
        n = ctypes.c_longlong()
        _check(lib().rle_launch_count(self.h, ctypes.byref(n)))
        return n.value

    def graph_stats(self):
        a, b = _int(), _int()
        _check(lib().rle_graph_stats(self.h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def describe(self, which=0):
        buf = ctypes.create_string_buffer(1 << 16)
        _check(lib().rle_graph_describe(self.h, which, buf, len(buf)))
        return buf.value.decode()

    def trace(self, which=0):
        """Per-workgroup phase timestamps of the last replay of graph `which` (RLE_TRACE=1):
        (workgroups, 4) -- or 16 columns from a -DRLE_TRACE_FINE build."""
        n = ctypes.c_longlong()
        _check(lib().rle_graph_trace(self.h, which, None, 0, ctypes.byref(n)))
        stride = lib().rle_trace_stride()
        if n.value == 0:
            return np.zeros((0, stride), np.uint64)
        out = np.zeros((n.value, stride), np.uint64)
        _check(lib().rle_graph_trace(self.h, which, out.ctypes.data, out.size, ctypes.byref(n)))
        return out

    def copy_state_from(self, other: "Engine"):
        _check(lib().rle_copy_state(self.h, other.h))

    def synchronize(self):
        _check(lib().rle_synchronize(self.h))


def make_config(algo, state_dim, action_dim, hidden, batch, use_lap=False, discount=0.99,
                policy_lr=3e-4, critic_lr=3e-4, tau=0.005, target_policy_noise=0.2,
                noise_clip=0.5, policy_freq=2, target_update_rate=250, min_log_std=-20.0,
                max_log_std=2.0, tmp=-1.0, seed=0, device=0, zs_dim=0, hidden_sizes=None,
                act_actor="default", act_critic="default", act_encoder="default") -> Config:
    """``hidden``: TD7 hdim, TD3 / SAC the width of both hidden layers; ``zs_dim`` (TD7, 0 = hidden) and
    ``hidden_sizes`` (TD3 / SAC: make_mlp's list, 2..6 layers) give the other net shapes (include/rle.h).
    ``act_*``: hidden activations, "relu" / "elu" / "identity" (make_mlp action_fn=None) or "default"."""
    hs = list(hidden_sizes) if hidden_sizes is not None else []
    if hs and not 2 <= len(hs) <= 6:
        raise ValueError(f"hidden_sizes {hs}: 2..6 hidden layers")
    acts = []
    for a in (act_actor, act_critic, act_encoder):
        if a not in ACT_CODES:
            raise ValueError(f"activation {a!r}: one of {sorted(ACT_CODES)}")
        acts.append(ACT_CODES[a])
    return Config(algo, state_dim, action_dim, hs[-1] if hs else hidden, batch, int(use_lap), discount,
                  policy_lr, critic_lr, tau, target_policy_noise, noise_clip, policy_freq, target_update_rate,
                  min_log_std, max_log_std, tmp, seed, device, zs_dim, len(hs),
                  (_int * 8)(*(hs + [0] * (8 - len(hs)))), *acts)
