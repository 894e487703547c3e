"""Shared machinery of the engine-backed TD7 / TD3 / SAC agents.

Each agent owns one ``rle_engine`` (include/rle.h): all networks, target copies,
Adam moments and step counters live in HBM and a gradient step is one replay of
a captured HIP graph.  The Python side keeps the reference's interface
(rl/agent/abc.py:16-55, rl/sampler.py:14-19): construction arguments,
``train_ops(batch, replay_buffer)`` returning the same info dict, ``sample``,
``to``, ``load_state_dict``, pickling (``save``/``load``/``deepcopy``).

There is no CPU path: constructing an agent without the HIP library raises.
"""

from __future__ import annotations

import math

import numpy as np

from rl import _engine as E
from rl.agent.abc import Agent
from rl.nn.layout import AGENT_COPIES, AGENT_NETS, init_agent, layers
from rl.replay_memory.base import BaseReplayMemory, DeviceBatch
from rl.sampler import Sampler
from rl.utils.envs import get_action_bias_scale, get_state_action_dims


def _device_index(device) -> int:
    if device is None:
        return 0
    if isinstance(device, int):
        return device
    s = str(device)
    if s == "cpu":
        return -1
    if s.startswith("cuda") or s.startswith("hip"):
        return int(s.split(":")[1]) if ":" in s else 0
    raise ValueError(f"unsupported device {device!r}")


class EngineAgent(Agent, Sampler):
    ALG = ""          # "td7" | "td3" | "sac"
    ALGO = -1         # RLE_TD7 / RLE_TD3 / RLE_SAC
    OPTIM_NETS: tuple = ()
    NULLABLE: tuple = ()  # info keys the reference sets to None on non-policy steps

    def _setup(self, env_id, *, hidden, batch_size, seed, device, make_nn, make_nn_kwargs, cfg):
        custom = None
        shape = {}  # net shapes beyond the defaults: zs_dim (SALE), hidden_sizes (make_mlp)
        acts = {}  # hidden activations of the make_nn nets (make_config act_*)
        if make_nn is not None:  # td7.py:56-61 / td3.py:53-56 / sac.py:47-50 (rl.nn.modules nets only)
            from rl.nn.modules import nets_from_make_nn

            S, A = get_state_action_dims(env_id)
            hidden, shape, custom, acts = nets_from_make_nn(self.ALG, make_nn, S, A, make_nn_kwargs)
            make_nn_kwargs = {}
        hdim = make_nn_kwargs.pop("hdim", None)
        zs = make_nn_kwargs.pop("zs_dim", None)
        hs = make_nn_kwargs.pop("hidden_sizes", None)
        if make_nn_kwargs:
            raise TypeError(f"unsupported arguments {sorted(make_nn_kwargs)}")
        if self.ALG == "td7":
            if hs is not None:
                raise TypeError("hidden_sizes is a make_mlp argument (TD3 / SAC); TD7 takes hdim / zs_dim")
            if hdim is not None:
                hidden = hdim
            if zs is not None and int(zs) != int(hidden):
                shape["zs_dim"] = int(zs)
        else:
            if hdim is not None or zs is not None:
                raise TypeError("hdim / zs_dim are SALE arguments (TD7); TD3 / SAC take hidden_sizes")
            if hs is not None:
                from rl.nn.modules import _sizes

                hs = _sizes(hs)
                shape["hidden_sizes"] = [int(h) for h in hs]
                hidden = hs[-1]
        if shape.get("hidden_sizes") == [int(hidden)] * 2:
            shape = {}  # (the default shape)
        self.shape = shape
        self.acts = acts
        self.env_id = env_id
        self.state_dim, self.action_dim = get_state_action_dims(env_id)
        self.action_bias, self.action_scale = get_action_bias_scale(env_id)
        self.hidden = int(hidden)
        if seed is None:
            import torch

            seed = torch.initial_seed() & 0x7FFFFFFF
        self.seed = int(seed)
        self._cfg = dict(cfg)
        self._device = max(_device_index(device), 0)
        self.device = device if device is not None else "cuda:0"
        self._replay = None
        self.engine = self._new_engine(int(batch_size))
        if custom is not None:  # the hook's nets, and their construction-time copies (td7.py:62-66)
            nets = dict(custom)
            for name, src in AGENT_COPIES[self.ALG].items():
                nets[name] = {k: v.copy() for k, v in custom[src].items()}
        else:
            nets = init_agent(self.ALG, self.state_dim, self.action_dim, self.hidden, self.seed, **self.shape)
        self._import({"params": nets})

    # ---- engine lifecycle ----------------------------------------------------
    def _new_engine(self, batch):
        c = E.make_config(self.ALGO, self.state_dim, self.action_dim, self.hidden, batch, seed=self.seed,
                          device=self._device, **self._cfg, **self.shape, **getattr(self, "acts", {}))
        return E.Engine(c)

    @property
    def batch_size(self) -> int:
        return self.engine.cfg.batch

    def _rebuild(self, batch=None, device=None):
        st = self._export()
        if device is not None:
            self._device = device
        self.engine.close()
        self.engine = self._new_engine(self.batch_size if batch is None else batch)
        self._import(st)
        self._replay = None

    def _prepare(self, replay: BaseReplayMemory, batch: int):
        if not isinstance(replay, BaseReplayMemory):
            raise TypeError("engine agents train from rl.replay_memory device replays")
        if self._cfg.get("use_lap") and not replay.LAP:
            raise AssertionError("use_lap=True needs a LAPReplayMemory (td7.py:307-309)")
        if replay.device != self._device:
            raise ValueError(f"replay on device {replay.device}, agent on {self._device}")
        if batch != self.batch_size or (self._replay is not None and self._replay is not replay):
            self._rebuild(batch)
        if self._replay is not replay:
            self.engine.bind(replay.dev)
            self._replay = replay
        replay.flush()

    # ---- parameters / state ---------------------------------------------------
    def _param_names(self):
        out = []
        for net, kind in AGENT_NETS[self.ALG].items():
            o = 2 * self.action_dim if (self.ALG == "sac" and net == "policy") else None
            names = []
            for prefix, fin, fout in layers(kind, self.state_dim, self.action_dim, self.hidden, o, **self.shape):
                names += [(prefix + ".weight", (fout, fin)), (prefix + ".bias", (fout,))]
            out.append((net, names))
            for copy, src in AGENT_COPIES[self.ALG].items():
                if src == net:
                    out.append((copy, names))
        return out

    def _export(self):
        e = self.engine
        params = {net: {n: e.get_param(net, n, shp) for n, shp in names} for net, names in self._param_names()}
        adam = {}
        for net, names in self._param_names():
            if net in self.OPTIM_NETS:
                adam[net] = {n: (e.get_adam(net, n, 0, shp), e.get_adam(net, n, 1, shp)) for n, shp in names}
        if self.ALG == "sac":
            params["tmp"] = {"log_alpha": e.get_param("tmp", "log_alpha")}
            adam["tmp"] = {"log_alpha": (e.get_adam("tmp", "log_alpha", 0), e.get_adam("tmp", "log_alpha", 1))}
        return {"params": params, "adam": adam, "counters": e.counters(), "vbounds": e.value_bounds(),
                "act_counter": e.act_counter()}

    def _import(self, st):
        e = self.engine
        for net, d in st["params"].items():
            for n, v in d.items():
                e.set_param(net, n, np.asarray(v, np.float32))
        for net, d in st.get("adam", {}).items():
            for n, (m, v) in d.items():
                e.set_adam(net, n, 0, m)
                e.set_adam(net, n, 1, v)
        if "counters" in st:
            e.set_counters(st["counters"])
        if "vbounds" in st:
            e.set_value_bounds(st["vbounds"])
        if "act_counter" in st:
            e.set_act_counter(st["act_counter"])

    def state_dict(self):
        """{net: {param name: ndarray}} in the reference's state_dict naming."""
        return self._export()["params"]

    def load_params(self, params):
        self._import({"params": params})

    def __getstate__(self):
        d = {k: v for k, v in self.__dict__.items() if k not in ("engine", "_replay")}
        d["_engine_state"] = self._export()
        d["_batch"] = self.batch_size
        return d

    def __setstate__(self, d):
        st = d.pop("_engine_state")
        batch = d.pop("_batch")
        self.__dict__.update(d)
        self._replay = None
        self.engine = self._new_engine(batch)
        self._import(st)

    def to(self, device):
        """td7.py:101-112: move to a device.  'cpu' is accepted as a no-op (pickling exports
        the HBM state; there is no CPU execution path); cuda:k moves the engine to GPU k."""
        k = _device_index(device)
        if k >= 0 and k != self._device:
            self._rebuild(device=k)
        self.device = device
        return self

    def load_state_dict(self, agent: "EngineAgent"):
        """td7.py:114-125 / td3.py:94-100 / sac.py:101-107: copy every network (not the
        optimiser state, counters or SAC temperature)."""
        if type(agent) is not type(self):
            raise TypeError("load_state_dict needs an agent of the same class")
        for net, names in self._param_names():
            for n, _ in names:
                self.engine.set_param(net, n, agent.engine.get_param(net, n))
        return self

    @property
    def n_runs(self) -> int:
        return int(self.engine.counters()[3])

    # ---- training ----------------------------------------------------------
    def _info(self, row):
        out = {}
        for k, v in zip(self._info_keys(), row):
            v = float(v)
            out[k] = None if (k in self.NULLABLE and math.isnan(v)) else v
        return out

    def train_ops(self, batch, replay_buffer=None, *args, **kwargs):
        """One gradient step on ``batch`` (td7.py:287-332 / td3.py:206-242 / sac.py:251-295).

        ``batch`` must come from ``replay_buffer.sample(B)`` of a device replay: the step
        reads rows ``batch.ind`` in HBM (the host tensors in the dict are not re-uploaded).
        Target-policy / rsample noise comes from the engine's Philox stream."""
        if not isinstance(batch, DeviceBatch):
            return self._train_host_batch(batch, replay_buffer)
        rep = replay_buffer if replay_buffer is not None else batch.replay
        if batch.replay is not rep:
            raise ValueError("batch was drawn from a different replay than replay_buffer")
        ind = np.ascontiguousarray(batch.ind, np.int64).reshape(1, -1)
        self._prepare(rep, ind.shape[1])
        self.engine.set_tapes(ind=ind)
        try:
            row = self.engine.step(1)[0]
        finally:
            self.engine.set_tapes()
        return self._info(row)

    def _train_host_batch(self, batch, replay_buffer):
        """train_ops on any BATCH dict (annotation.py:23-30: state, action, reward, next_state,
        done as arrays or tensors; action in the replay's stored form, done the not-done mask):
        the rows go into a B-row device ring bound to the engine, the step runs on rows 0..B-1,
        and a LAP replay_buffer gets the new priorities through its own update_priority (and its
        reset_max_priority at TD7 hard updates), as td7.py:236-240, 325-331 would call them."""

        missing = [k for k in ("state", "action", "reward", "next_state", "done") if k not in batch]
        if missing:
            raise ValueError(f"BATCH (annotation.py:23-30) without {missing}")

        def arr(k, shape):
            v = batch[k]
            if hasattr(v, "detach"):
                v = v.detach().cpu().numpy()
            return np.ascontiguousarray(np.asarray(v, np.float32).reshape(shape))

        B = int(np.asarray(batch["reward"].shape[0] if hasattr(batch["reward"], "shape") else len(batch["reward"])))
        s, a = arr("state", (B, self.state_dim)), arr("action", (B, self.action_dim))
        r, s2, d = arr("reward", (B,)), arr("next_state", (B, self.state_dim)), arr("done", (B,))
        lap = bool(self._cfg.get("use_lap")) and self.ALG != "sac"
        # td7.py:310 / td3.py:221 assert a LAP replay before update_priority (here before the step,
        # which runs as one device program: the reference would have stepped the encoder first)
        assert not lap or (replay_buffer is not None and getattr(replay_buffer, "LAP", hasattr(replay_buffer, "update_priority"))), \
            "a LAP agent's train_ops needs the LAPReplayMemory its priorities go to (td7.py:310)"
        ring = getattr(self, "_host_ring", None)
        if ring is None or ring.capacity != B or getattr(ring, "device", None) != self._device:
            ring = self._host_ring = E.Replay(B, self.state_dim, self.action_dim, lap, self._device)
            ring.device = self._device
        ring.append(s, a, r, s2, d)  # (capacity B: the write pointer returns to row 0)
        # (graphs capture the bound replay: another replay or batch size means a fresh engine)
        if B != self.batch_size or (self._replay is not None and self._replay is not ring):
            self._rebuild(B)
        if self._replay is not ring:
            self.engine.bind(ring)
            self._replay = ring
        hard_before = self.engine.counters()[3]
        self.engine.set_tapes(ind=np.arange(B, dtype=np.int64)[None])
        try:
            row = self.engine.step(1)[0]
        finally:
            self.engine.set_tapes()
        if lap:
            import torch

            replay_buffer.update_priority(torch.from_numpy(ring.get_priority(B).copy()))
            tur = int(self._cfg.get("target_update_rate", 250))
            if self.ALG == "td7" and (hard_before + 1) % tur == 0 and hasattr(replay_buffer, "reset_max_priority"):
                replay_buffer.reset_max_priority()
        return self._info(row)

    def train_n(self, replay_buffer: BaseReplayMemory, batch_size: int, n_ops: int):
        """n_ops x (sample + train_ops) fused on the device (run_train_ops, run.py:87-96)."""
        self._prepare(replay_buffer, batch_size)
        rows = self.engine.step(n_ops) if n_ops > 0 else []
        if n_ops > 0:
            replay_buffer._mark_engine_indices(self.engine)
        return [self._info(r) for r in rows]

    # ---- acting --------------------------------------------------------------
    def _act(self, state, deterministic, eps=None):
        """Agent.sample as one device program (rle_act_sample): forward, exploration noise
        (the engine's Philox stream, or the tape `eps` [A]), clip and the action map, written
        into pinned memory by the last kernel.  Returns the first row as the reference does."""
        eng = self.engine
        # the reference reads action_scale / action_bias / exploration_noise on every call
        # (td7.py:151-155): re-send the map whenever any of them changed
        amap = (np.asarray(self.action_scale, np.float32).tobytes(), np.asarray(self.action_bias, np.float32).tobytes(),
                float(getattr(self, "exploration_noise", 0.1)))
        if getattr(eng, "_act_map", None) != amap:
            eng.set_action_map(self.action_scale, self.action_bias, amap[2])
            eng._act_map = amap
        if hasattr(state, "detach"):
            state = state.detach().cpu().numpy()
        if eps is not None:
            return eng.act_sample(state, 2, eps)[0].copy()
        return eng.act_sample(state, 0 if deterministic else 1)[0].copy()

    def _forward(self, state, width):
        if hasattr(state, "detach"):
            state = state.detach().cpu().numpy()
        x = np.asarray(state, np.float32)
        if x.ndim == 1:
            x = x[None]
        return self.engine.act(x, width)
