"""Replay memories held in HBM (rl/replay_memory/base.py:9-26 interface).

The reference keeps float64 NumPy rings on the host and casts gathered rows to
float32 tensors in ``sample`` (lap.py:55-60).  Here the ring lives on the GPU as
float32 structure-of-arrays (``rle_replay_*`` in include/rle.h), which is the
same data after that cast.  Host appends are staged and flushed in one batched
copy before any device use, so the per-env-step cost is a host memcpy.
"""

from __future__ import annotations

from typing import Any

import numpy as np

from rl import _engine as E
from rl.utils.envs import get_action_bias_scale, get_state_action_dims


class DeviceBatch(dict):
    """The BATCH dict (annotation.py:23-30) plus the indices and replay it was drawn from.

    Engine-backed ``train_ops`` trains on rows ``ind`` of ``replay`` on the device;
    the tensors in the dict are the host copy the reference would have built.
    """

    def __init__(self, data, ind: np.ndarray, replay: "BaseReplayMemory"):
        super().__init__(data)
        self.ind = ind
        self.replay = replay


class BaseReplayMemory:
    """Device ring of (state, action, reward, next_state, notdone) rows."""

    LAP = False
    STAGE = 4096  # host rows staged before one batched H2D append

    def __init__(self, replay_buffer_size: int, env_id: str | None = None, *, state_dim: int | None = None,
                 action_dim: int | None = None, device: int = 0, **kwargs) -> None:
        self.replay_buffer_size = int(replay_buffer_size)
        if env_id is not None:
            state_dim, action_dim = get_state_action_dims(env_id)
            self.action_bias, self.action_scale = get_action_bias_scale(env_id)
        else:
            if state_dim is None or action_dim is None:
                raise ValueError("need env_id or state_dim/action_dim")
            self.action_bias = np.zeros(action_dim, np.float32)
            self.action_scale = np.ones(action_dim, np.float32)
        self.env_id = env_id
        self.state_dim, self.action_dim = int(state_dim), int(action_dim)
        self.device = int(device)
        self.dev = E.Replay(self.replay_buffer_size, self.state_dim, self.action_dim, self.LAP, self.device)
        self._stage: list[tuple] = []
        self._ind = None
        self._ind_src = None  # engine whose last step drew the current indices

    # ---- appends ---------------------------------------------------------
    def _normalise(self, action):
        # lap.py:35 / simple.py:32, in the operands' own NumPy dtypes like the reference
        return np.asarray(action) / self.action_scale - self.action_bias

    def append(self, transition: list[Any]) -> None:
        """lap.py:31-43: one transition [obs, action, reward, next_obs, float_done]."""
        assert len(transition) == 5
        obs, action, reward, next_obs, float_done = transition
        self._stage.append((obs, self._normalise(action), reward, next_obs, float_done))
        if len(self._stage) >= self.STAGE:
            self.flush()

    def append_batch(self, obs, action, reward, next_obs, float_done) -> None:
        """Vectorised append of n transitions (row order = append order)."""
        self.flush()
        a = self._normalise(np.asarray(action).reshape(-1, self.action_dim))
        self.dev.append(np.asarray(obs).reshape(-1, self.state_dim), a, np.asarray(reward).reshape(-1),
                        np.asarray(next_obs).reshape(-1, self.state_dim), np.asarray(float_done).reshape(-1))

    def flush(self) -> None:
        if not self._stage:
            return
        st, a, r, s2, d = zip(*self._stage)
        self._stage = []
        n = len(r)
        self.dev.append(np.asarray(st, np.float64).reshape(n, self.state_dim).astype(np.float32),
                        np.asarray(a, np.float64).reshape(n, self.action_dim).astype(np.float32),
                        np.asarray(r, np.float64).reshape(n).astype(np.float32),
                        np.asarray(s2, np.float64).reshape(n, self.state_dim).astype(np.float32),
                        np.asarray(d, np.float64).reshape(n).astype(np.float32))

    # ---- state -----------------------------------------------------------
    @property
    def ptr(self) -> int:
        self.flush()
        return self.dev.state()[0]

    @property
    def size(self) -> int:
        self.flush()
        return self.dev.state()[1]

    def __len__(self) -> int:
        """lap.py:75-76: the write pointer (not the size) — kept as in the reference."""
        return self.ptr

    @property
    def ind(self):
        """Indices of the last batch: from sample(), or from the engine's last fused step."""
        if self._ind_src is not None:
            self._ind = self._ind_src.last_indices()
            self._ind_src = None
        return self._ind

    @ind.setter
    def ind(self, value):
        self._ind = None if value is None else np.asarray(value, np.int64)
        self._ind_src = None

    def _mark_engine_indices(self, eng) -> None:
        self._ind_src = eng

    # ---- sampling --------------------------------------------------------
    def sample(self, batch_size: int, use_torch: bool = True):
        """lap.py:45-64 / simple.py:45-62: u = torch.rand(B) from torch's global generator,
        device index search, row gather."""
        import torch

        self.flush()
        u = torch.rand(batch_size).numpy()
        ind = self.dev.sample_indices(u)
        s, a, r, s2, d = self.dev.gather(ind)
        data = dict(state=s, action=a, reward=r[:, None], next_state=s2, done=d[:, None])
        if use_torch:
            data = {k: torch.from_numpy(v) for k, v in data.items()}
        self.ind = ind
        return DeviceBatch(data, ind, self)
