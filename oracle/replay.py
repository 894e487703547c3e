"""Replay memories restated in NumPy (TEST INFRASTRUCTURE ONLY).

Follows ``rl/replay_memory/lap.py:12-76`` and ``simple.py:12-65``:
transitions are stored as fp32 (bit-identical to the reference's f64 storage
followed by its fp32 cast at sample time, Q7), the priority cumsum is an exact
fp64 prefix rounded to fp32 (torch's CPU fp32 cumsum accumulates in double,
Q8) and duplicate priority writes resolve last-writer-wins (Q9).
"""

from __future__ import annotations

import numpy as np


def lap_indices(priority: np.ndarray, size: int, u: np.ndarray) -> np.ndarray:
    """LAPReplayMemory.sample index law (lap.py:47-54)."""
    c = np.cumsum(priority[:size].astype(np.float64)).astype(np.float32)
    v = (u.astype(np.float32) * c[-1]).astype(np.float32)
    return np.searchsorted(c, v, side="left").astype(np.int64)


def uniform_indices(size: int, u: np.ndarray) -> np.ndarray:
    """SimpleReplayMemory.sample index law (simple.py:45-54): searchsorted over
    cumsum(ones) = 1..size, i.e. ind = clamp(ceil(fp32(u*size)) - 1, 0, size-1)."""
    v = (u.astype(np.float32) * np.float32(size)).astype(np.float32)
    c = np.arange(1, size + 1, dtype=np.float32)
    return np.searchsorted(c, v, side="left").astype(np.int64)


class Replay:
    """Ring buffer with optional LAP priorities."""

    def __init__(self, capacity, S, A, action_scale, action_bias, lap: bool):
        self.N, self.S, self.A = capacity, S, A
        self.lap = lap
        self.scale = np.asarray(action_scale)
        self.bias = np.asarray(action_bias)
        self.state = np.zeros((capacity, S), np.float32)
        self.action = np.zeros((capacity, A), np.float32)
        self.reward = np.zeros((capacity, 1), np.float32)
        self.next_state = np.zeros((capacity, S), np.float32)
        self.done = np.zeros((capacity, 1), np.float32)
        self.priority = np.zeros(capacity, np.float32)
        self.max_priority = 1.0
        self.ptr = 0
        self.size = 0
        self.ind = None

    def append(self, obs, action, reward, next_obs, notdone):
        """lap.py:31-43 / simple.py:29-40 (action normalised in numpy, Q5)."""
        a = np.asarray(action) / self.scale - self.bias
        i = self.ptr
        self.state[i] = np.asarray(obs, np.float64)
        self.action[i] = a
        self.reward[i] = reward
        self.next_state[i] = np.asarray(next_obs, np.float64)
        self.done[i] = notdone
        if self.lap:
            self.priority[i] = self.max_priority
        self.ptr = (self.ptr + 1) % self.N
        self.size = min(self.size + 1, self.N)

    def sample_indices(self, u):
        if self.lap:
            return lap_indices(self.priority, self.size, u)
        return uniform_indices(self.size, u)

    def gather(self, ind):
        self.ind = ind
        return {
            "state": self.state[ind], "action": self.action[ind],
            "reward": self.reward[ind], "next_state": self.next_state[ind],
            "done": self.done[ind],
        }

    def update_priority(self, p):
        """lap.py:66-69; sequential writes => last duplicate wins (Q9)."""
        p = np.asarray(p, np.float32)
        for b, i in enumerate(self.ind):
            self.priority[i] = p[b]
        self.max_priority = max(float(p.max()), self.max_priority)

    def reset_max_priority(self):
        """lap.py:71-73."""
        self.max_priority = float(self.priority[: self.size].max())
