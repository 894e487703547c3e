"""Uniform replay memory on the device (rl/replay_memory/simple.py:12-62)."""

from rl.replay_memory.base import BaseReplayMemory


class SimpleReplayMemory(BaseReplayMemory):
    """Uniform sampling: searchsorted(cumsum(ones(size)), u * size) (simple.py:45-54),
    evaluated in closed form on the device."""

    LAP = False
