"""Offline stand-in for the parts of ``gymnasium`` the reference imports.

Used ONLY by ``make_golden.py`` (this container, never the GPU box) so that
``import rl`` from ``/root/reference`` succeeds: the reference touches
gymnasium only for observation/action space shapes and bounds
(``rl/utils/miscellaneous.py:50-66``) and for wrapper base classes that the
gradient step never calls.  No environment dynamics are provided.

Spaces follow the MuJoCo-v4 tasks' published shapes/bounds; ``Tiny-v0`` is a
small synthetic task used for full-dump fixtures.
"""

from __future__ import annotations

import sys
import types

import numpy as np

# env_id -> (obs_dim, act_dim, action high bound)
TASKS = {
    "Humanoid-v4": (376, 17, 0.4),
    "Ant-v4": (27, 8, 1.0),
    "HalfCheetah-v4": (17, 6, 1.0),
    "Hopper-v4": (11, 3, 1.0),
    "Walker2d-v4": (17, 6, 1.0),
    "Tiny-v0": (11, 3, 0.5),
}


class Box:
    def __init__(self, low, high, shape, dtype=np.float32):
        self.shape = tuple(shape)
        self.dtype = dtype
        self.low = np.full(self.shape, low, dtype=dtype)
        self.high = np.full(self.shape, high, dtype=dtype)
        self._rng = np.random.default_rng(0)

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        return [seed]

    def sample(self):
        return self._rng.uniform(self.low, self.high).astype(self.dtype)


class Spec:
    def __init__(self, env_id):
        self.id = env_id


class Env:
    def __init__(self, env_id):
        s, a, hi = TASKS[env_id]
        self.spec = Spec(env_id)
        self.observation_space = Box(-np.inf, np.inf, (s,), np.float64)
        self.action_space = Box(-hi, hi, (a,), np.float32)

    def reset(self, seed=None, **kw):
        return np.zeros(self.observation_space.shape), {}

    def step(self, action):  # pragma: no cover - never used by the fixtures
        raise RuntimeError("gym_stub has no dynamics")


class Wrapper(Env):
    def __init__(self, env, *a, **k):
        self.env = env
        self.spec = env.spec
        self.observation_space = env.observation_space
        self.action_space = env.action_space


def make(env_id, **kwargs):
    if hasattr(env_id, "id"):
        env_id = env_id.id
    return Env(env_id)


def install() -> None:
    """Register the stand-in as ``gymnasium`` in ``sys.modules``."""
    gym = types.ModuleType("gymnasium")
    gym.registry = dict.fromkeys(TASKS)
    gym.make = make
    gym.Env = Env
    gym.Space = Box
    gym.Wrapper = Wrapper
    gym.ActionWrapper = Wrapper
    utils = types.ModuleType("gymnasium.utils")

    class RecordConstructorArgs:  # noqa: D401
        def __init__(self, **kw):
            pass

    utils.RecordConstructorArgs = RecordConstructorArgs
    gym.utils = utils
    wrappers = types.ModuleType("gymnasium.wrappers")
    wrappers.TimeLimit = Wrapper
    wrappers.FlattenObservation = Wrapper
    res = types.ModuleType("gymnasium.wrappers.record_episode_statistics")
    res.RecordEpisodeStatistics = Wrapper
    rv = types.ModuleType("gymnasium.wrappers.record_video")
    rv.RecordVideo = Wrapper
    wrappers.record_episode_statistics = res
    wrappers.record_video = rv
    wrappers.RecordEpisodeStatistics = Wrapper
    wrappers.RecordVideo = Wrapper
    gym.wrappers = wrappers
    spaces = types.ModuleType("gymnasium.spaces")
    spaces.Box = Box
    gym.spaces = spaces
    for name, mod in {
        "gymnasium": gym,
        "gymnasium.utils": utils,
        "gymnasium.wrappers": wrappers,
        "gymnasium.wrappers.record_episode_statistics": res,
        "gymnasium.wrappers.record_video": rv,
        "gymnasium.spaces": spaces,
    }.items():
        sys.modules[name] = mod
