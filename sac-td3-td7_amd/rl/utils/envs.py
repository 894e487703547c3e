"""Environment shapes without gymnasium.

The reference derives (obs_dim, act_dim) and the action affine map from the
live gym spaces (``get_state_action_dims`` / ``get_action_bias_scale``,
rl/utils/miscellaneous.py:50-66).  Only those numbers reach the hot path, so
this module keeps a table of the MuJoCo-v4 spaces the reference's scripts use
(scripts/*.sh) and lets callers register others.  When gymnasium is importable
its registry is used for ids the table does not know.
"""

from __future__ import annotations

import numpy as np

# env_id -> (obs_dim, act_dim, action low, action high); Box bounds are uniform per task
_SPECS: dict[str, tuple[int, int, np.ndarray, np.ndarray]] = {}


def register_env(env_id: str, state_dim: int, action_dim: int, low=-1.0, high=1.0) -> None:
    """Register an environment's observation/action shapes and action bounds."""
    lo = np.broadcast_to(np.asarray(low, np.float32), (action_dim,)).copy()
    hi = np.broadcast_to(np.asarray(high, np.float32), (action_dim,)).copy()
    if not np.all(hi > lo):
        raise ValueError(f"{env_id}: action high must exceed low")
    _SPECS[env_id] = (int(state_dim), int(action_dim), lo, hi)


for _id, _s, _a, _hi in (("Humanoid-v4", 376, 17, 0.4), ("Ant-v4", 27, 8, 1.0),
                         ("HalfCheetah-v4", 17, 6, 1.0), ("Hopper-v4", 11, 3, 1.0),
                         ("Walker2d-v4", 17, 6, 1.0)):
    register_env(_id, _s, _a, -_hi, _hi)


def _lookup(env_id: str):
    if env_id not in _SPECS:
        try:
            import gymnasium as gym  # optional: only for ids outside the table
        except ImportError as e:
            raise KeyError(f"unknown env_id {env_id!r}: register_env() it (gymnasium is absent)") from e
        env = gym.make(env_id)
        if "dm_control" in env_id:
            env = gym.wrappers.FlattenObservation(env)
        sp = env.action_space
        register_env(env_id, env.observation_space.shape[0], sp.shape[0], sp.low, sp.high)
    return _SPECS[env_id]


def get_state_action_dims(env_id: str) -> tuple[int, int]:
    """miscellaneous.py:50-56."""
    s, a, _, _ = _lookup(env_id)
    return s, a


def get_action_bias_scale(env_id: str) -> tuple[np.ndarray, np.ndarray]:
    """miscellaneous.py:59-66: bias = (lo + hi) / 2, scale = (hi - lo) / 2 (float32 like the Box)."""
    _, _, lo, hi = _lookup(env_id)
    return (lo + hi) / 2.0, (hi - lo) / 2.0


def action_bounds(env_id: str) -> tuple[np.ndarray, np.ndarray]:
    _, _, lo, hi = _lookup(env_id)
    return lo.copy(), hi.copy()
