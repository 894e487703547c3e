"""Action samplers (rl/sampler.py:14-37)."""

from __future__ import annotations

import numpy as np

from rl.utils.envs import action_bounds


class Sampler:
    """Anything with ``sample(state, ...)`` -> env action (sampler.py:14-19)."""

    def sample(self, *args, **kwargs):
        raise NotImplementedError("!!")


class RandomSampler(Sampler):
    """Uniform actions over the Box (sampler.py:22-37; the reference seeds the space with 777)."""

    def __init__(self, env_id: str | None = None, low=None, high=None, seed: int = 777) -> None:
        if env_id is not None:
            low, high = action_bounds(env_id)
        self.low = np.asarray(low, np.float32)
        self.high = np.asarray(high, np.float32)
        self.rng = np.random.default_rng(seed)

    def sample(self, *args, **kwargs) -> np.ndarray:
        return self.rng.uniform(self.low, self.high).astype(np.float32)
