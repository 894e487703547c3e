"""TD3 (rl/agent/td3.py:30-245) on the HIP engine."""

from __future__ import annotations

import numpy as np

from rl import _engine as E
from rl.agent.engine_agent import EngineAgent


class TD3(EngineAgent):
    """MLP actor + twin critics with target policy smoothing and delayed Polyak updates.

    Constructor arguments as the reference (td3.py:33-47) plus ``hidden``,
    ``batch_size``, ``seed`` and ``device`` (see TD7)."""

    ALG = "td3"
    ALGO = E.RLE_TD3
    OPTIM_NETS = ("policy", "q1", "q2")
    NULLABLE = ("train/policy", "norm/policy")

    def __init__(self, env_id: str, discount_factor: float = 0.99, policy_lr: float = 3e-4,
                 critic_lr: float = 3e-4, exploration_noise: float = 0.1, target_policy_noise: float = 0.2,
                 noise_clip: float = 0.5, policy_freq: int = 2, tau: float = 0.005, use_lap: bool = False,
                 make_nn=None, *, hidden: int = 256, batch_size: int = 256, seed: int | None = None,
                 device=None, **make_nn_kwargs) -> None:
        self.discount_factor = discount_factor
        self.target_policy_noise = target_policy_noise
        self.exploration_noise = exploration_noise
        self.noise_clip = noise_clip
        self.policy_freq = policy_freq
        self.use_lap = use_lap
        self.tau = tau
        cfg = dict(use_lap=use_lap, discount=discount_factor, policy_lr=policy_lr, critic_lr=critic_lr,
                   tau=tau, target_policy_noise=target_policy_noise, noise_clip=noise_clip,
                   policy_freq=policy_freq)
        self._setup(env_id, hidden=hidden, batch_size=batch_size, seed=seed, device=device, make_nn=make_nn,
                    make_nn_kwargs=make_nn_kwargs, cfg=cfg)

    def _info_keys(self):
        return ("train/q_fn", "train/policy", "norm/policy")  # td3.py:226-235

    def sample(self, state, deterministic: bool = False, **kwargs):
        """td3.py:114-135: clip(tanh(policy(s)) + exploration_noise * randn, -1, 1) * scale + bias, one
        device program (rle_act_sample).  The noise comes from the engine's Philox stream (the
        reference uses torch's global generator); kwargs eps=[A] supplies it instead (parity)."""
        return self._act(state, deterministic, kwargs.get("eps"))

    def __repr__(self) -> str:
        return "TD3"
