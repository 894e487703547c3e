"""TD7 (rl/agent/td7.py:31-332) on the HIP engine."""

from __future__ import annotations

import numpy as np

from rl import _engine as E
from rl.agent.engine_agent import EngineAgent


class TD7(EngineAgent):
    """SALE encoder + actor + twin critics, LAP, value clipping, fixed/target encoders.

    Same constructor arguments as the reference (td7.py:34-48) plus ``hidden``
    (hdim = zs_dim), ``batch_size`` (the captured step's B; train_ops with another
    B rebuilds the step graphs), ``seed`` (weight init + Philox stream) and ``device``.
    """

    ALG = "td7"
    ALGO = E.RLE_TD7
    OPTIM_NETS = ("encoder", "policy", "q1", "q2")
    NULLABLE = ("train/policy",)

    def __init__(self, env_id: str, discount_factor: float = 0.99, policy_lr: float = 3e-4,
                 critic_lr: float = 3e-4, target_update_rate: int = 250, exploration_noise: float = 0.1,
                 target_policy_noise: float = 0.2, noise_clip: float = 0.5, policy_freq: int = 2,
                 use_lap: bool = False, make_nn=None, *, hidden: int = 256, batch_size: int = 256,
                 seed: int | None = None, device=None, **make_nn_kwargs) -> None:
        self.discount_factor = discount_factor
        self.target_update_rate = target_update_rate
        self.target_policy_noise = target_policy_noise
        self.exploration_noise = exploration_noise
        self.noise_clip = noise_clip
        self.policy_freq = policy_freq
        self.use_lap = use_lap
        cfg = dict(use_lap=use_lap, discount=discount_factor, policy_lr=policy_lr, critic_lr=critic_lr,
                   target_policy_noise=target_policy_noise, noise_clip=noise_clip, policy_freq=policy_freq,
                   target_update_rate=target_update_rate)
        self._setup(env_id, hidden=hidden, batch_size=batch_size, seed=seed, device=device, make_nn=make_nn,
                    make_nn_kwargs=make_nn_kwargs, cfg=cfg)

    def _info_keys(self):
        return ("train/encoder", "train/q_fn", "train/policy")  # td7.py:302,314,317

    @property
    def value_max(self):
        return float(self.engine.value_bounds()[0])

    @property
    def value_min(self):
        return float(self.engine.value_bounds()[1])

    @property
    def value_target_max(self):
        return float(self.engine.value_bounds()[2])

    @property
    def value_target_min(self):
        return float(self.engine.value_bounds()[3])

    def sample(self, state, deterministic: bool = False, **kwargs):
        """td7.py:141-156: clip(tanh(policy(s)) + exploration_noise * randn, -1, 1) * scale + bias, one
        device program (rle_act_sample).  The noise comes from the engine's Philox stream (the
        reference uses torch's global generator); kwargs eps=[A] supplies it instead (parity)."""
        return self._act(state, deterministic, kwargs.get("eps"))

    def __repr__(self) -> str:
        return "TD7"
