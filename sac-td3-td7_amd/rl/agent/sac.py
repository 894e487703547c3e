"""SAC (rl/agent/sac.py:24-299) on the HIP engine."""

from __future__ import annotations

import numpy as np

from rl import _engine as E
from rl.agent.engine_agent import EngineAgent


class SAC(EngineAgent):
    """Squashed-Gaussian actor, twin critics, Polyak targets, optional auto temperature.

    Constructor arguments as the reference (sac.py:27-42) plus ``hidden``,
    ``batch_size``, ``seed`` and ``device``.  ``max_grad_norm`` is stored but, as in
    the reference, never applied."""

    ALG = "sac"
    ALGO = E.RLE_SAC
    OPTIM_NETS = ("policy", "q1", "q2")

    def __init__(self, env_id: str, discount_factor: float = 0.99, policy_lr: float = 3e-4,
                 critic_lr: float = 3e-4, min_log_std: float = -20.0, max_log_std: float = 2.0,
                 tau: float = 0.005, tmp: float = -1.0, use_lap: bool = False,
                 max_grad_norm: float = float("inf"), make_nn=None, *, hidden: int = 256,
                 batch_size: int = 256, seed: int | None = None, device=None, **make_nn_kwargs) -> None:
        self.auto_tmp_mode = tmp < 0.0
        self.discount_factor = discount_factor
        self.min_log_std, self.max_log_std = min_log_std, max_log_std
        self.tau = tau
        self.use_lap = use_lap
        self.max_grad_norm = max_grad_norm
        cfg = dict(use_lap=use_lap, discount=discount_factor, policy_lr=policy_lr, critic_lr=critic_lr,
                   tau=tau, min_log_std=min_log_std, max_log_std=max_log_std, tmp=tmp)
        self._setup(env_id, hidden=hidden, batch_size=batch_size, seed=seed, device=device, make_nn=make_nn,
                    make_nn_kwargs=make_nn_kwargs, cfg=cfg)
        if self.auto_tmp_mode:
            self.target_entropy = -self.action_dim

    def train_ops(self, batch, replay_buffer=None, *args, **kwargs):
        if self.use_lap:
            # sac.py:199-203 calls self._lap_huber, which SAC does not define
            raise AttributeError("'SAC' object has no attribute '_lap_huber' (reference sac.py:202)")
        return super().train_ops(batch, replay_buffer, *args, **kwargs)

    def train_n(self, replay_buffer, batch_size, n_ops):
        if self.use_lap:
            raise AttributeError("'SAC' object has no attribute '_lap_huber' (reference sac.py:202)")
        return super().train_n(replay_buffer, batch_size, n_ops)

    def _info_keys(self):
        if self.auto_tmp_mode:  # sac.py:268-290
            return ("train/q_fn", "tmp", "norm/tmp", "train/policy", "train/tmp", "entropy")
        return ("train/q_fn", "train/policy", "entropy")

    @property
    def tmp(self):
        """exp-space temperature parameter: log_alpha (auto mode) or the fixed value."""
        if not self.auto_tmp_mode:  # sac.py:56-60: the fixed float itself
            return float(self._cfg["tmp"])
        return float(self.engine.get_param("tmp", "log_alpha")[0])

    def _inference(self, state):
        """sac.py:154-159: Normal(mean, exp(clamp(log_std))) from the device actor head."""
        import torch

        raw = torch.from_numpy(self._forward(state, 2 * self.action_dim))
        mean, log_std = raw.chunk(2, dim=-1)
        log_std = torch.clamp(log_std, self.min_log_std, self.max_log_std)
        return torch.distributions.Normal(mean, log_std.exp())

    def sample(self, state, deterministic: bool = False, **kwargs):
        """sac.py:132-152: tanh(mean) or tanh(mean + std * randn) (rsample), * scale + bias, one
        device program (rle_act_sample; engine Philox stream, or kwargs eps=[A] for parity)."""
        return self._act(state, deterministic, kwargs.get("eps"))

    def __repr__(self) -> str:
        return "SAC"
