"""run_train_ops (rl/runner/run.py:87-96) with the fused device loop."""

from __future__ import annotations

from rl.agent.engine_agent import EngineAgent
from rl.replay_memory.base import BaseReplayMemory


def run_train_ops(rollout, agent, batch_size: int, n_ops: int = 1) -> list[dict]:
    """n_ops x ``agent.train_ops(rollout.get_batch(batch_size), replay_buffer)``.

    With an engine agent and a device replay the whole loop (sampling, the step,
    LAP priority update) runs on the GPU as n_ops graph replays with one host sync;
    otherwise it is the reference's Python loop."""
    replay = getattr(rollout, "replay_buffer", rollout)
    if isinstance(agent, EngineAgent) and isinstance(replay, BaseReplayMemory):
        return agent.train_n(replay, batch_size, n_ops)
    infos = []
    for _ in range(n_ops):
        batch = rollout.get_batch(batch_size)
        infos.append(agent.train_ops(batch, replay_buffer=replay))
    return infos
