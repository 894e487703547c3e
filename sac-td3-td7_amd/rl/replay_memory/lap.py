"""LAP replay memory on the device (rl/replay_memory/lap.py:12-76)."""

from __future__ import annotations

import numpy as np

from rl.replay_memory.base import BaseReplayMemory


class LAPReplayMemory(BaseReplayMemory):
    """Prioritised ring: append writes max_priority (lap.py:41), sample draws
    searchsorted(cumsum(priority), u * sum) (lap.py:47-54) on the device."""

    LAP = True

    @property
    def max_priority(self) -> float:
        self.flush()
        return self.dev.state()[2]

    @property
    def priority(self):
        """torch view of the priority vector [replay_buffer_size] (lap.py:28)."""
        import torch

        self.flush()
        return torch.from_numpy(self.dev.get_priority())

    def update_priority(self, priority) -> None:
        """lap.py:66-69: priority[self.ind] = p (last duplicate wins); max_priority = max(...)."""
        p = priority.detach().cpu().numpy() if hasattr(priority, "detach") else np.asarray(priority)
        self.flush()
        self.dev.update_priority(self.ind, np.asarray(p, np.float32).reshape(-1))

    def reset_max_priority(self) -> None:
        """lap.py:71-73."""
        self.flush()
        self.dev.reset_max_priority()
