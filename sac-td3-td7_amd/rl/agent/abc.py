"""Agent interface (rl/agent/abc.py:16-55)."""

from __future__ import annotations

import os
import pickle
from pathlib import Path


class Agent:
    """Base agent: train_ops / to / load_state_dict / save / load."""

    def make_optimizers(self, *args, **kwargs) -> None:
        raise NotImplementedError

    def train_ops(self, batch, *args, **kwargs):
        raise NotImplementedError("`train_ops` should be implemented.")

    def to(self, device):
        raise NotImplementedError("`to` should be implemented.")

    def load_state_dict(self, agent: "Agent") -> None:
        raise NotImplementedError("`load_state_dict` should be implemented.")

    def save(self, path) -> None:
        """abc.py:38-47: pickle the agent (engine state is exported through __getstate__)."""
        path = Path(path)
        os.makedirs(path.parent, exist_ok=True)
        with open(path, "wb") as fh:
            pickle.dump(self, fh)

    @staticmethod
    def load(path) -> "Agent":
        """abc.py:49-55.  Like the reference this unpickles: load only files you wrote."""
        assert os.path.isfile(path)
        with open(path, "rb") as fh:
            return pickle.load(fh)
