"""rl.runner (reference: rl/runner/__init__.py, run.py).  ``rl.runner.run.run_train_ops`` is the
import path the reference's runners use (rl/runner/run.py:87-96); ``rl.runner.run_train_ops``
is kept as a short alias."""

from .run import run_train_ops

__all__ = ["run_train_ops"]
