"""rl.nn: the reference's net classes (rl/nn/sale.py, rl/nn/mlp.py) for make_nn hooks, loaded on
first use (they import torch)."""

_MODULES = ("SALEActor", "SALECritic", "SALEEncoder", "MLPActor", "MLPCritic", "avg_l1_norm")


def __getattr__(name):
    if name in _MODULES:
        from rl.nn import modules

        return getattr(modules, name)
    raise AttributeError(name)
