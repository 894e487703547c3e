import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "sac-td3-td7_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP engine calls)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


@pytest.fixture
def golden():
    return load_golden


def shape_of(g):
    """Net shapes beyond the defaults a golden was made with (make_golden.py ``shape``): make_mlp's
    hidden_sizes (TD3 / SAC) or SALE's zs_dim (TD7); {} for the default nets."""
    out = {}
    if "meta_hidden" in g:
        out["hidden_sizes"] = [int(x) for x in g["meta_hidden"]]
    if "meta_zs" in g:
        out["zs_dim"] = int(g["meta_zs"])
    return out


def acts_of(g):
    """Hidden activations beyond the defaults a golden was made with (make_golden.py ``acts``):
    {"actor", "critic", "encoder"} -> "relu" / "elu" / "identity"; {} for the default nets."""
    if "meta_acts" not in g:
        return {}
    return {k: str(v) for k, v in zip(("actor", "critic", "encoder"), g["meta_acts"]) if str(v) != "default"}
