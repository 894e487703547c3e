"""CPU-side checks of the C-ABI boundary: library loads, every declared symbol exported."""

import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "rle.h")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(rle_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared()
    for n in ("rle_create", "rle_step", "rle_replay_create", "rle_replay_append", "rle_set_tapes",
              "rle_act", "rle_last_error"):
        assert n in names


def test_library_exports_every_symbol():
    from rl import _engine

    if not os.path.exists(_engine.LIB_PATH):
        pytest.fail("librle.so not built (run __graft_entry__.build())")
    lib = _engine.lib()  # loads without a GPU (no HIP calls at load)
    for n in declared():
        assert hasattr(lib, n), n
    assert set(_engine.SIGNATURES) == set(declared())


def test_errors_are_reported_not_raised_across_abi():
    from rl import _engine

    lib = _engine.lib()
    import ctypes

    out = ctypes.c_void_p()
    rc = lib.rle_replay_create(0, -5, 3, 2, 0, ctypes.byref(out))
    assert rc == -1
    assert b"bad args" in lib.rle_last_error()
