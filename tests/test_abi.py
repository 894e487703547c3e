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


def test_aql_wait_policy_releases_the_host_core():
    """rle_step's AQL wait (engine.cpp aql_wait_step): sleep while more than the 150 us spin tail of the
    expected duration remains (slices <= 2 ms), spin for the tail, time out past the limit (the engine's
    queue is then closed: aql_flush refuses every later packet).  No GPU: the policy alone."""
    import ctypes

    from rl import _engine

    lib = _engine.lib()
    sl = ctypes.c_double()

    def plan(expected, elapsed, timeout=60.0):
        return lib.rle_aql_wait_plan(expected, elapsed, timeout, ctypes.byref(sl)), sl.value

    assert plan(250_000.0, 0.0) == (1, 2000.0)          # a 2000-step burst: sleep in 2 ms slices
    act, us = plan(250_000.0, 249_000.0)
    assert act == 1 and abs(us - 850.0) < 1e-6          # ... up to 150 us before the expected end
    assert plan(250_000.0, 249_900.0)[0] == 0           # then spin
    assert plan(100.0, 0.0)[0] == 0                     # short flushes never sleep
    assert plan(250_000.0, 400_000.0)[0] == 0           # overran the estimate: spin, no more sleeping
    assert plan(250_000.0, 61e6)[0] == 2                # past 60 s: time out
    assert plan(250_000.0, 1.5e6, timeout=1.0)[0] == 2


def test_aql_failed_queue_fails_fast_and_doorbells_stay_in_one_ring_pass():
    """A queue closed by a timed-out burst refuses new bursts and completes at once (so rle_destroy and every
    later entry point return instead of waiting another 60 s), also for engines sharing its hardware queue;
    doorbell groups never straddle the ring's end (engine.cpp aql_doorbell_after, the rocprofv3 crash of
    profiles/r05_prof_crash.txt).  No GPU: rle_aql_selftest reaches no HSA call."""
    from rl import _engine

    lib = _engine.lib()
    assert lib.rle_aql_selftest() == 0, lib.rle_last_error()


def test_ctypes_structs_match_the_header_layout(tmp_path):
    """rl/_engine.py Config / Plan mirror rle_config / rle_plan field by field: a C program compiled against
    include/rle.h prints each struct's size and every field's offset (gcc on the host, no GPU)."""
    import ctypes
    import shutil
    import subprocess

    from rl import _engine

    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    lines = []
    for cname, cls in (("rle_config", _engine.Config), ("rle_plan", _engine.Plan)):
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, *_ in cls._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    src = tmp_path / "layout.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "rle.h"\nint main(void) {\n'
                   + "\n".join(lines) + "\nreturn 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(ln.split() for ln in subprocess.run([str(exe)], check=True, capture_output=True,
                                                    text=True).stdout.splitlines())
    for cname, cls in (("rle_config", _engine.Config), ("rle_plan", _engine.Plan)):
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f, *_ in cls._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(cls, f).offset, (cname, f)


def test_create_rejects_bad_activation_codes_before_any_hip_call():
    """rle_create validates rle_config.act_* (RLE_ACT_DEFAULT..RLE_ACT_IDENTITY; act_encoder is TD7's) before it
    touches a device, so the errors come back through the ABI on a host without a GPU."""
    import ctypes

    from rl import _engine as E

    lib = E.lib()
    out = ctypes.c_void_p()
    cfg = E.make_config(E.RLE_TD7, 17, 6, 32, 16)
    cfg.act_actor = 7
    assert lib.rle_create(ctypes.byref(cfg), ctypes.byref(out)) == -1
    assert b"activation" in lib.rle_last_error()
    cfg = E.make_config(E.RLE_TD3, 17, 6, 32, 16, act_encoder="elu")
    assert lib.rle_create(ctypes.byref(cfg), ctypes.byref(out)) == -1
    assert b"act_encoder" in lib.rle_last_error()
    with pytest.raises(ValueError, match="activation"):
        E.make_config(E.RLE_SAC, 17, 6, 32, 16, act_critic="tanh")
