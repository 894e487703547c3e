"""Bitwise comparison of two engine builds on a golden trajectory (GPU box, diagnostics).

    RLE_LIB=lib_a.so python tools/bitcmp.py dump NAME STEPS out_a.npz
    RLE_LIB=lib_b.so python tools/bitcmp.py dump NAME STEPS out_b.npz
    python tools/bitcmp.py cmp out_a.npz out_b.npz

Per step: every parameter, the priorities and the info row after a single-step replay.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd"), os.path.join(REPO, "tests")]


def dump(name, steps, out):
    from conftest import load_golden
    from harness import engine_from_golden, parse, shape_of
    from oracle import spec

    g = load_golden(name)
    alg, env, H, B, Ncap, n_fill, n_steps, use_lap, seed, extra = parse(g)
    steps = min(steps, n_steps)  # (the golden's tapes cover n_steps)
    S, A, hi = spec.TASKS[env]
    eng, rep, tp = engine_from_golden(g)
    shapes = {net: {k: np.shape(v) for k, v in p.items()}
              for net, p in spec.agent_params(alg, S, A, H, seed, **shape_of(g)).items()}
    names = {net: list(p.keys()) for net, p in shapes.items()}
    keep = os.environ.get("BITCMP_NETS")  # comma-separated nets to dump (default: all)
    if keep:
        names = {n: v for n, v in names.items() if n in keep.split(",")}
    eng.set_tapes(u=tp["u"][:steps], eps=tp["eps"][:steps],
                  eps_pi=tp.get("eps_pi", None) if "eps_pi" in tp else None)
    res = {}
    burst = int(os.environ.get("BITCMP_BURST", "1"))  # steps per rle_step call (6: TD7's multi-step graphs)
    for t in range(0, steps, burst):
        res[f"info_{t}"] = np.asarray(eng.step(min(burst, steps - t)))
        if use_lap:
            res[f"prio_{t}"] = rep.get_priority(Ncap)
        for net, ps in names.items():
            for p in ps:
                res[f"{t}/{net}/{p}"] = np.asarray(eng.get_param(net, p)).reshape(shapes[net][p])
    np.savez(out, **res)


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    for k in A.files:
        x, y = A[k], B[k]
        d = np.abs(x.astype(np.float64) - y.astype(np.float64))
        # bitwise (NaN payloads included: the info row's NaN on plain steps is equal to itself)
        xb = x.view(np.uint32) if x.dtype == np.float32 else x
        yb = y.view(np.uint32) if y.dtype == np.float32 else y
        n = int((xb != yb).sum())
        if n:
            print(f"{k:50s} differ {n:7d}/{x.size:7d} max {d.max():.3e}")
            if x.ndim == 2:
                r, c = np.nonzero(xb != yb)
                print(f"    rows {sorted(set((r // 16).tolist()))} (16-blocks), cols {sorted(set((c // 16).tolist()))} (16-blocks)")
    print("compared", len(A.files), "arrays")


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2], int(sys.argv[3]), sys.argv[4])
    else:
        cmp(sys.argv[2], sys.argv[3])
