"""SAC fused-epilogue diagnosis (GPU box): first-step info rows of the sac_tiny golden under the
RLE_NO_SACFWD / RLE_NO_SACBWD / RLE_NO_HEADDX switches against the golden."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd"), os.path.join(REPO, "tests")]
import numpy as np
from conftest import load_golden
from harness import engine_from_golden, parse
np.set_printoptions(precision=5, suppress=True, linewidth=150)
name = sys.argv[1] if len(sys.argv) > 1 else "sac_tiny"
g = load_golden(name)
print("meta", parse(g)[:8])
print("golden info[0]", np.asarray(g["info"])[0] if "info" in g else None)
for env in ({}, {"RLE_NO_SACFWD": "1"}, {"RLE_NO_SACBWD": "1"}, {"RLE_NO_SACFWD": "1", "RLE_NO_SACBWD": "1"},
            {"RLE_NO_SACFWD": "1", "RLE_NO_SACBWD": "1", "RLE_NO_HEADDX": "1"}):
    for k in ("RLE_NO_SACFWD", "RLE_NO_SACBWD", "RLE_NO_HEADDX"):
        os.environ.pop(k, None)
    os.environ.update(env)
    eng, rep, tp = engine_from_golden(g)
    eng.set_tapes(u=tp["u"][:2], eps=tp["eps"][:2], eps_pi=tp.get("eps_pi"))
    rows = [eng.step(1)[0] for _ in range(2)]
    eng.set_tapes()
    print(env, np.array(rows)[:, :6])
    print("   desc:", eng.describe(0).replace("\n", " | ")[:600])
