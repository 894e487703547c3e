"""Engine construction + graph build time (GPU box): TD7 Humanoid B=256 on a 64K replay."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd")]
from rl import _engine as E  # noqa: E402
from rl.nn.layout import init_agent  # noqa: E402

S, A, H, B = 376, 17, 256, 256
rep = E.Replay(65536, S, A, True)
rep.fill_random(65536, 1)
for i in range(2):
    t0 = time.perf_counter()
    eng = E.Engine(E.make_config(E.RLE_TD7, S, A, H, B, use_lap=True))
    for net, params in init_agent("td7", S, A, H, 1).items():
        for k, v in params.items():
            eng.set_param(net, k, v)
    eng.bind(rep)
    t1 = time.perf_counter()
    eng.step(1)
    t2 = time.perf_counter()
    print(f"create+params+bind {t1 - t0:.3f} s, first step (graph build) {t2 - t1:.3f} s")
    del eng
