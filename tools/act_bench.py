"""Per-env-step costs around the gradient step (GPU box):
agent.sample latency (one device program: B=1 fixed-encoder + actor forward, Philox exploration
noise, clip and action map into pinned memory, rle_act_sample), the bare ABI call, and
replay append throughput (staged host rows -> one batched H2D append kernel).
python tools/act_bench.py  -> one JSON line."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd")]
from rl.agent import TD7  # noqa: E402
from rl.replay_memory import LAPReplayMemory  # noqa: E402

env = "Humanoid-v4"
agent = TD7(env, use_lap=True, batch_size=256, seed=111, device=0)
rep = LAPReplayMemory(1_000_000, env, device=0)
rng = np.random.default_rng(0)
obs = rng.standard_normal(376).astype(np.float32)
out = {}
for det in (False, True):
    for _ in range(20):
        agent.sample(obs, deterministic=det)
    n = 2000
    t0 = time.perf_counter()
    for _ in range(n):
        agent.sample(obs, deterministic=det)
    out[f"sample_us_{'det' if det else 'explore'}"] = round((time.perf_counter() - t0) / n * 1e6, 2)
x = obs[None].copy()
for mode in (0, 1):
    for _ in range(20):
        agent.engine.act_sample(x, mode)
    n = 2000
    t0 = time.perf_counter()
    for _ in range(n):
        agent.engine.act_sample(x, mode)
    out[f"engine_act_sample_us_mode{mode}"] = round((time.perf_counter() - t0) / n * 1e6, 2)
rows = 200_000
s = rng.standard_normal((rows, 376)).astype(np.float32)
a = rng.uniform(-0.4, 0.4, (rows, 17)).astype(np.float32)
r = rng.standard_normal(rows).astype(np.float32)
d = np.ones(rows, np.float32)
t0 = time.perf_counter()
for i in range(rows):
    rep.append([s[i], a[i], float(r[i]), s[i], float(d[i])])
rep.flush()
t1 = time.perf_counter()
out["append_rows_per_s_single"] = round(rows / (t1 - t0))
t0 = time.perf_counter()
rep.append_batch(s, a, r, s, d)
rep.flush()
len(rep)
t1 = time.perf_counter()
out["append_rows_per_s_batch"] = round(rows / (t1 - t0))
out["replay_size"] = len(rep)
print(json.dumps(out))
