"""Standalone LAP sampler dispatches for rocprofv3: TD7 Humanoid replay (S 376,
A 17), 1M rows, random priorities >= 1, B = 256 queries per dispatch.  Each
rle_replay_sample_indices call is ONE rle_level launch of OP_SAMPLE_GATHER (64 workgroups, one
wave per query: three-level LAP search + row gather into the batch images, kernels.hip
op_sample_gather), the op the step graphs run; tools/sampler_summary.py picks those dispatches
out of the kernel trace by grid size.

Usage (GPU box): rocprofv3 --kernel-trace --stats ... -- python3 tools/sampler_prof.py [calls]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd")]
from rl import _engine as E  # noqa: E402

N, S, A, B = 1_000_000, 376, 17, 256
calls = int(sys.argv[1]) if len(sys.argv) > 1 else 300
rep = E.Replay(N, S, A, True)
rep.fill_random(N, seed=0)
rng = np.random.default_rng(5)
p = ((1.0 + np.abs(rng.standard_normal(N)) * 2.0) ** 0.4).astype(np.float32)
rep.set_priority(p, float(p.max()))
for i in range(calls):
    ind = rep.sample_indices(rng.random(B, dtype=np.float32))
assert ind.min() >= 0 and ind.max() < N
print(f"sampler_prof: {calls} dispatches of B={B} over N={N}")
