"""Steps/s of the engine with non-default hidden activations (rle_config act_*) beside the defaults, on bench.py's
synthetic workload (1M-row replay, random weights).  Not part of the product path; backs DESIGN round 6
"hidden activations".

    python tools/acts_bench.py [steps]
"""

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-td3-td7_amd"))
sys.path.insert(0, ROOT)

from rl import _engine as E  # noqa: E402
from rl.nn.layout import init_agent  # noqa: E402

TASKS = {"Humanoid-v4": (376, 17), "HalfCheetah-v4": (17, 6)}
CASES = [
    ("td7", "Humanoid-v4", {}),
    ("td7", "Humanoid-v4", {"act_actor": "elu", "act_critic": "relu", "act_encoder": "relu"}),
    ("td7", "Humanoid-v4", {"act_critic": "elu", "act_encoder": "elu", "act_actor": "relu"}),  # (= default)
    ("td3", "HalfCheetah-v4", {}),
    ("td3", "HalfCheetah-v4", {"act_actor": "elu", "act_critic": "elu"}),
    ("sac", "Humanoid-v4", {}),
    ("sac", "Humanoid-v4", {"act_actor": "elu", "act_critic": "elu"}),
]


def run(alg, env, acts, steps, warmup=100):
    S, A = TASKS[env]
    algo = {"td7": E.RLE_TD7, "td3": E.RLE_TD3, "sac": E.RLE_SAC}[alg]
    lap = alg == "td7"
    eng = E.Engine(E.make_config(algo, S, A, 256, 256, use_lap=lap, seed=111, **acts))
    for net, params in init_agent(alg, S, A, 256, 123).items():
        for name, v in params.items():
            eng.set_param(net, name, v)
    rep = E.Replay(1_000_000, S, A, lap)
    rep.fill_random(1_000_000, seed=0)
    eng.bind(rep)
    eng.step_timed(warmup)
    eng.synchronize()
    t0 = time.perf_counter()
    eng.step_timed(steps)
    eng.synchronize()
    dt = time.perf_counter() - t0
    out = {"algo": alg, "env": env, "acts": acts, "steps_per_s": round(steps / dt, 1),
           "launches_per_step": round(sum(eng.graph_stats()) / 2, 2)}
    eng.close()
    rep.close()
    return out


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    for alg, env, acts in CASES:
        print(json.dumps(run(alg, env, acts, n)), flush=True)
