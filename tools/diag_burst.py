"""Per-burst wall time of short bursts (GPU box, diagnostics): python tools/diag_burst.py [warmup] [n] [reps]
Times `reps` consecutive rle_step_timed(n) bursts after `warmup` steps, as bench.py does for one.
RLE_DIAG_FILL_LAST=1: the replay fill (device work) runs after the engine is bound and built, right before
the warmup."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd")]
import bench  # noqa: E402
from rl import _engine as E  # noqa: E402
from rl.nn.layout import init_agent  # noqa: E402
import torch  # noqa: E402

W, n, reps = (int(a) for a in (sys.argv[1:4] + ["5", "20", "8"][len(sys.argv[1:4]):]))
S, A, _ = bench.TASKS["Humanoid-v4"]
eng = E.Engine(E.make_config(E.RLE_TD7, S, A, 256, 256, use_lap=True, seed=111, device=0), E.parse_plan(""))
for net, params in init_agent("td7", S, A, 256, 123).items():
    for name, v in params.items():
        eng.set_param(net, name, v)
rep = E.Replay(bench.N_REPLAY, S, A, True, device=0)
last = os.environ.get("RLE_DIAG_FILL_LAST") == "1"
if not last:
    rep.fill_random(bench.N_REPLAY, seed=0)
eng.bind(rep)
eng.graph_stats()
if last:
    rep.fill_random(bench.N_REPLAY, seed=0)
pre = int(os.environ.get("RLE_DIAG_PREWARM", "0"))
if pre:  # another engine on the same replay steps first (its row gathers touch the replay's pages)
    e0 = E.Engine(E.make_config(E.RLE_TD7, S, A, 256, 256, use_lap=True, seed=7, device=0), E.parse_plan(""))
    for net, params in init_agent("td7", S, A, 256, 5).items():
        for name, v in params.items():
            e0.set_param(net, name, v)
    e0.bind(rep)
    e0.step_timed(pre)
    del e0
eng.step_timed(W)
torch.cuda.synchronize(0)
gap = float(os.environ.get("RLE_DIAG_GAP_MS", "0"))
for r in range(reps):
    if gap:
        time.sleep(gap / 1e3)
    l0 = eng.launch_count()
    t0 = time.perf_counter()
    ms = eng.step_timed(n)
    torch.cuda.synchronize(0)
    t1 = time.perf_counter()
    print(f"burst {r}: wall {(t1 - t0) * 1e3:.3f} ms ({n / (t1 - t0):.0f} steps/s), engine {ms:.3f} ms, "
          f"launches {eng.launch_count() - l0}")
