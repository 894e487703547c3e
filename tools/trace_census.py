"""How many workgroups of each level start at once (GPU box): residency census from the
RLE_TRACE=1 entry stamps.  RLE_TRACE=1 python tools/trace_census.py [steps]"""
import os
import sys

import numpy as np

os.environ.setdefault("RLE_TRACE", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd")]
from rl import _engine as E  # noqa: E402
from rl.nn.layout import init_agent  # noqa: E402

S, A, H, B = 376, 17, 256, 256
eng = E.Engine(E.make_config(E.RLE_TD7, S, A, H, B, use_lap=True))
for net, params in init_agent("td7", S, A, H, 1).items():
    for k, v in params.items():
        eng.set_param(net, k, v)
rep = E.Replay(1000000, S, A, True)
rep.fill_random(1000000, 1)
eng.bind(rep)
eng.step_timed(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
for which in (0, 1):
    tr = eng.trace(which).astype(np.int64)
    desc = [l for l in eng.describe(which).splitlines() if l.startswith("L")]
    off = 0
    for line in desc:
        nwg = int(line.split("wg=")[1].split(":")[0])
        t = tr[off:off + nwg]
        off += nwg
        st = (t[:, 0] - t[:, 0].min()) * 10 / 1000.0
        en = (t[:, 3] - t[:, 0].min()) * 10 / 1000.0
        first_end = en.min()
        early = int((st < first_end).sum())
        print(f"g{which} {line.split(':')[0]:14s} started before first exit {early:5d}  "
              f"start pct50/90/max {np.percentile(st, 50):5.2f} {np.percentile(st, 90):5.2f} {st.max():5.2f}  first exit {first_end:5.2f}")
