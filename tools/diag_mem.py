"""Device memory of a TD7 Humanoid engine (+ an 8K-row replay) after its programs are built (GPU box):
python tools/diag_mem.py"""
import os, sys, ctypes
REPO = "/root/repo" if os.path.exists("/root/repo/bench.py") else os.getcwd()
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd")]
import torch
import bench
from rl import _engine as E
from rl.nn.layout import init_agent
for B in (256, 1024):
    torch.cuda.synchronize(0)
    f0, tot = torch.cuda.mem_get_info(0)
    S, A, _ = bench.TASKS["Humanoid-v4"]
    eng = E.Engine(E.make_config(E.RLE_TD7, S, A, 256, B, use_lap=True, seed=1, device=0), E.parse_plan(""))
    for net, params in init_agent("td7", S, A, 256, 1).items():
        for k, v in params.items():
            eng.set_param(net, k, v)
    rep = E.Replay(8192, S, A, True, device=0)
    rep.fill_random(8192, seed=0)
    eng.bind(rep)
    eng.step_timed(20)
    torch.cuda.synchronize(0)
    f1, _ = torch.cuda.mem_get_info(0)
    print(f"B={B}: engine + 8K replay device memory {(f0 - f1) / 2**30:.2f} GiB")
    del eng, rep
