"""CPU baseline for the multi-seed figure (8 processes x cores/8 threads, pinned).

P processes run the torch-CPU oracle's TD7 Humanoid B=256 step (bench.cpu_baseline: LAP over a
1M-row replay, same synthetic workload as the GPU bench) concurrently, each pinned to its own
T CPUs of this process's affinity set.  Aggregate = sum of the per-process rates (all run over
the same wall window).  Prints one JSON line.

Usage (GPU box host cores; no GPU is touched): python tools/cpu_multiseed.py --procs 8 --threads 2
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd")]


def child(idx, threads, seconds, cpus):
    os.sched_setaffinity(0, cpus)
    import torch

    torch.set_num_threads(threads)
    import bench

    r = bench.cpu_baseline(seconds, pin=False)  # (pinned here: this process's own CPU set)
    r["proc"] = idx
    r["cpus"] = sorted(cpus)
    print(json.dumps(r), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--threads", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=12.0)
    ap.add_argument("--child", type=int, default=-1)
    ap.add_argument("--cpus", type=str, default="")
    a = ap.parse_args()
    if a.child >= 0:
        return child(a.child, a.threads, a.seconds, {int(c) for c in a.cpus.split(",")})
    allowed = sorted(os.sched_getaffinity(0))
    need = a.procs * a.threads
    # one logical CPU per physical core (SMT siblings left idle), socket by socket, so each
    # process owns whole cores of one socket (/proc/cpuinfo physical id / core id)
    phys, seen = [], set()
    try:
        ent, cur = [], {}
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if not k:
                if cur:
                    ent.append(cur)
                cur = {}
            elif k in ("processor", "physical id", "core id"):
                cur[k] = int(v)
        if cur:
            ent.append(cur)
        for e in sorted(ent, key=lambda e: (e.get("physical id", 0), e.get("core id", 0), e["processor"])):
            key = (e.get("physical id", 0), e.get("core id", e["processor"]))
            if e["processor"] in allowed and key not in seen:
                seen.add(key)
                phys.append(e["processor"])
    except OSError:
        phys = []
    pool = phys if len(phys) >= need else allowed
    if need > len(pool):
        raise SystemExit(f"need {need} CPUs, {len(pool)} allowed")
    procs = []
    for i in range(a.procs):
        cpus = pool[i * a.threads:(i + 1) * a.threads]
        env = dict(os.environ, OMP_NUM_THREADS=str(a.threads))
        procs.append(subprocess.Popen([sys.executable, __file__, "--child", str(i), "--threads", str(a.threads),
                                       "--seconds", str(a.seconds), "--cpus", ",".join(map(str, cpus))],
                                      stdout=subprocess.PIPE, text=True, env=env))
    rows = []
    for p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise SystemExit(f"child failed rc={p.returncode}")
        rows.append(json.loads(out.strip().splitlines()[-1]))
    import bench

    agg = sum(r["value"] for r in rows)
    print(json.dumps({"metric": "gradient-steps/sec, TD7 Humanoid-v4 B=256, torch-CPU oracle, independent seeds",
                      "value": round(agg, 3), "unit": "gradient-steps/s", "procs": a.procs,
                      "threads_per_proc": a.threads, "cores": need, "kind": "port", "host": bench.host_cpu(),
                      "one_cpu_per_physical_core": pool is phys,
                      "per_proc": [r["value"] for r in rows], "cpus": [r["cpus"] for r in rows]}), flush=True)


if __name__ == "__main__":
    main()
