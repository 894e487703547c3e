"""Benchmark: TD7 Humanoid-v4 (obs 376, act 17) batch 256 gradient-steps/sec on MI355X.

One gradient step = one ``Agent.train_ops(replay.sample(B), replay)`` of the reference
(rl/runner/run.py:87-96): LAP sampling over a full 1M-transition HBM replay, encoder /
critic / (every 2nd step) actor updates with Adam, LAP priority update, hard target update
every 250 steps.  Synthetic replay: s, s' ~ N(0,1), a ~ U(-1,1),
r ~ N(0,1), notdone ~ Bernoulli(0.99), priorities 1.0; random-init weights of the
reference architecture (nn.Linear default init family).

Multi-GPU: ``python bench.py --gpus N`` starts N fresh rank processes itself (one per GPU,
before the parent touches any GPU); ``python -m torch.distributed.run --nproc-per-node N
bench.py --gpus N`` does the same through the launcher.  Each rank runs one independent seed
(replicas; no collective on the data path); a gloo group is used only for the
start barrier and the max-over-ranks timing.

Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "sac-td3-td7_amd")]

S, A, H, B, N_REPLAY = 376, 17, 256, 256, 1_000_000
METRIC = "gradient-steps/sec (whole node), TD7 Humanoid-v4 batch=256 at 1/2/4/8 GPUs"
TASKS = {"Humanoid-v4": (376, 17, 0.4), "Ant-v4": (27, 8, 1.0), "HalfCheetah-v4": (17, 6, 1.0)}
# SURVEY.md §8(d) algorithmic work per step: (algo, env, B) -> (GFLOP/step, HBM MB/step).
# The headline (default) config is TD7 Humanoid B=256; the others are BASELINE.json's
# secondary configs, run with --algo/--env/--batch (not part of the default JSON line).
WORK = {("td7", "Humanoid-v4", 256): (3.183, 41.37), ("td7", "Humanoid-v4", 1024): (12.733, 43.74),
        ("td7", "Ant-v4", 256): (2.502, 31.66), ("sac", "Humanoid-v4", 256): (1.121, 18.93),
        ("td3", "HalfCheetah-v4", 256): (0.449, 6.39)}
PEAK_FP32_TFLOPS = 157.3   # MI355X fp32 MFMA dense (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
# SURVEY.md §8(d) algorithmic work for TD7 Humanoid B=256: 6,217,088 MAC/sample (3.183 GFLOP/step).
SURVEY_MACS_PER_SAMPLE = 6_217_088


def td7_macs_per_sample(S, A, H, policy_freq=2):
    """Algorithmic MACs per sample (SURVEY.md §8d convention): forward i*o, weight-grad i*o for
    trained layers, input-grad only for needed columns, no grads into frozen nets, policy phase
    weighted by 1/policy_freq."""
    HH = H * H
    enc_fwd = 2 * (S * H + 2 * HH) + (H + A) * H + 2 * HH          # zs(s'), zs(s), zsa(s)
    enc_w = S * H + 2 * HH + (H + A) * H + 2 * HH
    enc_i = 5 * HH                                                 # zsa3, zsa2, zsa1[zs], zs3, zs2
    E = enc_fwd + enc_w + enc_i
    critic_fwd = (S + A) * H + 3 * HH + HH + H                     # q01, q1 (3H in), q2, q3
    actor_fwd = S * H + 2 * HH + HH + H * A                        # l0, l1 (2H in), l2, l3
    zs = S * H + 2 * HH
    zsa = (H + A) * H + 2 * HH
    Q = (zs + actor_fwd + zsa + 2 * critic_fwd                     # target branch
         + zs + zsa                                                # fixed encoder on s
         + 2 * critic_fwd + 2 * critic_fwd                         # online fwd + weight grads
         + 2 * (H + HH + HH))                                      # input grads q3, q2, q1[norm]
    P = (actor_fwd + zsa + 2 * critic_fwd
         + 2 * (H + HH + 2 * HH + A * H)                           # critics: q3, q2, q1[norm,zsa], q01[a]
         + HH + HH + A * H                                         # fe.zsa3, zsa2, zsa1[a]
         + H * A + HH + HH                                         # actor l3, l2, l1[l0]
         + actor_fwd)                                              # actor weight grads
    return E + Q + P / policy_freq


def td7_param_counts(S, A, H):
    enc = S * H + H + 2 * (HH := H * H) + 2 * H + (H + A) * H + H + 2 * HH + 2 * H
    actor = S * H + H + 2 * HH + H + HH + H + A * H + A
    critic = (S + A) * H + H + 3 * HH + H + HH + H + H + 1
    return enc, actor, critic


def td7_bytes_per_step(S, A, H, B, N, target_update_rate=250, policy_freq=2):
    """Algorithmic HBM bytes per step: gather + index/priority + LAP scan +
    Adam 28 B/updated param + hard-copy traffic amortised."""
    enc, actor, critic = td7_param_counts(S, A, H)
    gather = B * (2 * S + A + 2) * 4
    adam = 28 * (enc + 2 * critic + actor / policy_freq)
    hard = 8 * (2 * critic + 2 * enc) / target_update_rate
    return gather + B * 8 + 4 * N + adam + hard


def socket_cores():
    """(socket, CPUs, physical cores of that socket): one logical CPU per physical core of the
    socket holding this process's first allowed CPU, among the allowed CPUs (/proc/cpuinfo)."""
    entries, cur = [], {}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if not k:
                    if cur:
                        entries.append(cur)
                    cur = {}
                elif k in ("processor", "physical id", "core id"):
                    cur[k] = int(v)
            if cur:
                entries.append(cur)
    except OSError:
        entries = []
    allowed = sorted(os.sched_getaffinity(0))
    by_cpu = {e["processor"]: e for e in entries if "processor" in e}
    if not allowed or allowed[0] not in by_cpu or "core id" not in by_cpu[allowed[0]]:
        return 0, allowed, len(allowed)
    sock = by_cpu[allowed[0]].get("physical id", 0)
    cores = {e.get("core id") for e in entries if e.get("physical id", 0) == sock}
    seen, cpus = set(), []
    for c in allowed:
        e = by_cpu.get(c)
        if e is None or e.get("physical id", 0) != sock or e.get("core id") in seen:
            continue
        seen.add(e.get("core id"))
        cpus.append(c)
    return sock, cpus, len(cores)


def cpu_baseline(seconds=12.0, algo="td7", env="Humanoid-v4", batch=B, lap=True, pin=True, cpus=None,
                 n_replay=N_REPLAY):
    """Oracle (torch-CPU restatement of train_ops + replay sample) on host cores, same
    synthetic workload as the GPU run (full 1M replay).  SURVEY §8(d): torch threads = the
    physical cores of one socket, the process pinned to one logical CPU of each (restored after).
    cpus: pin to exactly these CPUs instead, one torch thread each (the N-process figure of
    BASELINE.md: one process per rank, each on its own slice of the host, cpu_baseline_ranks)."""
    import torch

    from oracle import agents, replay, spec

    s_dim, a_dim, hi = TASKS[env]
    old_aff, old_threads = os.sched_getaffinity(0), torch.get_num_threads()
    if cpus is not None:
        sock, ncore = -1, len(cpus)
    else:
        sock, cpus, ncore = socket_cores()
        # the GPU box is a one-GPU share of an 8-GPU host: 16 of its CPUs are this box's (more threads
        # contend with other tenants and measure less); RLE_CPU_THREADS overrides
        cpus = cpus[:int(os.environ.get("RLE_CPU_THREADS", "16"))]
    if pin and cpus:
        os.sched_setaffinity(0, cpus)
        torch.set_num_threads(len(cpus))
    try:
        return _cpu_run(seconds, algo, env, batch, lap, s_dim, a_dim, hi, agents, replay, spec, torch,
                        {"socket": sock, "physical_cores_socket": ncore, "pinned_cpus": len(cpus) if pin else 0},
                        n_replay)
    finally:
        if pin and cpus:
            os.sched_setaffinity(0, old_aff)
            torch.set_num_threads(old_threads)


def _cpu_run(seconds, algo, env, batch, lap, s_dim, a_dim, hi, agents, replay, spec, torch, pinning,
             n_replay=N_REPLAY):
    threads = torch.get_num_threads()
    rng = np.random.default_rng(0)
    nets = spec.agent_params(algo, s_dim, a_dim, H, 123)
    orc = agents.make_oracle(algo, nets, a_dim, lap)
    N = n_replay
    rep = replay.Replay(N, s_dim, a_dim, np.full(a_dim, hi, np.float32), np.zeros(a_dim, np.float32), lap)
    blk = 4096
    base_s = rng.standard_normal((blk, s_dim), dtype=np.float32)
    base_s2 = rng.standard_normal((blk, s_dim), dtype=np.float32)
    for i in range(0, N, blk):
        n = min(blk, N - i)
        rep.state[i:i + n] = base_s[:n]
        rep.next_state[i:i + n] = base_s2[:n]
    rep.action[:] = rng.uniform(-1, 1, (N, a_dim)).astype(np.float32)
    rep.reward[:, 0] = rng.standard_normal(N).astype(np.float32)
    rep.done[:, 0] = (rng.random(N) < 0.99).astype(np.float32)
    rep.priority[:] = 1.0
    rep.size, rep.ptr = N, 0

    def one():
        u = rng.random(batch, dtype=np.float32)
        batch_d = rep.gather(rep.sample_indices(u))
        eps = rng.standard_normal((batch, a_dim), dtype=np.float32)
        if algo == "sac":
            orc.step(batch_d, rep, eps, rng.standard_normal((batch, a_dim), dtype=np.float32))
        else:
            orc.step(batch_d, rep, eps)

    for _ in range(3):
        one()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < seconds or n < 10:
        one()
        n += 1
    dt = time.perf_counter() - t0
    hc = host_cpu()
    hc.update(pinning)
    return {"value": round(n / dt, 3), "unit": "gradient-steps/s", "cores": threads, "threads": threads,
            "kind": "port",
            "sample": f"{n} {algo.upper()} {env} B={batch} steps ({'LAP' if lap else 'uniform'} over a "
                      f"{N // 1000}K replay) of the torch-CPU oracle, {dt:.1f} s, torch threads={threads} "
                      + (f"pinned one per physical core of socket {pinning['socket']} "
                         f"({pinning['physical_cores_socket']} physical cores; the box's share is 16 CPUs)"
                         if pinning["socket"] >= 0 else "pinned to the rank's own CPU slice"),
            # the GPU boxes share their host with other jobs: the same oracle run measured 34.5-53.9 steps/s
            # (TD7 Humanoid B=256) on different boxes in rounds 3-4, i.e. about 1.5x box to box
            "box_to_box_spread": "about 2x (TD7 Humanoid B=256: 28.5-53.9 steps/s across GPU boxes and runs, rounds 3-5)",
            "host": hc}


def host_cpu():
    """CPU model, sockets and logical CPUs of this host (/proc/cpuinfo), and the CPUs this
    process may run on."""
    model, sockets, logical = "unknown", set(), 0
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name" and model == "unknown":
                    model = v
                elif k == "physical id":
                    sockets.add(v)
                elif k == "processor":
                    logical += 1
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = os.cpu_count() or 0
    return {"cpu_model": model, "sockets": max(1, len(sockets)), "logical_cpus": logical,
            "cpus_allowed": allowed}


def max_over_ranks(vals, dist=None):
    """Element-wise max of per-rank timings (the slowest rank defines the job's time)."""
    if dist is None:
        return [float(v) for v in vals]
    import torch

    t = torch.tensor(vals, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t]


def _latest_profile(name):
    """Newest committed profiles/rNN_<name> (the round's own evidence), or None."""
    import glob

    c = sorted(glob.glob(os.path.join(REPO, "profiles", f"r[0-9][0-9]_{name}")))
    return c[-1] if c else None


PMC_FILES = {("td7", "Humanoid-v4", 256): "pmc.json", ("td7", "Humanoid-v4", 1024): "pmc_td7_b1024.json",
             ("td7", "Ant-v4", 256): "pmc_td7_ant.json", ("td3", "HalfCheetah-v4", 256): "pmc_td3_halfcheetah.json",
             ("sac", "Humanoid-v4", 256): "pmc_sac_humanoid.json"}


def pmc_evidence(cfg=("td7", "Humanoid-v4", 256)):
    """Counters of the dominant kernel from the committed PMC summary of the same command
    (tools/pmc.sh + tools/pmc_summary.py --json; mean per rle_level dispatch of a
    `bench.py --steps 200` run), NOT measured in this process:
    * traffic: HBM bytes per launch = 2 x FETCH_SIZE (gfx950 reports half of wide coalesced
      reads, MI355X_MICROARCH.md 'HBM') + WRITE_SIZE, both in KB;
    * mfma_busy: SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x shader cycles), shader cycles =
      GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs; it reads high on dispatches this short,
      MI355X_MICROARCH.md 'DVFS', so this fraction is a lower bound; summarize() adds the same
      cycles over the measured launch time)."""
    path = _latest_profile(PMC_FILES[cfg])
    if path is None:
        return {"traffic": None}
    with open(path) as f:
        pmc = json.load(f)
    out = {"traffic": round((2.0 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024.0),
           "traffic_source": f"profiles/{os.path.basename(path)} (rocprofv3 --pmc, mean per rle_level dispatch)"}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in pmc and "GRBM_GUI_ACTIVE" in pmc:
        cycles = pmc["GRBM_GUI_ACTIVE"] / 8.0
        out["mfma_busy"] = round(pmc["SQ_VALU_MFMA_BUSY_CYCLES"] / (cycles * 256 * 4), 5)
        out["mfma_busy_source"] = out["traffic_source"]
    return out


def traffic_model_evidence():
    """How much of the measured per-level HBM traffic the per-XCD traffic model explains (tools/pmc_levels.py on
    the committed per-level PMC passes of the 6-step TD7 graph: every XCD's L2 fetches its own copy of what its
    workgroups read; engine.cpp LevelTraffic).  {} when no such table is committed."""
    path = _latest_profile("pmc_levels.txt")
    if path is None:
        return {}
    last = None
    with open(path) as f:
        for line in f:
            parts = line.split()
            if parts and parts[0] == "sum" and len(parts) == 10:
                last = parts
    if last is None:
        return {}
    model, pmc = float(last[7]), float(last[8])
    return {"traffic_model_xcd": {"model_KB_per_graph": model, "pmc_KB_per_graph": pmc,
                                  "explained_frac": round(model / pmc, 4),
                                  "reads_pmc_over_model": float(last[3]), "stores_pmc_over_model": float(last[6]),
                                  "source": f"profiles/{os.path.basename(path)} (per level of the 6-step graph)"}}


def _pmc_value(key, cfg=("td7", "Humanoid-v4", 256)):
    path = _latest_profile(PMC_FILES[cfg])
    if path is None:
        return None
    with open(path) as f:
        return json.load(f).get(key)


def gather_evidence(s_dim, a_dim, batch, n_replay, lap):
    """Achieved GB/s of the replay sampler (OP_SAMPLE_GATHER: three-level LAP index search + row
    gather, kernels.hip op_sample_gather) from the committed rocprofv3 kernel trace of standalone
    sampler dispatches (tools/sampler_prof.py -> tools/sampler_summary.py: B = 256 queries over a
    1M-row TD7 Humanoid replay, one rle_level launch each; mean duration after warm-up).

    Bytes per query are what the kernel issues: the block sums its lanes load (64 lanes x
    ceil(blocks / 64) x 8 B), the 64 sub-block sums (8 B) and 64 priorities (4 B) of the chosen
    block / sub-block, the row (2 Sp + Ap floats + reward + notdone) and its stores into the
    batch's T images (+ reward, notdone, index, uniform).  The PMC traffic of the same dispatches
    (2 x FETCH_SIZE + WRITE_SIZE, profiles/rNN_sampler_pmc.json) is reported beside it."""
    path = _latest_profile("sampler.csv")
    if path is None or (s_dim, a_dim, batch, n_replay) != (S, A, B, N_REPLAY):
        return {}
    with open(path) as f:
        durs = [int(r.split(",")[2]) for r in f.read().splitlines()[2:] if r]
    durs = durs[10:]  # (tools/sampler_summary.py: the first 10 dispatches are warm-up)
    us = sum(durs) / len(durs) / 1e3
    sp = (s_dim + 15) // 16 * 16
    ap = (a_dim + 15) // 16 * 16
    nblk = math.ceil(n_replay / 4096)
    search = (64 * math.ceil(nblk / 64) * 8 + 64 * 8 + 64 * 4) if lap else 0
    row_rd = (2 * sp + ap) * 4 + 8
    row_wr = (2 * sp + ap) * 4 + 4 + 4 + 8 + 4
    q = search + row_rd + row_wr
    out = {"gather_GBs": round(batch * q / (us * 1e-6) / 1e9, 2), "gather_bytes": batch * q,
           "gather_bytes_per_query": {"search": search, "row_read": row_rd, "row_write": row_wr},
           "gather_us": round(us, 3), "gather_frac_hbm": round(batch * q / (us * 1e-6) / 1e9 / PEAK_HBM_GBS, 5),
           "gather_source": f"profiles/{os.path.basename(path)} (rocprofv3 --kernel-trace, standalone sampler "
                            f"dispatches, B={batch})"}
    pm = _latest_profile("sampler_pmc.json")
    if pm is not None:
        with open(pm) as f:
            c = json.load(f)
        out["gather_traffic"] = round((2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0)
        out["gather_traffic_source"] = f"profiles/{os.path.basename(pm)} (rocprofv3 --pmc, same dispatches)"
    return out


def summarize(n_gpus, steps, warmup, wall, gpu_s, lv_policy, lv_plain, algo="td7", env="Humanoid-v4",
              batch=B, lap=True, launches=None, dispatch=1):
    """The bench JSON line (everything but cpu_baseline) from the max-over-ranks timings.  dispatch: the
    engine's rle_plan.dispatch (1 direct AQL, 0 hipGraph replays, 2 launches on the stream)."""
    value = n_gpus * steps / wall
    headline = (algo, env, batch) == ("td7", "Humanoid-v4", B)
    if headline:
        macs = SURVEY_MACS_PER_SAMPLE  # the §8(d) contract figure (own derivation: td7_macs_per_sample)
        flop_step = 2.0 * macs * B
        bytes_step = td7_bytes_per_step(S, A, H, B, N_REPLAY)
    else:
        gflop, mb = WORK[(algo, env, batch)]
        flop_step, bytes_step = gflop * 1e9, mb * 1e6
    s_dim, a_dim, _ = TASKS[env]
    # launches per step: counted by the engine over the timed steps (rle_launch_count: single-
    # and multi-step graphs, batch primes, hard updates); else the single-step graph average
    if launches is None:
        launches = (lv_policy + lv_plain) / 2.0
    per_launch_s = gpu_s / (steps * launches)
    achieved = flop_step / launches / per_launch_s / 1e12
    roofline = {
        "bound": "mfma",
        "achieved": round(achieved, 3),
        "peak": PEAK_FP32_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved / PEAK_FP32_TFLOPS, 5),
        **pmc_evidence((algo, env, batch)),
        "traffic_algorithmic": round(bytes_step / launches),
        "kernel": "rle_level (one launch per dependency level of the step graph)",
        "flop_per_step": flop_step,
        "launches_per_step": round(launches, 4),
        "avg_launch_us": round(per_launch_s * 1e6, 3),
        "hbm_bytes_per_step_algorithmic": round(bytes_step),
        "hbm_achieved_GBs": round(bytes_step * steps / gpu_s / 1e9, 2),
    }
    if headline:
        roofline.update(gather_evidence(s_dim, a_dim, batch, N_REPLAY, lap))
        roofline.update(traffic_model_evidence())
    busy = _pmc_value("SQ_VALU_MFMA_BUSY_CYCLES", (algo, env, batch))
    if busy is not None:  # the same counter over this run's measured launch duration, 2.4 GHz
        roofline["mfma_busy_vs_launch_time"] = round(busy / (1024 * 2.4e9 * per_launch_s), 5)
    metric = METRIC if headline else (f"gradient-steps/sec, {algo.upper()} {env} batch={batch}"
                                      f"{' LAP' if lap else ''} (secondary config)")
    return {
        "metric": metric,
        "value": round(value, 2),
        "unit": "gradient-steps/s",
        "n_gpus": n_gpus,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(wall / steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic",
        "config": {"workload": f"{algo.upper()} {env} gradient step, {'LAP' if lap else 'uniform'} over 1M HBM replay",
                   "algo": algo, "obs_dim": s_dim, "act_dim": a_dim, "hidden": H, "batch": batch,
                   "replay": N_REPLAY, "lap": lap, "policy_freq": 2, "target_update_rate": 250,
                   "parallelism": f"replicas x{n_gpus} (one seed per GPU, no collective)"},
        "roofline": roofline,
        # the engine's own elapsed time over the timed steps: under the default direct AQL dispatch it is host
        # wall time from the first doorbell to the last packet's completion signal (rle_step_timed, rle.h);
        # with rle_plan dispatch 0 / 2 HIP event time on the engine's stream
        "engine_s": round(gpu_s, 6),
        "engine_timer": ENGINE_TIMERS[dispatch],
    }


ENGINE_TIMERS = {1: "host wall, first AQL doorbell to completion signal", 0: "HIP events on the engine stream",
                 2: "HIP events on the engine stream"}


def multi_seed(args, K, world, rank, local, dist, algo_id, lap, E, init_agent, cuda_sync, chunk=25):
    """K independent seeds per GPU: K engines, each with its own replay,
    weights, Philox stream and HIP stream, stepped round-robin in chunks without host syncs.
    value = steps of all seeds on all ranks / max-rank wall time."""

    s_dim, a_dim, _ = TASKS[args.env]
    engs = []
    for k in range(K):
        seed = 111 * (rank * K + k + 1)
        eng = E.Engine(E.make_config(algo_id, s_dim, a_dim, H, args.batch, use_lap=lap, seed=seed, device=local),
                       E.parse_plan(args.plan))
        for net, params in init_agent(args.algo, s_dim, a_dim, H, 123 + rank * K + k).items():
            for name, v in params.items():
                eng.set_param(net, name, v)
        rep = E.Replay(N_REPLAY, s_dim, a_dim, lap, device=local)
        rep.fill_random(N_REPLAY, seed=rank * K + k)
        eng.bind(rep)
        engs.append((eng, rep))

    def run(n):
        done = 0
        while done < n:
            c = min(chunk, n - done)
            for eng, _ in engs:
                eng.step_async(c)
            done += c
        for eng, _ in engs:
            eng.synchronize()

    run(args.warmup)
    if dist:
        dist.barrier()
    cuda_sync(local)
    t0 = time.perf_counter()
    run(args.steps)
    cuda_sync(local)
    wall = max_over_ranks([time.perf_counter() - t0], dist)[0]
    if rank == 0:
        gflop, mb = (SURVEY_MACS_PER_SAMPLE * 2.0 * B / 1e9, None) if (args.algo, args.env, args.batch) == (
            "td7", "Humanoid-v4", B) else WORK[(args.algo, args.env, args.batch)]
        value = world * K * args.steps / wall
        out = {
            "metric": f"gradient-steps/sec, {K} independent seeds per GPU, "
                      f"{args.algo.upper()} {args.env} "
                      f"batch={args.batch} (secondary: SURVEY §8(f) rank 4)",
            "value": round(value, 2), "unit": "gradient-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": f"{K} x {args.algo.upper()} {args.env} gradient step per GPU",
                       "seeds_per_gpu": K, "batch": args.batch, "replay": N_REPLAY, "lap": lap,
                       "parallelism": f"replicas x{world * K} ({K} seeds per GPU, one HIP stream each)",
                       "plan": engs[0][0].plan()},
            "roofline": {"bound": "mfma", "achieved": round(gflop * 1e9 * value / world / 1e12, 3),
                         "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(gflop * 1e9 * value / world / 1e12 / PEAK_FP32_TFLOPS, 5),
                         "traffic": None, "note": "device aggregate over the K seeds (wall clock)"},
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()


def kfd_gpu_count(root="/sys/class/kfd/kfd/topology/nodes"):
    """GPUs visible to this process without any HIP / HSA call: the KFD topology nodes that have
    SIMDs (/sys/class/kfd/kfd/topology/nodes/*/properties), narrowed by HIP_VISIBLE_DEVICES /
    ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES when set."""
    import glob

    n = 0
    for f in glob.glob(os.path.join(root, "*", "properties")):
        try:
            props = dict(line.split() for line in open(f) if len(line.split()) == 2)
        except OSError:
            continue
        n += int(props.get("simd_count", "0")) > 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def parse_cpulist(text):
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11] (sysfs cpulist format)."""
    out = []
    for part in filter(None, (t.strip() for t in text.split(","))):
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def kfd_gpu_nodes(root="/sys/class/kfd/kfd/topology/nodes"):
    """The KFD topology's GPU nodes (those with SIMDs) in node order -- the order HIP numbers the devices
    in -- narrowed by *_VISIBLE_DEVICES (integer lists) when set: [(node, properties dict)]."""
    import glob

    nodes = []
    for f in glob.glob(os.path.join(root, "*", "properties")):
        try:
            props = dict(line.split() for line in open(f) if len(line.split()) == 2)
            node = int(os.path.basename(os.path.dirname(f)))
        except (OSError, ValueError):
            continue
        if int(props.get("simd_count", "0")) > 0:
            nodes.append((node, props))
    nodes.sort(key=lambda t: t[0])
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            try:
                idx = [int(x) for x in v.split(",") if x.strip() != ""]
            except ValueError:
                continue
            nodes = [nodes[i] for i in idx if 0 <= i < len(nodes)]
    return nodes


def gpu_local_cpus(local, n_local, kfd_root="/sys/class/kfd/kfd/topology/nodes", pci_root="/sys/bus/pci/devices",
                   allowed=None):
    """The host CPUs rank `local` (of n_local ranks on this node, one GPU each) is pinned to, without any
    HIP / HSA call (bench.py pins its ranks before they touch a GPU): the CPUs NUMA-local to its GPU (the
    PCI device's local_cpulist, found from the KFD node's domain / location_id) among this process's
    allowed CPUs, split evenly among the ranks whose GPUs share them -- where MuJoCo stepping for that
    seed would run.  Returns (cpus, info); the allowed CPUs split by rank when the GPU's
    locality cannot be read or none of its local CPUs is allowed."""
    allowed = sorted(os.sched_getaffinity(0) if allowed is None else allowed)
    nodes = kfd_gpu_nodes(kfd_root)

    def local_set(i):
        if i >= len(nodes):
            return None, None
        props = nodes[i][1]
        loc, dom = int(props.get("location_id", "0")), int(props.get("domain", "0"))
        bdf = f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 31:02x}.{loc & 7:x}"
        try:
            with open(os.path.join(pci_root, bdf, "local_cpulist")) as f:
                cpus = [c for c in parse_cpulist(f.read()) if c in set(allowed)]
            with open(os.path.join(pci_root, bdf, "numa_node")) as f:
                numa = int(f.read().strip())
        except (OSError, ValueError):
            return bdf, None
        return bdf, (numa, tuple(cpus)) if cpus else None

    sets = [local_set(i) for i in range(n_local)]
    bdf, mine = sets[local] if local < len(sets) else (None, None)
    if mine is None:  # (no locality: an even split of the allowed CPUs by rank)
        k = max(1, len(allowed) // max(1, n_local))
        cpus = allowed[local * k:(local + 1) * k] or allowed
        return cpus, {"gpu_bdf": bdf, "numa_node": None, "numa_local": False, "cpus": len(cpus)}
    sharers = [i for i, t in enumerate(sets) if t[1] is not None and t[1][1] == mine[1]]
    k = max(1, len(mine[1]) // len(sharers))
    j = sharers.index(local)
    cpus = list(mine[1][j * k:(j + 1) * k]) or list(mine[1])
    return cpus, {"gpu_bdf": bdf, "numa_node": mine[0], "numa_local": True, "cpus": len(cpus)}


def physical_core_cpus(cpus):
    """One logical CPU per physical core among `cpus` (/proc/cpuinfo physical id / core id)."""
    by_cpu, cur = {}, {}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if not k:
                    if "processor" in cur:
                        by_cpu[cur["processor"]] = cur
                    cur = {}
                elif k in ("processor", "physical id", "core id"):
                    cur[k] = int(v)
        if "processor" in cur:
            by_cpu[cur["processor"]] = cur
    except OSError:
        return list(cpus)
    seen, out = set(), []
    for c in cpus:
        e = by_cpu.get(c, {})
        key = (e.get("physical id", 0), e.get("core id", ("cpu", c)))
        if key not in seen:
            seen.add(key)
            out.append(c)
    return out


def cpu_baseline_ranks(dist, rank, world, cpus, seconds, algo, env, batch, lap, n_replay=N_REPLAY):
    """BASELINE.md's N-process CPU figure for an N-GPU line: every rank runs the torch-CPU oracle at the
    same time, pinned to its own CPU slice (gpu_local_cpus: cores/N of the host, one thread per physical
    core), after the GPU timing; rank 0 gets the sum.  None on ranks other than 0."""
    dist.barrier()
    r = cpu_baseline(seconds, algo, env, batch, lap, cpus=physical_core_cpus(cpus), n_replay=n_replay)
    rows = [None] * world
    dist.all_gather_object(rows, r)
    if rank != 0:
        return None
    return {"value": round(sum(x["value"] for x in rows), 3), "unit": "gradient-steps/s",
            "cores": sum(x["cores"] for x in rows), "kind": "port", "procs": world,
            "threads_per_proc": [x["threads"] for x in rows], "per_proc": [x["value"] for x in rows],
            "sample": f"{world} concurrent processes (one per rank), each: {rows[0]['sample']}",
            "host": rows[0]["host"]}


def launch_ranks(n, argv, device_count):
    """``--gpus N`` without a launcher (WORLD_SIZE unset): start N fresh rank processes of this
    script, one per GPU, each with RANK / LOCAL_RANK / WORLD_SIZE and a local rendezvous.  The
    parent has not initialised any GPU (it only counted devices); ranks inherit stdout, so rank
    0's JSON line is the output.  Returns the first failing rank's exit code, else 0."""
    import socket
    import subprocess

    visible = device_count()
    if n > visible:
        raise SystemExit(f"bench.py: --gpus {n} but only {visible} GPU(s) visible")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:  # the others would wait at the barrier forever
                    q.terminate()
        time.sleep(0.05)
    return rc


def _stub_engine_module(path):
    """Test hook (tests/test_host.py): RLE_BENCH_STUB=<file> replaces the engine module by a
    CPU stub so the rank launcher and the JSON line can be tested without a GPU."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("rle_bench_stub", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-replay", type=int, default=N_REPLAY,
                    help="replay rows of the CPU baseline's oracle (default the GPU run's 1M; tests use fewer)")
    ap.add_argument("--algo", choices=("td7", "td3", "sac"), default="td7")
    ap.add_argument("--env", choices=tuple(TASKS), default="Humanoid-v4")
    ap.add_argument("--batch", type=int, default=B)
    ap.add_argument("--seeds-per-gpu", type=int, default=1,
                    help="independent seeds (engines, one stream each) sharing each GPU (SURVEY §8(f) rank 4)")
    ap.add_argument("--plan", default=os.environ.get("RLE_PLAN", ""),
                    help="step-program plan (rle_plan) fields, e.g. 'level_cap=512,fuse_off=headdx' (A/B tools; "
                         "default: the engine's default plan, or $RLE_PLAN); reported in the JSON line's config")
    args = ap.parse_args()
    if (args.algo, args.env, args.batch) not in WORK:
        ap.error(f"no SURVEY §8(d) work figures for {args.algo} {args.env} B={args.batch}")
    lap = args.algo == "td7"  # TD7 runs LAP (td7_exp.sh); SAC / TD3 the uniform replay
    stub = _stub_engine_module(os.environ["RLE_BENCH_STUB"]) if os.environ.get("RLE_BENCH_STUB") else None

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        if stub:
            count = stub.device_count
        else:
            import torch

            count = kfd_gpu_count  # (no HIP call in the parent before the ranks start)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], count))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    pin_cpus, pinning = None, None
    if world > 1:
        # each rank on its GPU's NUMA-local cores (its share of them), before anything touches a GPU
        n_local = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        pin_cpus, pinning = gpu_local_cpus(local, n_local)
        os.sched_setaffinity(0, pin_cpus)
        import torch.distributed as dist  # gloo: start barrier + timing reduction only
        dist.init_process_group("gloo")

    if stub:
        E, init_agent, cuda_sync = stub, stub.init_agent, stub.synchronize
    else:
        import torch

        from rl import _engine as E
        from rl.nn.layout import init_agent

        cuda_sync = torch.cuda.synchronize

    # --- engine: one independent seed per GPU (seed 111, 222, ... as scripts/td7_exp.sh)
    s_dim, a_dim, _ = TASKS[args.env]
    algo_id = {"td7": E.RLE_TD7, "td3": E.RLE_TD3, "sac": E.RLE_SAC}[args.algo]
    K = max(1, args.seeds_per_gpu)
    if K > 1:
        # K seeds on streams: the tile planner sizes each seed's levels for 512 resident workgroups
        # (half the device) so two seeds' levels co-reside (A/B, 3 seeds: 13.1k default, 14.1k at 512,
        # 13.9k at 384; profiles/r03_ab.txt "multiseed_cap"), 384 from 4 seeds on (round 6, 2 pairs each:
        # 4 seeds 15.46k at 512 / 15.59k at 384, 2 and 3 seeds 6% / 3% slower at 384;
        # profiles/r06_ab_multiseed_cap.txt).  --plan overrides.
        if "level_cap" not in args.plan:
            args.plan = ",".join(filter(None, [args.plan, f"level_cap={512 if K < 4 else 384}"]))
        return multi_seed(args, K, world, rank, local, dist, algo_id, lap, E, init_agent, cuda_sync)
    cfg = E.make_config(algo_id, s_dim, a_dim, H, args.batch, use_lap=lap, seed=111 * (rank + 1), device=local)
    eng = E.Engine(cfg, E.parse_plan(args.plan))
    for net, params in init_agent(args.algo, s_dim, a_dim, H, 123 + rank).items():
        for name, v in params.items():
            eng.set_param(net, name, v)
    rep = E.Replay(N_REPLAY, s_dim, a_dim, lap, device=local)
    rep.fill_random(N_REPLAY, seed=rank)
    eng.bind(rep)
    lv_policy, lv_plain = eng.graph_stats()

    eng.step_timed(args.warmup)
    if dist:
        dist.barrier()
    cuda_sync(local)
    n_l0 = eng.launch_count()
    t0 = time.perf_counter()
    c0 = time.thread_time()  # (CPU time of this thread: rle_step_timed waits in it, ctypes releases the GIL)
    gpu_ms = eng.step_timed(args.steps)
    c1 = time.thread_time()
    cuda_sync(local)
    t1 = time.perf_counter()
    launches = (eng.launch_count() - n_l0) / args.steps
    wall = t1 - t0
    wall, gpu_s = max_over_ranks([wall, gpu_ms / 1e3], dist)

    cb = None
    if world > 1 and not args.no_cpu_baseline:  # (every rank: the N concurrent CPU processes)
        cb = cpu_baseline_ranks(dist, rank, world, pin_cpus, args.cpu_seconds, args.algo, args.env, args.batch, lap,
                                args.cpu_replay)
    pins = [None] * world
    if dist:
        dist.all_gather_object(pins, pinning)
    if rank != 0:
        if dist:
            dist.barrier()
        return
    plan = eng.plan()
    out = summarize(world, args.steps, args.warmup, wall, gpu_s, lv_policy, lv_plain, args.algo, args.env,
                    args.batch, lap, launches, plan.get("dispatch", 1))
    out["config"]["plan"] = plan
    # share of the timed region the stepping thread spent on a host core (the AQL wait sleeps: engine.cpp
    # aql_wait_step), i.e. what is left for MuJoCo stepping beside the engine (north_star)
    out["host_thread_busy_frac"] = round((c1 - c0) / max(wall, 1e-9), 4)
    if world > 1:
        out["config"]["rank_pinning"] = pins
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.algo, args.env, args.batch, lap,
                                           n_replay=args.cpu_replay)
    elif cb is not None:
        out["cpu_baseline"] = cb
    print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()


if __name__ == "__main__":
    main()
