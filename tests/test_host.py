"""Host-side logic of the reference-interface mirror and the bench (no GPU calls)."""

import json
import math
import os
import subprocess
import sys

import numpy as np
import pytest

from rl import _engine as E
from rl.agent import SAC, TD3, TD7
from rl.replay_memory import DeviceBatch, LAPReplayMemory
from rl.sampler import RandomSampler
from rl.utils import get_action_bias_scale, get_state_action_dims, register_env

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_env_table_matches_mujoco_v4_spaces():
    # SURVEY.md §8 dims table (miscellaneous.py:50-66 on the real gym spaces)
    assert get_state_action_dims("Humanoid-v4") == (376, 17)
    assert get_state_action_dims("Ant-v4") == (27, 8)
    assert get_state_action_dims("HalfCheetah-v4") == (17, 6)
    bias, scale = get_action_bias_scale("Humanoid-v4")
    assert bias.dtype == np.float32 and np.all(bias == 0) and np.all(scale == np.float32(0.4))
    register_env("Odd-v0", 5, 2, [-1.0, 0.0], [3.0, 1.0])
    bias, scale = get_action_bias_scale("Odd-v0")
    np.testing.assert_array_equal(bias, [1.0, 0.5])
    np.testing.assert_array_equal(scale, [2.0, 0.5])
    with pytest.raises(KeyError):
        get_state_action_dims("NoSuchEnv-v9")


def test_random_sampler_stays_in_box():
    rs = RandomSampler("Humanoid-v4")
    a = np.stack([rs.sample() for _ in range(200)])
    assert a.shape == (200, 17) and np.all(np.abs(a) <= 0.4)


def test_append_normalisation_uses_reference_dtypes():
    # lap.py:35: action / scale - bias in the operands' NumPy dtypes, stored then cast to fp32
    rep = LAPReplayMemory.__new__(LAPReplayMemory)
    rep.action_bias, rep.action_scale = get_action_bias_scale("Humanoid-v4")
    a64 = np.linspace(-0.4, 0.4, 17)
    np.testing.assert_array_equal(rep._normalise(a64), a64 / np.float32(0.4) - 0.0)
    a32 = a64.astype(np.float32)
    out = rep._normalise(a32)
    assert out.dtype == np.float32


def test_info_rows_map_to_reference_keys():
    td7 = TD7.__new__(TD7)
    row = np.array([1.0, 2.0, np.nan, 0, 0, 0, 0, 0], np.float32)
    assert td7._info(row) == {"train/encoder": 1.0, "train/q_fn": 2.0, "train/policy": None}
    td3 = TD3.__new__(TD3)
    assert td3._info(np.array([0.5, np.nan, np.nan], np.float32)) == {
        "train/q_fn": 0.5, "train/policy": None, "norm/policy": None}
    sac = SAC.__new__(SAC)
    sac.auto_tmp_mode = True
    got = sac._info(np.arange(8, dtype=np.float32))
    assert list(got) == ["train/q_fn", "tmp", "norm/tmp", "train/policy", "train/tmp", "entropy"]
    sac.auto_tmp_mode = False
    nan_loss = sac._info(np.array([np.nan, 1.0, 2.0], np.float32))
    assert math.isnan(nan_loss["train/q_fn"])  # a diverged loss stays NaN, only policy keys go None


def test_train_ops_rejects_malformed_batches_and_foreign_replays():
    """A BATCH dict without the reference's keys (annotation.py:23-30), or a device batch drawn from
    another replay than the one passed, is a ValueError."""
    td7 = TD7.__new__(TD7)
    with pytest.raises(ValueError):
        td7.train_ops({"state": np.zeros((4, 3))}, None)
    rep_a, rep_b = object(), object()
    batch = DeviceBatch({}, np.zeros(4, np.int64), rep_a)
    with pytest.raises(ValueError):
        td7.train_ops(batch, rep_b)


def test_make_nn_activation_and_init_options():
    """make_mlp's action_fn / init_weight / init_bias (mlp.py:10-35) and the SALE nets' `activ` (sale.py:25,67,97)
    reach the engine as rle_config act_* names (nets_from_make_nn, no engine needed): ReLU, ELU (alpha 1) and
    Identity, as strings or modules; the init functions are nn.init's, applied in make_mlp's order.  Refused:
    action_fn=None (make_mlp then pops the output Linear, mlp.py:34), other activations, critics that disagree."""
    import torch
    from torch.nn import functional as F

    from rl.nn import MLPActor, MLPCritic, SALEActor, SALECritic, SALEEncoder
    from rl.nn.modules import nets_from_make_nn

    torch.manual_seed(0)
    m = MLPActor(5, 2, [8, 8], action_fn="ELU", init_weight="orthogonal_", init_bias="normal_")
    torch.manual_seed(0)  # make_mlp's own order: Linear(), init_weight(w), init_bias(b), layer by layer
    ref = []
    for fin, fout in ((5, 8), (8, 8), (8, 2)):
        lin = torch.nn.Linear(fin, fout)
        torch.nn.init.orthogonal_(lin.weight.data)
        torch.nn.init.normal_(lin.bias.data)
        ref.append(lin)
    for i, lin in enumerate(ref):
        np.testing.assert_array_equal(m.mlp[2 * i].weight.detach().numpy(), lin.weight.detach().numpy())
        np.testing.assert_array_equal(m.mlp[2 * i].bias.detach().numpy(), lin.bias.detach().numpy())
    assert m.act == "elu" and isinstance(m.mlp[1], torch.nn.ELU)
    assert MLPCritic(5, 2, 8, action_fn=torch.nn.Identity()).act == "identity"
    assert MLPCritic(5, 2, 8).act == "relu"
    with pytest.raises(NotImplementedError, match="output layer"):
        MLPActor(5, 2, 8, action_fn=None)
    with pytest.raises(NotImplementedError, match="ReLU, ELU"):
        MLPActor(5, 2, 8, action_fn="Tanh")
    with pytest.raises(NotImplementedError, match="ReLU, ELU"):
        MLPActor(5, 2, 8, action_fn=torch.nn.ELU(alpha=0.5))

    def mk3(state_dim, action_dim, **kw):
        return (MLPActor(state_dim, action_dim, 16, action_fn="ELU"), MLPCritic(state_dim, action_dim, 16),
                MLPCritic(state_dim, action_dim, 16))

    assert nets_from_make_nn("td3", mk3, 3, 2, {})[3] == {"act_actor": "elu", "act_critic": "relu"}

    def mk7(state_dim, action_dim, **kw):
        return (SALEActor(state_dim, action_dim, 16, 16, activ=F.elu), SALECritic(state_dim, action_dim, 16, 16, activ=F.relu),
                SALECritic(state_dim, action_dim, 16, 16, activ=torch.relu), SALEEncoder(state_dim, action_dim, 16, 16))

    assert nets_from_make_nn("td7", mk7, 3, 2, {})[3] == {"act_actor": "elu", "act_critic": "relu", "act_encoder": "elu"}

    def mixed(state_dim, action_dim, **kw):
        return (MLPActor(state_dim, action_dim, 16), MLPCritic(state_dim, action_dim, 16, action_fn="ELU"),
                MLPCritic(state_dim, action_dim, 16))

    with pytest.raises(NotImplementedError, match="both critics"):
        nets_from_make_nn("td3", mixed, 3, 2, {})

    def tanh7(state_dim, action_dim, **kw):
        return (SALEActor(state_dim, action_dim, 16, 16, activ=torch.tanh), SALECritic(state_dim, action_dim, 16, 16),
                SALECritic(state_dim, action_dim, 16, 16), SALEEncoder(state_dim, action_dim, 16, 16))

    with pytest.raises(NotImplementedError, match="ReLU, ELU"):
        nets_from_make_nn("td7", tanh7, 3, 2, {})


def test_engine_agents_reject_non_default_net_types():
    """make_nn hooks must return the reference's default net types (rl.nn.*), one net shape across the
    agent's nets and make_mlp depths of 2..6 (rle.h RLE_MAX_HIDDEN), checked before any engine exists;
    anything else is a clear NotImplementedError."""
    with pytest.raises(TypeError):
        TD3("HalfCheetah-v4", make_nn=lambda **k: None)
    import torch

    from rl.nn import MLPActor, MLPCritic

    with pytest.raises(NotImplementedError):
        TD3("HalfCheetah-v4", make_nn=lambda state_dim, action_dim, **k: (torch.nn.Linear(1, 1),) * 3)
    with pytest.raises(NotImplementedError, match="one net shape"):
        TD3("HalfCheetah-v4", make_nn=lambda state_dim, action_dim, **k: (
            MLPActor(state_dim, action_dim, [64, 64, 64]), MLPCritic(state_dim, action_dim, 64),
            MLPCritic(state_dim, action_dim, 64)))
    with pytest.raises(NotImplementedError, match="2 to 6 hidden layers"):
        MLPActor(17, 6, [64] * 7)
    with pytest.raises(TypeError, match="hidden_sizes"):
        TD3("HalfCheetah-v4", zs_dim=64)


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    monkeypatch.setattr(E, "LIB_PATH", str(tmp_path / "librle.so"))
    monkeypatch.setattr(E, "_lib", None)
    with pytest.raises(RuntimeError, match="not built"):
        E.Replay(16, 3, 1, False)


def test_bench_timer_label_follows_the_dispatch_path():
    """The line's engine_timer names the clock of the engine's rle_plan.dispatch (no environment variable
    chooses the dispatch path: it is a plan field, rle.h)."""
    sys.path.insert(0, REPO)
    import bench

    kw = dict(wall=0.5, gpu_s=0.45, lv_policy=30, lv_plain=20)
    assert bench.summarize(1, 1000, 10, **kw)["engine_timer"].startswith("host wall, first AQL doorbell")
    assert bench.summarize(1, 1000, 10, dispatch=0, **kw)["engine_timer"] == "HIP events on the engine stream"


def test_bench_workload_figures_match_survey():
    sys.path.insert(0, REPO)
    import bench

    # 6,217,088 MAC/sample, 3.183 GFLOP/step, 41.37 MB/step for TD7 Humanoid B=256
    assert bench.SURVEY_MACS_PER_SAMPLE == 6_217_088
    # own derivation (bench.td7_macs_per_sample) agrees within 2%; the bench uses the §8(d) figure
    assert abs(bench.td7_macs_per_sample(376, 17, 256) / bench.SURVEY_MACS_PER_SAMPLE - 1) < 0.02
    assert abs(2 * bench.SURVEY_MACS_PER_SAMPLE * 256 / 1e9 - 3.183) < 1e-3
    assert abs(bench.td7_bytes_per_step(376, 17, 256, 256, 1_000_000) / 1e6 - 41.4) < 0.1
    out = bench.summarize(2, 1000, 10, wall=0.5, gpu_s=0.45, lv_policy=30, lv_plain=20)
    assert out["value"] == 4000.0 and out["n_gpus"] == 2 and out["scaling"] == "weak"
    assert out["roofline"]["launches_per_step"] == 25.0
    assert abs(out["roofline"]["avg_launch_us"] - 0.45 / (1000 * 25) * 1e6) < 1e-3
    json.dumps(out)


def test_bench_max_over_ranks_gloo_world2(tmp_path):
    """The N>1 bench path: two gloo ranks, the job time is the slowest rank's."""
    script = tmp_path / "w.py"
    script.write_text(
        "import os, sys, json\n"
        f"sys.path.insert(0, {REPO!r})\n"
        "import torch.distributed as dist\n"
        "import bench\n"
        "dist.init_process_group('gloo')\n"
        "r = dist.get_rank()\n"
        "wall, gpu = bench.max_over_ranks([1.0 + r, 0.5 * (2 - r)], dist)\n"
        "out = bench.summarize(dist.get_world_size(), 100, 5, wall, gpu, 30, 20)\n"
        "if r == 0: print(json.dumps([wall, gpu, out['value']]))\n"
        "dist.barrier(); dist.destroy_process_group()\n")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    res = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                          "--master-addr", "127.0.0.1", "--master-port", "29517", str(script)],
                         capture_output=True, text=True, timeout=240, env=env)
    assert res.returncode == 0, res.stderr[-2000:]
    wall, gpu, value = json.loads(res.stdout.strip().splitlines()[-1])
    assert (wall, gpu) == (2.0, 1.0)
    assert value == 2 * 100 / 2.0


def test_bench_gpus_n_launches_its_own_ranks():
    """``bench.py --gpus 2`` with no launcher (how the driver runs ``--gpus 1``): the script
    starts two rank processes itself (gloo rendezvous on 127.0.0.1) and rank 0 prints one
    JSON line with n_gpus 2.  The engine is a CPU stub (tests/bench_stub.py)."""
    env = dict(os.environ, RLE_BENCH_STUB=os.path.join(REPO, "tests", "bench_stub.py"))
    env.pop("WORLD_SIZE", None)
    res = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "40",
                          "--warmup", "2", "--cpu-seconds", "0.5", "--cpu-replay", "8192"], capture_output=True,
                         text=True, timeout=240, env=env)
    assert res.returncode == 0, res.stderr[-2000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 40 and out["scaling"] == "weak"
    assert out["value"] > 0
    # BASELINE.md's N-process CPU figure: both ranks ran the oracle concurrently, each on its own CPU slice
    cb = out["cpu_baseline"]
    assert cb["procs"] == 2 and len(cb["per_proc"]) == 2 and all(v > 0 for v in cb["per_proc"])
    assert cb["kind"] == "port" and abs(cb["value"] - sum(cb["per_proc"])) < 1e-2
    assert cb["cores"] == sum(cb["threads_per_proc"]) >= 2
    # each rank pinned (here: no KFD topology, so an even split of the allowed CPUs)
    pins = out["config"]["rank_pinning"]
    assert len(pins) == 2 and all(p["cpus"] >= 1 for p in pins)


def test_rank_pinning_follows_gpu_numa_locality(tmp_path, monkeypatch):
    """bench.gpu_local_cpus: a rank is pinned to the CPUs NUMA-local to its GPU (the PCI device's
    local_cpulist, found from the KFD node's domain / location_id), split among the ranks whose GPUs share
    them, without a HIP call; the allowed CPUs split by rank when the locality cannot be read."""
    import bench

    kfd, pci = tmp_path / "kfd", tmp_path / "pci"
    # node 0: CPU; nodes 1-4: GPUs at buses 0x11, 0x21 (NUMA 0: CPUs 0-7) and 0x81, 0x91 (NUMA 1: CPUs 8-15)
    for node, bus in ((0, None), (1, 0x11), (2, 0x21), (3, 0x81), (4, 0x91)):
        d = kfd / str(node)
        d.mkdir(parents=True)
        props = "simd_count 0\n" if bus is None else f"simd_count 1024\nlocation_id {bus << 8}\ndomain 0\n"
        d.joinpath("properties").write_text(props)
        if bus is not None:
            p = pci / f"0000:{bus:02x}:00.0"
            p.mkdir(parents=True)
            p.joinpath("local_cpulist").write_text("0-7\n" if bus < 0x80 else "8-15\n")
            p.joinpath("numa_node").write_text("0\n" if bus < 0x80 else "1\n")
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    allowed = list(range(16))
    got = [bench.gpu_local_cpus(r, 4, str(kfd), str(pci), allowed) for r in range(4)]
    assert [c for c, _ in got] == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9, 10, 11], [12, 13, 14, 15]]
    assert [i["numa_node"] for _, i in got] == [0, 0, 1, 1] and all(i["numa_local"] for _, i in got)
    assert got[2][1]["gpu_bdf"] == "0000:81:00.0"
    # two ranks on GPUs of different NUMA nodes each get their node's CPUs
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1,2")
    got = [bench.gpu_local_cpus(r, 2, str(kfd), str(pci), allowed)[0] for r in range(2)]
    assert got == [list(range(0, 8)), list(range(8, 16))]
    # a box whose allowed CPUs are all off the GPU's node, or no topology: an even split of the allowed CPUs
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    cpus, info = bench.gpu_local_cpus(1, 2, str(kfd), str(pci), [20, 21, 22, 23])
    assert cpus == [22, 23] and not info["numa_local"]
    cpus, info = bench.gpu_local_cpus(0, 2, str(tmp_path / "none"), str(pci), allowed)
    assert cpus == list(range(8)) and info["gpu_bdf"] is None
    assert bench.parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]


def test_bench_seeds_per_gpu_line():
    """``bench.py --seeds-per-gpu 2`` (stub engine): one JSON line whose value counts both seeds."""
    env = dict(os.environ, RLE_BENCH_STUB=os.path.join(REPO, "tests", "bench_stub.py"))
    env.pop("WORLD_SIZE", None)
    res = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--seeds-per-gpu", "2",
                          "--steps", "40", "--warmup", "2", "--no-cpu-baseline"], capture_output=True, text=True,
                         timeout=240, env=env)
    assert res.returncode == 0, res.stderr[-2000:]
    out = json.loads([ln for ln in res.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["config"]["seeds_per_gpu"] == 2 and "one HIP stream each" in out["config"]["parallelism"]
    assert out["value"] > 0


def test_bench_gpus_more_than_visible_fails():
    env = dict(os.environ, RLE_BENCH_STUB=os.path.join(REPO, "tests", "bench_stub.py"))
    env.pop("WORLD_SIZE", None)
    res = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "9", "--steps", "4",
                          "--warmup", "1", "--no-cpu-baseline"], capture_output=True, text=True, timeout=120,
                         env=env)
    assert res.returncode != 0 and "only 8 GPU(s) visible" in res.stderr


def test_sac_lap_fails_like_the_reference():
    # sac.py:202 calls an undefined _lap_huber: train_ops raises before any engine call
    sac = SAC.__new__(SAC)
    sac.use_lap = True
    with pytest.raises(AttributeError, match="_lap_huber"):
        sac.train_ops(DeviceBatch({}, np.zeros(4, np.int64), None), None)


def test_kfd_gpu_count_reads_topology_without_hip(tmp_path, monkeypatch):
    """bench.launch_ranks counts GPUs from the KFD topology (nodes with SIMDs; the CPU node has
    none), narrowed by the *_VISIBLE_DEVICES variables -- no HIP call in the parent."""
    import bench

    for i, simd in enumerate((0, 1024, 1024, 1024)):
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count {64 if simd == 0 else 0}\nsimd_count {simd}\n")
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert bench.kfd_gpu_count(str(tmp_path)) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1,2")
    assert bench.kfd_gpu_count(str(tmp_path)) == 2


def test_bench_line_reports_the_per_xcd_traffic_model():
    """The headline line's roofline carries how much of the measured per-level traffic the per-XCD model explains
    (>= 90%), read from the committed per-level PMC table."""
    sys.path.insert(0, REPO)
    import bench

    ev = bench.traffic_model_evidence()["traffic_model_xcd"]
    assert ev["explained_frac"] >= 0.9 and ev["source"].startswith("profiles/r")
    out = bench.summarize(1, 1000, 10, wall=0.5, gpu_s=0.45, lv_policy=30, lv_plain=20)
    assert out["roofline"]["traffic_model_xcd"] == ev
