"""Self-launcher (bench.py --gpus N without torchrun) and per-rank CPU placement."""
import os
import subprocess
import sys
import textwrap

import pytest

from thinvids_amd.parallel import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_plan_affinity_numa_split():
    nodes = {0: list(range(0, 16)), 1: list(range(16, 32))}
    gpu_nodes = [0, 0, 0, 0, 1, 1, 1, 1]
    sets = [launch.plan_affinity(r, 8, list(range(32)), nodes, gpu_nodes) for r in range(8)]
    assert sets[0] == [0, 1, 2, 3] and sets[3] == [12, 13, 14, 15]
    assert sets[4] == [16, 17, 18, 19] and sets[7] == [28, 29, 30, 31]
    flat = [c for s in sets for c in s]
    assert len(flat) == len(set(flat)) == 32  # disjoint and covering


def test_plan_affinity_fallback_even_split():
    sets = [launch.plan_affinity(r, 3, list(range(8)), {0: list(range(8))}, []) for r in range(3)]
    assert sets == [[0, 1], [2, 3], [4, 5, 6, 7]]
    assert launch.plan_affinity(0, 1, [5, 6], {0: [5, 6]}, []) == [5, 6]


def test_plan_affinity_respects_allowed_set():
    nodes = {0: list(range(8)), 1: list(range(8, 16))}
    s = launch.plan_affinity(1, 2, [8, 9, 10], nodes, [0, 1])
    assert s == [8, 9, 10]


_SCRIPT = textwrap.dedent("""
    import os, sys, json
    sys.path.insert(0, {root!r})
    import torch, torch.distributed as dist
    from thinvids_amd.parallel.comm import allreduce_stats, gather_bytes_to_root
    from thinvids_amd.parallel.launch import pin_rank
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    cpus = pin_rank(int(os.environ["LOCAL_RANK"]), int(os.environ["LOCAL_WORLD_SIZE"]))
    dist.init_process_group("gloo")
    assert dist.get_world_size() == world
    s = allreduce_stats([rank + 1.0, 2.0], torch.device("cpu"))
    g = gather_bytes_to_root(bytes([65 + rank]) * (rank + 1), torch.device("cpu"))
    if rank == 0:
        with open({out!r}, "w") as f:
            json.dump({{"sum": list(s), "g": [x.decode() for x in g], "cpus": len(cpus)}}, f)
    dist.destroy_process_group()
""")


@pytest.mark.parametrize("n", [1, 3])
def test_spawn_ranks_runs_a_live_group(tmp_path, n):
    out = tmp_path / "o.json"
    script = tmp_path / "s.py"
    script.write_text(_SCRIPT.format(root=ROOT, out=str(out)))
    assert launch.spawn_ranks(n, [str(script)], timeout=120) == 0
    import json

    d = json.loads(out.read_text())
    assert d["sum"] == [n * (n + 1) / 2, 2.0 * n]
    assert d["g"] == [chr(65 + r) * (r + 1) for r in range(n)]
    assert d["cpus"] >= 1


def test_spawn_ranks_propagates_failure_and_kills_peers(tmp_path):
    script = tmp_path / "f.py"
    script.write_text("import os, time\nif os.environ['RANK'] == '1': raise SystemExit(3)\ntime.sleep(60)\n")
    assert launch.spawn_ranks(2, [str(script)], timeout=50) == 3


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0


def test_visible_gpu_count_without_hip(monkeypatch):
    """The node supervisor counts GPUs from the visibility list / sysfs (no HIP call)."""
    from thinvids_amd.parallel import launch

    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,2,5")
    assert launch.visible_gpu_count() == 3
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    for v in ("ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setattr(launch, "gpu_numa_nodes", lambda: [0, 0, 1, 1])
    assert launch.visible_gpu_count() == 4


def test_tv_cpus_caps_the_rank_cpu_set(tmp_path):
    """TV_CPUS=N restricts a rank (and the CABAC pool it spawns later) to N CPUs."""
    script = tmp_path / "c.py"
    script.write_text(f"import os, sys\nsys.path.insert(0, {ROOT!r})\n"
                      "from thinvids_amd.parallel.launch import pin_rank\n"
                      "c = pin_rank(0, 1)\nprint(len(c), len(os.sched_getaffinity(0)))\n")
    env = dict(os.environ, TV_CPUS="2")
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=60)
    a, b = map(int, r.stdout.split())
    want = min(2, len(os.sched_getaffinity(0)))
    assert a == b == want, r.stdout + r.stderr


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("mode", [[], ["--kbps", "300"], ["--codec", "av1"], ["--ladder", "96"]],
                         ids=["1pass", "2pass", "av1", "ladder"])
def test_bench_cpu_rehearsal_n_ranks(n, mode):
    """bench.py's N-rank logic (self-launch, post-thread collective ordering, the 2-pass
    plan all-reduce and pass-1 look-ahead, the AV1 step pipeline, the ladder fan-out and the
    bitstream gather) end-to-end on N gloo ranks with the golden encoders (--cpu) — the
    paths the driver's multi-GPU run takes, exercised before it does (verdict r3 item 2)."""
    import json

    args = [sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", str(n), "--steps", "2", "--warmup", "1",
            "--batch", "2", "--gop", "4", "--threads", "1", *mode]
    r = subprocess.run(args, capture_output=True, text=True, timeout=240, env=dict(os.environ, TV_NO_PIN="1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout  # rank 0 prints exactly one JSON line
    d = json.loads(line[0])
    c = d["config"]
    assert d["n_gpus"] == n and d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0
    assert c["global_batch"] == 2 * n and "CPU REHEARSAL" in d["data"]
    assert len(c["per_rank_cpu"]) == n
    # every rank's bitstream bytes reached the stitch rank: the gathered total equals the
    # all-reduced sum of the per-rank byte counts
    assert c["gathered_mb_at_root"] == c["bytes_all_reduced_mb"] > 0
    frames_per_step = 2 * 4 * n
    assert abs(d["value"] * d["ms_per_step"] / 1000 - frames_per_step) < 1e-3 * frames_per_step
    if "--kbps" in mode:
        assert c["kbps_error_pct"] is not None and c["pass1_kbps_rank0"] > 0
