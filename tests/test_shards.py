"""world_size-2 gloo run of the shard harness on CPU: each rank owns a
distinct shard (its own seed), the timing is the max over ranks and the
aggregate unit count is the sum over ranks, with no data collective."""
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent("""
    import sys, time, json
    sys.path.insert(0, %r); sys.path.insert(0, %r)
    import numpy as np
    from capsule_amd.shards import ShardGroup
    from capsule_amd import synth
    import oracle_lib
    g = ShardGroup(backend="gloo")
    seed = g.shard_seed(0xC0FFEE)
    a, o, l = synth.imix(2000, seed=seed)
    meta, csum, h, _ = oracle_lib.parse_batch(a, o, l, 0x7f, fields=False)
    def step():
        time.sleep(0.01 * (g.rank + 1))
    t = g.timed(step, 3)
    total = g.sum(len(o))
    # one file per rank: two ranks printing to a shared stdout can interleave
    with open(sys.argv[1] + "/rank%%d.json" %% g.rank, "w") as f:
        json.dump({"rank": g.rank, "seed": seed, "t": t, "total": total,
                   "h0": int(h[0]), "ok": bool((meta & 0xff == 0).all())}, f)
    g.close()
""") % (ROOT, os.path.join(ROOT, "tests"))


def _free_port():
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def test_two_rank_gloo_shards(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER)
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(
        [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
         "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(script),
         str(tmp_path)],
        capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    rows = [json.loads((tmp_path / f"rank{i}.json").read_text()) for i in range(2)]
    assert len(rows) == 2
    a, b = sorted(rows, key=lambda x: x["rank"])
    assert a["seed"] != b["seed"] and a["h0"] != b["h0"]   # independent shards
    assert a["ok"] and b["ok"]
    assert a["total"] == b["total"] == 4000                 # aggregate = sum of shards
    assert abs(a["t"] - b["t"]) < 1e-9 and a["t"] >= 0.06   # max over ranks (rank 1 slower)


def _bench_line(out):
    import json

    lines = [x for x in out.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out[-2000:]  # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


def _stub_env():
    return dict(os.environ, OMP_NUM_THREADS="1")


def test_bench_launcher_spawns_n_ranks():
    """`bench.py --gpus 2` without torch.distributed.run starts two rank
    processes itself (GPU-free worker stub here) and reports both."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--stub", "--steps", "3",
                        "--warmup", "1"], capture_output=True, text=True, timeout=300,
                       env=_stub_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _bench_line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * d["config"]["packets_per_step"]
    assert [x["rank"] for x in d["roofline"]["per_rank"]] == [0, 1]
    sh = d["shards"]
    assert [x["rank"] for x in sh["per_rank"]] == [0, 1] and sh["config"] == "imix"
    # rank 1's stub launches are twice as slow: max over ranks sets the time
    assert sh["per_rank"][1]["kernel_us"] == 2 * sh["per_rank"][0]["kernel_us"]
    assert "sizes" not in d and "cpu_baseline" not in d  # N=1-only objects
    assert d["scaling"] == "weak" and "no collective" in d["config"]["parallelism"]


def test_bench_under_torchrun_stub():
    """The driver's own launch (torch.distributed.run, WORLD_SIZE set): no
    second launcher, the ranks join one gloo group."""
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr=127.0.0.1",
                        f"--master-port={port}", "bench.py", "--gpus", "2", "--stub",
                        "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=_stub_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _bench_line(r.stdout)
    assert d["n_gpus"] == 2 and len(d["shards"]["per_rank"]) == 2


def test_bench_single_gpu_line_shape():
    """N=1: the metric line plus `shards` (config 5 at N=1) and `sizes`
    (the metric's other sizes and configs 3/3'/4)."""
    r = subprocess.run([sys.executable, "bench.py", "--stub", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=_stub_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _bench_line(r.stdout)
    assert d["n_gpus"] == 1 and d["steps"] == 2
    for k in ("metric", "value", "unit", "ms_per_step", "higher_is_better", "scaling", "dtype",
              "config", "roofline"):
        assert k in d
    assert set(d["sizes"]) == {"parse256", "parse1500", "imix", "imix_csum", "nat64",
                               "nat64_4to6", "nat64_cold", "reconcile64", "reconcile_imix"}
    for obj in (d["shards"], d["sizes"]["imix"], d["sizes"]["imix_csum"]):
        assert obj["line_floor_bytes"] > 0 and 0 < obj["frac_of_line_floor"]
    assert d["roofline"]["per_rank"][0]["device"]["pci"] == "0000:01:00"
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(d["roofline"])
    assert "unpinned" in d["parity"]["flow_hash"]


def test_shard_group_refuses_device_backend():
    from capsule_amd.shards import ShardGroup
    import pytest

    with pytest.raises(ValueError):
        ShardGroup(backend="nccl")


def test_bench_eight_ranks_stub():
    """The driver's 8-GPU line shape: 8 rank processes, one row per rank with
    its own device (distinct PCI addresses), n_gpus 8."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--stub", "--steps", "2",
                        "--warmup", "1"], capture_output=True, text=True, timeout=600,
                       env=_stub_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _bench_line(r.stdout)
    assert d["n_gpus"] == 8 and d["config"]["global_batch"] == 8 * d["config"]["packets_per_step"]
    rows = d["roofline"]["per_rank"]
    assert [x["rank"] for x in rows] == list(range(8))
    assert len({x["device"]["pci"] for x in rows}) == 8
    assert len(d["shards"]["per_rank"]) == 8
    # every rank reports its NUMA binding (no GPU here: not bound, and why)
    for x in rows:
        numa = x["device"]["numa"]
        assert set(numa) == {"node", "cpus", "bound", "reason"}
        assert numa["bound"] is False and numa["reason"]


def test_numa_bind_on_a_sysfs_tree(tmp_path):
    """numa_bind reads the GPU's numa_node and the node's cpulist and pins
    the calling thread to the node's allowed CPUs (restored afterwards)."""
    from capsule_amd.shards import _cpulist, numa_bind

    assert _cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    allowed = sorted(os.sched_getaffinity(0))
    dev = tmp_path / "bus" / "pci" / "devices" / "0000:c1:00.0"
    dev.mkdir(parents=True)
    (dev / "numa_node").write_text("1\n")
    node = tmp_path / "devices" / "system" / "node" / "node1"
    node.mkdir(parents=True)
    pick = allowed[: max(1, len(allowed) // 2)]
    (node / "cpulist").write_text(",".join(map(str, pick)) + ",100000\n")
    try:
        info = numa_bind("0000:c1:00", sysfs=str(tmp_path))
        assert info == {"node": 1, "cpus": len(pick), "bound": True, "reason": None}
        assert sorted(os.sched_getaffinity(0)) == pick
    finally:
        os.sched_setaffinity(0, allowed)
    (dev / "numa_node").write_text("-1\n")
    info = numa_bind("0000:c1:00", sysfs=str(tmp_path))
    assert not info["bound"] and info["node"] == -1
    assert not numa_bind("0000:c2:00", sysfs=str(tmp_path))["bound"]


def test_bench_refuses_shared_device_stub():
    """Ranks that report the same PCI address fail the run unless the
    one-device rehearsal is asked for."""
    env = dict(_stub_env(), CGPU_BENCH_STUB_SAME_DEVICE="1")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--stub", "--steps", "2",
                        "--warmup", "1"], capture_output=True, text=True, timeout=300,
                       env=env, cwd=ROOT)
    assert r.returncode != 0 and "share a GPU" in r.stderr
    env["CGPU_BENCH_ONE_DEVICE"] = "1"
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--stub", "--steps", "2",
                        "--warmup", "1"], capture_output=True, text=True, timeout=300,
                       env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
