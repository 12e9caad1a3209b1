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
