"""Config 2 served as 1..4 RX queues of one GPU (one HIP stream each, launch
k on queue k mod q), timed like bench.py's rx_queues object.

    python tools/queues_probe.py [--steps K]
"""
import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    args = ap.parse_args()
    import torch

    from capsule_amd import packets
    from capsule_amd.shards import ShardGroup

    g = ShardGroup()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ctx = packets.Context(0)
    w = bench.make_workload("parse64", g.shard_seed(0xC0FFEE + bench.SEEDS["parse64"]))
    for q in (1, 2, 3, 4):
        r = bench.bench_config("parse64", g, ctx, dev, args.steps, args.warmup, w=w, queues=q)
        print(json.dumps({"queues": q, "mpps": round(r["n"] * r["steps"] / r["elapsed"] / 1e6, 1),
                          "us_per_launch_wall": round(r["elapsed"] / r["steps"] * 1e6, 3),
                          "frac_of_8TBs": round(r["algo_bytes"] / (r["elapsed"] / r["steps"]) / 8e12, 4)}),
              flush=True)
    ctx.close()
    g.close()


if __name__ == "__main__":
    main()
