"""How much of the IMIX-with-checksums launch is load imbalance between waves.

The parse kernel gives each wave 64 consecutive frames; on the stream path a
wave's time grows with its span (the bytes from its first frame to the end
of its last), which for shuffled IMIX ranges from about 11 to 37 KB.  A
1 Mi-packet launch is 16,384 waves, two per wave slot of the chip, so the
waves dispatched last decide when the launch ends.  This probe times the
same frames (same arena, same descriptors) with the 64-frame groups taken
in three orders: as generated, longest span first (the order that leaves
short waves for the end) and shortest first, and with only the groups after
the first G taken longest first.  The committed logs
(profiles/round5/imix_order_probe*.log) were taken before the kernel ordered
its last round itself (parse.hip, "Longest span first"); with that order in
place the probe measures the two orders stacked.  Diagnostic only:
python tools/imix_order_probe.py [steps]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    from capsule_amd import packets
    from capsule_amd.shards import ShardGroup

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    g = ShardGroup()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = packets.Context(0)
    w0 = bench.make_workload("imix_csum", g.shard_seed(0xC0FFEE + bench.SEEDS["imix_csum"]))
    off = w0["off"].astype(np.int64)
    ln = w0["len"].astype(np.int64)
    grp = off.reshape(-1, 64)
    span = (grp[:, -1] + ln.reshape(-1, 64)[:, -1]) - grp[:, 0]
    orders = {"generated": np.arange(len(span)),
              "longest_first": np.argsort(-span, kind="stable"),
              "shortest_first": np.argsort(span, kind="stable")}
    # the first G groups as generated (the waves resident from the start),
    # the rest longest first: what a schedule built during the first round
    # could do for the second
    for first in (4096, 6144, 8192, 10240):
        rest = np.arange(first, len(span))
        orders[f"gen{first}+longest"] = np.concatenate(
            [np.arange(first), rest[np.argsort(-span[rest], kind="stable")]])
    for name, order in orders.items():
        idx = (order[:, None] * 64 + np.arange(64)[None, :]).reshape(-1)
        w = dict(w0, off=w0["off"][idx].copy(), len=w0["len"][idx].copy())
        r = bench.bench_config("imix_csum", g, ctx, dev, steps, 500, w=w)
        print(f"{name:15s} kernel_us {r['kern_us']:.3f}", flush=True)
    ctx.close()
    g.close()


if __name__ == "__main__":
    main()
