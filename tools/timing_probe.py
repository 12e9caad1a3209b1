"""Where the fixed cost of a short timed region goes (bench.py's 20-step
driver run): wall time of K back-to-back parse launches between syncs, vs
K x the steady per-launch device time, for several ways of ending the region."""
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from capsule_amd import packets  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = packets.Context(0)
    w = bench.make_workload("parse64", 0xC0FFEE + 2)
    n = len(w["off"])
    b0 = packets.PacketBatch.from_numpy(w["arena"], w["off"], w["len"], dev)
    copies = 8
    batches = [b0] + [packets.PacketBatch(b0.arena.clone(), b0.off.clone(), b0.len.clone())
                      for _ in range(copies - 1)]
    outs = [packets.ParseBuffers(n, dev, csum=False) for _ in range(2)]
    stream = torch.cuda.current_stream(dev)
    L = [packets.ParseLauncher(ctx, batches[k % copies], outs[k & 1], w["flags"], stream)
         for k in range(2 * copies)]
    k = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.2:
        for _ in range(64):
            L[k % 16]()
            k += 1
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(2000):
        L[k % 16]()
        k += 1
    e1.record(stream)
    torch.cuda.synchronize()
    tk = e0.elapsed_time(e1) / 2000 * 1e3
    print(f"steady kernel+gap us {tk:.3f}")
    ends = {
        "device_sync": lambda: torch.cuda.synchronize(),
        "stream_sync": lambda: stream.synchronize(),
    }
    for K in (1, 20, 100):
        for name, end in ends.items():
            walls = []
            for rep in range(60):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(K):
                    L[k % 16]()
                    k += 1
                end()
                walls.append((time.perf_counter() - t0) * 1e6)
            med = statistics.median(walls[10:])
            print(f"K={K:4d} {name:12s} wall us {med:9.2f}  per step {med / K:8.3f}  "
                  f"overhead {med - K * tk:8.2f}")
    # launch cost on the host alone (queue already busy)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(1000):
        L[k % 16]()
        k += 1
    host = (time.perf_counter() - t0) / 1000 * 1e6
    torch.cuda.synchronize()
    print(f"host cost per launch us {host:.2f}")
    ctx.close()


if __name__ == "__main__":
    main()
