"""nat64 6to4 steady-state time against the number of distinct keys (port
map lines the probes touch): how much of the call is the probe lines' L2
misses.  Same stream shape as the bench (1 Mi x 256 B, packed 236-B output
frames), the map at the library default (2^20 slots).  Diagnostic only:
python tools/nat64_keys_probe.py [keys ...]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
from capsule_amd import packets, synth  # noqa: E402


def main():
    keys = [int(k) for k in sys.argv[1:]] or [50_000, 25_000, 12_500, 6_250, 1_000]
    ctx = packets.Context(0)
    dev = torch.device("cuda:0")
    n = 1 << 20
    for nk in keys:
        a, o, l = synth.nat64_stream(n, n_keys=nk, seed=0xC0FFEE + 4)
        new_len = l.astype(np.int64) - 20
        out_off = np.zeros(n, np.int64)
        out_off[1:] = np.cumsum(new_len)[:-1]
        copies = 4
        bs = [packets.PacketBatch.from_numpy(a, o, l, dev) for _ in range(copies)]
        oo = torch.from_numpy(out_off.astype(np.uint32).view(np.int32)).to(dev)
        outs = [torch.empty(int(new_len.sum()) + 64, dtype=torch.uint8, device=dev) for _ in range(2)]
        gw = packets.Nat64Gateway(ctx)
        for k in range(40):  # first pass commits every key; then warm
            gw.nat_6to4(bs[k % copies], out_arena=outs[k & 1], out_off=oo)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        K = 400
        e0.record()
        for k in range(K):
            gw.nat_6to4(bs[k % copies], out_arena=outs[k & 1], out_off=oo)
        e1.record()
        torch.cuda.synchronize()
        print(f"keys {nk:6d}: {e0.elapsed_time(e1) / K * 1e3:.1f} us per call", flush=True)
        gw.close()
        del bs, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
