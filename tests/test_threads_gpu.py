"""Several RX queues on one GPU: one context per core thread, each on its own
stream (runtime/core_map.rs:236-293, one pipeline per core; the C ABI takes
no global lock on the launch path).  Two threads drive two contexts at once
-- parse, group_by and a stateful nat64 port map each -- and every result
equals the oracle's for that thread's own stream of batches."""
import threading

import numpy as np
import pytest
import torch

import oracle_lib
from capsule_amd import _native as N
from capsule_amd import synth

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
FLAGS = N.F_ACCEPT_ALL | N.F_CSUM_IP | N.F_CSUM_L4 | N.F_FLOW_HASH


def test_two_contexts_two_streams_two_threads():
    from capsule_amd import packets

    T, rounds = 2, 12
    ctxs = [packets.Context(0) for _ in range(T)]
    streams = [torch.cuda.Stream() for _ in range(T)]
    parse_in = [synth.imix(40_000, seed=100 + t, vlan_frac=0.1) for t in range(T)]
    nat_in = [synth.nat64_stream(30_000, n_keys=2000 + 500 * t, seed=200 + t, drop_frac=0.05)
              for t in range(T)]
    pb = [packets.PacketBatch.from_numpy(*parse_in[t], DEV) for t in range(T)]
    nb = [packets.PacketBatch.from_numpy(*nat_in[t], DEV) for t in range(T)]
    torch.cuda.synchronize()
    got = [None] * T
    errors = []

    def core(t):
        try:
            ctx, s = ctxs[t], streams[t]
            gw = packets.Nat64Gateway(ctx, capacity_log2=13)
            with torch.cuda.stream(s):
                outs = [packets.ParseBuffers(pb[t].n, DEV) for _ in range(2)]
                for k in range(rounds):
                    r = packets.parse(ctx, pb[t], FLAGS, out=outs[k & 1], stream=s)
                g = packets.group_by(ctx, r.meta, by="class", stream=s)
                nat = [gw.nat_6to4(nb[t], stream=s) for _ in range(3)]  # port map carried over
            s.synchronize()
            got[t] = dict(meta=r.meta.cpu().numpy().view(np.uint32),
                          csum=r.csum.cpu().numpy().view(np.uint32),
                          hash=r.flow_hash.cpu().numpy().view(np.uint64),
                          idx=g.idx.cpu().numpy().view(np.uint32),
                          off=g.off.cpu().numpy().view(np.uint32),
                          nat=[(ob.arena.cpu().numpy(), ob.len.cpu().numpy().view(np.uint16),
                                d.cpu().numpy()) for ob, d, _ in nat],
                          next_port=gw.next_port(), size=gw.size())
            gw.close()
        except Exception as e:  # surfaced in the main thread
            errors.append((t, repr(e)))

    threads = [threading.Thread(target=core, args=(t,)) for t in range(T)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not errors, errors
    for t in range(T):
        a, o, l = parse_in[t]
        om, oc, oh, _ = oracle_lib.parse_batch(a, o, l, FLAGS, fields=False)
        g = got[t]
        assert (g["meta"] == om).all() and (g["csum"] == oc).all() and (g["hash"] == oh).all()
        idx, off = oracle_lib.group_by(om, 5, N.KEY_META_CLASS)
        assert (g["idx"] == idx).all() and (g["off"] == off).all()
        pm = oracle_lib.PortMap()
        a, o, l = nat_in[t]
        for out, olen, disp in g["nat"]:
            o_out, o_len, o_disp, _ = pm.nat_6to4(a, o, l)
            assert (disp == o_disp).all() and (olen == o_len).all() and (out == o_out).all()
        assert g["next_port"] == pm.next_port() and g["size"] == pm.size()
    for c in ctxs:
        c.close()
