"""Parity at the exact benchmark workloads: every config bench.py times is
compared with the C oracle on every packet of the full 1 M batch, with the
bench's own generator, seed and flags (bench.make_workload), in the mode the
bench runs it (checksum verify: csum = NULL).  Plus the reference's own
IPv6 inputs (examples/pktdump/tcp6.pcap) through nat64 in both directions.
"""
import json
import pathlib

import numpy as np
import pytest
import torch

import nat64_replies
import oracle_lib
from capsule_amd import _native as N
from capsule_amd import synth

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
GOLD = pathlib.Path(__file__).resolve().parent / "golden"


def _workload(cfg, rank=0):
    import bench

    return bench.make_workload(cfg, 0xC0FFEE + bench.SEEDS[cfg] + 7919 * rank)


@pytest.mark.parametrize("cfg,rank", [("parse64", 0), ("parse256", 0), ("parse1500", 0),
                                      ("imix", 0), ("imix", 7), ("imix_csum", 0)])
def test_bench_parse_config_every_packet(ctx, cfg, rank):
    """The bench's batch (rank r's shard for config 5), its flags, verify
    mode: meta (status, offsets, CSUM_OK bits) and flow hash of all 1 M
    packets equal the oracle's; then the same batch with the checksum values
    stored, compared too."""
    from capsule_amd import packets

    w = _workload(cfg, rank)
    n = len(w["off"])
    assert n == 1 << 20
    b = packets.PacketBatch.from_numpy(w["arena"], w["off"], w["len"], DEV)
    r = packets.parse(ctx, b, flags=w["flags"], out=packets.ParseBuffers(n, DEV, csum=False))
    torch.cuda.synchronize()
    om, oc, oh, _ = oracle_lib.parse_batch(w["arena"], w["off"], w["len"], w["flags"],
                                           fields=False)
    gm = r.meta.cpu().numpy().view(np.uint32)
    bad = np.nonzero(gm != om)[0]
    assert not len(bad), f"meta differs at {bad[:8]}"
    gh = r.flow_hash.cpu().numpy().view(np.uint64)
    bad = np.nonzero(gh != oh)[0]
    assert not len(bad), f"flow hash differs at {bad[:8]}"
    assert (om & 0xFF == 0).all()  # reconciled frames: everything parses
    if w["flags"] & N.F_CSUM_L4:
        assert (om & N.META_L4_CSUM_OK).all()
        r2 = packets.parse(ctx, b, flags=w["flags"])
        torch.cuda.synchronize()
        gc = r2.csum.cpu().numpy().view(np.uint32)
        bad = np.nonzero(gc != oc)[0]
        assert not len(bad), f"checksum values differ at {bad[:8]}"
        assert torch.equal(r2.meta, r.meta)


def _compare_nat(g, o, what):
    (g_out, g_len, g_disp, g_st), (o_out, o_len, o_disp, o_st) = g, o
    for name, x, y in (("disposition", g_disp, o_disp), ("status", g_st, o_st),
                       ("length", g_len, o_len)):
        bad = np.nonzero(x != y)[0]
        assert not len(bad), f"{what}: {name} differs at {bad[:8]}"
    bad = np.nonzero(g_out != o_out)[0]
    assert not len(bad), f"{what}: output arena differs at bytes {bad[:8]}"


def _gpu_nat(gw, direction, arena, off, ln, out_off, size):
    from capsule_amd import packets

    b = packets.PacketBatch.from_numpy(arena, off, ln, DEV)
    out = torch.zeros(size, dtype=torch.uint8, device=DEV)
    oo = torch.from_numpy(np.ascontiguousarray(out_off, np.uint32).view(np.int32)).to(DEV)
    fn = gw.nat_6to4 if direction == "6to4" else gw.nat_4to6
    ob, disp, st = fn(b, out_arena=out, out_off=oo)
    torch.cuda.synchronize()
    return (out.cpu().numpy(), ob.len.cpu().numpy().view(np.uint16), disp.cpu().numpy(),
            st.cpu().numpy())


def test_bench_nat64_config_every_byte(ctx):
    """BASELINE config 4 exactly as benched: the 1 M x 256-B stream through
    a map of the bench's capacity (bench.PORTMAP_LOG2), first pass (every
    key new: the nat64_cold config) and the steady-state pass the timed loop
    repeats (every key known); all output
    bytes, lengths, dispositions and the port map state equal the oracle's.
    Then a cold pass again after cgpu_portmap_reset (how nat64_cold times
    it), and the replies through 4to6 (the nat64_4to6 bench config)."""
    import bench
    from capsule_amd import packets

    w = _workload("nat64")
    a, o, l = w["arena"], w["off"], w["len"]
    gw = packets.Nat64Gateway(ctx, capacity_log2=bench.PORTMAP_LOG2)
    pm = oracle_lib.PortMap()
    oo, size = w["out_off"], w["out_size"]  # the bench's packed egress layout
    for p in range(2):
        g = _gpu_nat(gw, "6to4", a, o, l, oo, size)
        ref = pm.nat_6to4(a, o, l, oo, size)
        _compare_nat(g, ref, f"6to4 pass {p}")
        assert (ref[2] == N.ACT).all()
        assert gw.next_port() == pm.next_port() and gw.size() == pm.size()
    gw.reset()
    _compare_nat(_gpu_nat(gw, "6to4", a, o, l, oo, size), oracle_lib.PortMap().nat_6to4(a, o, l, oo, size),
                 "6to4 after reset")
    assert gw.next_port() == pm.next_port() and gw.size() == pm.size()
    ra, ro, rl = synth.nat64_replies(ref[0], oo, ref[1])
    o6 = (np.arange(len(ro), dtype=np.int64) * 256).astype(np.uint32)  # +20 B per frame
    g = _gpu_nat(gw, "4to6", ra, ro, rl, o6, 256 * len(ro) + 64)
    _compare_nat(g, pm.nat_4to6(ra, ro, rl, o6, 256 * len(ro) + 64), "4to6")
    assert (g[2] == N.ACT).all()
    gw.close()


def test_reference_tcp6_pcap_through_nat64(ctx):
    """examples/pktdump/tcp6.pcap: 10 IPv6/TCP frames (the reference's own
    6to4 inputs) through nat_6to4, then their replies through nat_4to6, GPU
    vs oracle on every byte, at several output alignments."""
    from capsule_amd import packets

    pk = json.loads((GOLD / "reference_packets.json").read_text())
    frames = [bytes.fromhex(h) for h in pk["pktdump_tcp6"]["packets"]]
    assert len(frames) == 10
    arena, off, ln = synth.pack_frames(frames)
    for shift in (0, 1, 3):
        gw = packets.Nat64Gateway(ctx, capacity_log2=8)
        pm = oracle_lib.PortMap()
        out_off = off + np.uint32(shift)
        size = len(arena) + 64
        g = _gpu_nat(gw, "6to4", arena, off, ln, out_off, size)
        ref = pm.nat_6to4(arena, off, ln, out_off, size)
        _compare_nat(g, ref, "tcp6.pcap 6to4")
        assert (ref[2] == N.ACT).all() and (ref[1] == 54).all()
        assert gw.next_port() == pm.next_port() == 1026  # one (src, port) key
        rep = nat64_replies.replies(ref[0], out_off, ref[1], ref[2],
                                    np.random.default_rng(shift), junk=0.0)
        ra, ro, rl = synth.pack_frames(rep)
        r_off = (ro + np.uint32(shift)).astype(np.uint32)
        rsize = len(ra) + 64 * len(ro) + 64
        r_off = (r_off + np.arange(len(ro), dtype=np.uint32) * 32).astype(np.uint32)
        g = _gpu_nat(gw, "4to6", ra, ro, rl, r_off, rsize)
        ref6 = pm.nat_4to6(ra, ro, rl, r_off, rsize)
        _compare_nat(g, ref6, "tcp6.pcap replies 4to6")
        assert (ref6[2] == N.ACT).all()
        gw.close()
