"""Batch combinators (capsule_amd.batch) -- the reference's batch tests,
core/src/batch/mod.rs:451-735, restated over bursts with its own fixture
packets (tests/golden/reference_packets.json).

The combinators that are tensor plumbing (filter, map, for_each, inspect,
emit, replace, send, splice, poll_fn) run here on the CPU; the ones that
call the device (parse, group_by) are `gpu` tests.
"""
import json
import pathlib

import numpy as np
import pytest
import torch

from capsule_amd import _native as N
from capsule_amd import batch as B

GOLD = pathlib.Path(__file__).resolve().parent / "golden"
PK = {k: bytes.fromhex(v["hex"]) for k, v in
      json.loads((GOLD / "reference_packets.json").read_text()).items() if "hex" in v}
UDP4, TCP4, ICMP4 = PK["IPV4_UDP_PACKET"], PK["IPV4_TCP_PACKET"], PK["ICMPV4_PACKET"]

REC = np.dtype(N.HDR_RECORD_FIELDS)
TTL, PROTO = REC.fields["ttl"][1], REC.fields["protocol"][1]
V4 = N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_ACCEPT_TCP | N.F_ACCEPT_ICMP


def new_batch(frames, ctx=None, device="cpu"):
    """`new_batch` of mod.rs:438-449: one burst through a channel, replenished."""
    ch = B.Channel()
    ch.transmit(list(frames))
    b = B.Poll(ctx, ch, device)
    b.replenish()
    return b


def disps(batch):
    out = batch.next_burst()
    return out.dispositions() if out is not None else None


def ttl_of(burst):
    """IPv4 TTL byte of each packet (untagged Ethernet)."""
    at = (burst.batch.off.long() & 0xFFFFFFFF) + 14 + 8
    return burst.batch.arena[at].tolist()


def set_ttl(v):
    def f(sub):
        sub.batch.arena[(sub.batch.off.long() & 0xFFFFFFFF) + 14 + 8] = v
    return f


def protocol(b):
    return b.parsed.fields[:, PROTO]


# ---- plumbing combinators (CPU) ------------------------------------------------
def test_emit_batch():
    tx = B.Channel()

    def broken(_):
        raise AssertionError("emit broken!")

    b = new_batch([UDP4]).emit(tx).for_each(broken)
    assert disps(b) == [B.EMIT]
    assert tx.receive().n == 1


def test_filter_batch():
    assert disps(new_batch([UDP4]).filter(lambda s: True)) == [B.ACT]
    assert disps(new_batch([UDP4]).filter(lambda s: False)) == [B.DROP]


def test_map_batch():
    assert disps(new_batch([UDP4]).map(lambda s: None)) == [B.ACT]
    # "can't shrink the mbuf that much": the closure's error aborts the packet
    b = new_batch([UDP4]).map(lambda s: torch.full((s.n,), N.PKT["NOT_RESIZED"]))
    out = b.next_burst()
    assert out.dispositions() == [B.ABORT]
    assert out.status.tolist() == [N.PKT["NOT_RESIZED"]]


def test_for_each_and_inspect_batch():
    seen = []
    b = new_batch([UDP4]).for_each(lambda s: seen.append(s.n))
    assert disps(b) == [B.ACT] and seen == [1]
    b = new_batch([UDP4]).inspect(lambda s: seen.append(s.n))
    assert disps(b) == [B.ACT] and seen == [1, 1]


def test_closures_see_only_act_packets():
    seen = []
    b = (new_batch([UDP4, TCP4, ICMP4])
         .filter(lambda s: torch.tensor([True, False, True]))
         .map(lambda s: seen.append(s.n) or torch.tensor([0, 7]))
         .inspect(lambda s: seen.append(s.n)))
    out = b.next_burst()
    assert out.dispositions() == [B.ACT, B.DROP, B.ABORT]
    assert out.status.tolist() == [0, 0, 7]
    assert seen == [2, 1]


def test_replace_batch():
    b = new_batch([UDP4]).replace(lambda s: [TCP4] * s.n)
    out = b.next_burst()
    # first the replacement, then the original
    assert out.dispositions() == [B.ACT, B.DROP]
    assert out.batch.n == 2
    first = out.batch.arena[int(out.batch.off[0]):][:len(TCP4)]
    assert bytes(first.numpy()) == TCP4
    assert disps(b) is None  # at the end


def test_replace_interleaves_and_aborts():
    b = new_batch([UDP4, TCP4, UDP4]).filter(lambda s: torch.tensor([True, False, True])).replace(
        lambda s: ([ICMP4] * s.n, torch.tensor([0, 9])))
    out = b.next_burst()
    assert out.dispositions() == [B.ACT, B.DROP, B.DROP, B.ABORT]
    assert out.origin.tolist() == [0, 0, 1, 2]
    assert out.status.tolist() == [0, 0, 0, 9]


def test_poll_fn_batch():
    b = B.Poll(None, lambda: [bytes(64)], "cpu")
    b.replenish()
    assert disps(b) == [B.ACT]
    assert disps(b) is None


def test_splice_pipeline():
    rx1, tx2 = B.Channel(), B.Channel()
    pipeline = B.Poll(None, rx1, "cpu").send(tx2)
    assert not pipeline.run_once()  # no packet yet
    assert tx2.q == []
    rx1.transmit([UDP4])
    assert pipeline.run_once()
    assert tx2.receive().n == 1


def test_send_counters():
    tx, emit_tx = B.Channel(), B.Channel()
    rx = B.Channel()
    for _ in range(3):
        rx.transmit([UDP4, TCP4, ICMP4, UDP4])
    pipe = (B.Poll(None, rx, "cpu")
            .filter(lambda s: torch.tensor([True, True, False, True]))
            .map(lambda s: torch.tensor([0, 5, 0]))
            .filter_map(lambda s: torch.tensor([B.ACT, B.ACT], dtype=torch.uint8))
            .send(tx))
    pipe.run()
    assert (pipe.transmitted, pipe.dropped, pipe.aborted, pipe.emitted) == (6, 3, 3, 0)
    assert pipe.processed == 6 and pipe.errors == 3
    assert [t.n for t in tx.q] == [2, 2, 2]
    # emit counts as processed, not transmitted
    rx.transmit([UDP4, TCP4])
    pipe2 = B.Poll(None, rx, "cpu").emit(emit_tx).send(tx)
    pipe2.run()
    assert (pipe2.transmitted, pipe2.emitted, pipe2.processed) == (0, 2, 2)


def test_concat_rebases_offsets():
    a = B.Burst(B.packets.PacketBatch.from_frames([UDP4, TCP4], "cpu"))
    c = B.Burst(B.packets.PacketBatch.from_frames([ICMP4], "cpu"))
    m = B.Burst.concat([a, c, a.take(torch.tensor([1]))])
    got = [bytes(m.batch.frame(i)) for i in range(m.n)]
    assert got == [UDP4, TCP4, ICMP4, TCP4]


# ---- device combinators ----------------------------------------------------------
@pytest.mark.gpu
def test_filter_map_batch(ctx):
    b = new_batch([UDP4, ICMP4], ctx, "cuda").parse(V4, fields=True, upto="l3").filter_map(
        lambda s: torch.where(protocol(s) == 17, B.ACT, B.DROP).to(torch.uint8))
    # udp is let through, icmp is dropped
    assert disps(b) == [B.ACT, B.DROP]
    assert disps(b) is None


@pytest.mark.gpu
def test_parse_depth_decides_what_aborts(ctx):
    arp = PK["ARP4_PACKET"]
    only_udp_tcp = N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_ACCEPT_TCP
    out = new_batch([UDP4, ICMP4, arp], ctx, "cuda").parse(only_udp_tcp, upto="l3").next_burst()
    assert out.dispositions() == [B.ACT, B.ACT, B.ABORT]
    assert out.status.tolist()[2] == N.PKT["NOT_IPV4"]
    out = new_batch([UDP4, ICMP4, arp], ctx, "cuda").parse(only_udp_tcp, upto="l4").next_burst()
    assert out.dispositions() == [B.ACT, B.ABORT, B.ABORT]
    assert out.status.tolist()[1] == N.PKT["NOT_L4"]
    out = new_batch([arp], ctx, "cuda").parse(only_udp_tcp, upto="l2").next_burst()
    assert out.dispositions() == [B.ACT]


def _v4_batch(ctx, frames):
    return new_batch(frames, ctx, "cuda").parse(V4, fields=True, upto="l3")


@pytest.mark.gpu
def test_group_by_batch(ctx):
    b = _v4_batch(ctx, [TCP4, UDP4, ICMP4]).group_by(
        protocol, {6: lambda g: g.inspect(set_ttl(1)), 17: lambda g: g.inspect(set_ttl(2))},
        catch_all=lambda g: g.filter(lambda s: False))
    out = b.next_burst()
    # tcp arm, udp arm, catch-all arm
    assert out.dispositions() == [B.ACT, B.ACT, B.DROP]
    assert ttl_of(out)[:2] == [1, 2]


@pytest.mark.gpu
def test_group_by_no_catchall(ctx):
    b = _v4_batch(ctx, [ICMP4]).group_by(protocol, {6: lambda g: g.filter(lambda s: False)})
    assert disps(b) == [B.ACT]  # did not match, passes through


@pytest.mark.gpu
def test_group_by_or(ctx):
    b = _v4_batch(ctx, [TCP4, UDP4, ICMP4]).group_by(
        protocol, {(6, 17): lambda g: g.inspect(set_ttl(1))},
        catch_all=lambda g: g.filter(lambda s: False))
    out = b.next_burst()
    assert out.dispositions() == [B.ACT, B.ACT, B.DROP]
    assert ttl_of(out)[:2] == [1, 1]


@pytest.mark.gpu
def test_group_by_or_no_catchall(ctx):
    b = _v4_batch(ctx, [TCP4, UDP4]).group_by(protocol, {(6, 17): lambda g: g.inspect(set_ttl(1))})
    out = b.next_burst()
    assert out.dispositions() == [B.ACT, B.ACT]
    assert ttl_of(out) == [1, 1]


@pytest.mark.gpu
def test_group_by_fanout(ctx):
    b = _v4_batch(ctx, [TCP4]).group_by(protocol, {6: lambda g: g.replace(lambda s: [UDP4] * s.n)})
    out = b.next_burst()
    # the replacement (a new UDP packet), then the original TCP packet dropped
    assert out.dispositions() == [B.ACT, B.DROP]
    assert out.batch.frame(0) == UDP4 and out.batch.frame(1) == TCP4
    assert disps(b) is None


@pytest.mark.gpu
def test_group_by_keeps_batch_order_at_scale(ctx):
    """A large mixed burst: every packet lands in its arm, the merged burst is
    in input order, and the arms' dispositions agree with a host model."""
    from capsule_amd import synth

    a, o, l = synth.imix(20000, seed=4, vlan_frac=0.0)
    pb = B.packets.PacketBatch.from_numpy(a, o, l, "cuda")
    src = B.Poll(ctx, iter([pb]), "cuda")
    src.replenish()
    seen = {}
    pipe = src.parse(N.F_ACCEPT_ALL | N.F_ACCEPT_ICMP, fields=True).group_by(
        protocol,
        {6: lambda g: g.inspect(lambda s: seen.__setitem__(6, s.n)),
         17: lambda g: g.filter(lambda s: (s.batch.len.long() & 0xFFFF) < 200)},
        catch_all=lambda g: g.filter(lambda s: False))
    out = pipe.next_burst()
    meta = out.parsed.meta.cpu().numpy()
    proto = out.parsed.fields[:, PROTO].cpu().numpy()
    ln = l.astype(np.int64)
    ok = (meta & 0xFF) == 0
    want = np.where(~ok, B.ABORT, np.where(proto == 6, B.ACT,
                    np.where(proto == 17, np.where(ln < 200, B.ACT, B.DROP), B.DROP)))
    assert (out.disp.cpu().numpy() == want).all()
    assert (out.origin.cpu().numpy() == np.arange(len(o))).all()
    assert (out.batch.off.cpu().numpy().view(np.uint32) == o).all()
    assert seen[6] == int((ok & (proto == 6)).sum())


# ---- burst aggregation at the GPU seam (Poll target) --------------------------
def _rx_bursts(frames, size=32):
    """An RX queue handing out bursts of at most `size` frames, then empty
    bursts (rte_eth_rx_burst with nothing left, dpdk/port.rs:149-171)."""
    chunks = [frames[i:i + size] for i in range(0, len(frames), size)]
    it = iter(chunks)
    return lambda: next(it, [])


def test_poll_target_gathers_rx_bursts_in_order():
    frames = [bytes([i & 0xFF, i >> 8]) + bytes(62) for i in range(200)]
    b = B.Poll(None, _rx_bursts(frames), "cpu", target=100)
    b.replenish()  # 4 pulls of 32 reach the target
    out = b.next_burst()
    assert out.n == 128 and b.pulls == 4
    assert [out.batch.frame(i) for i in range(out.n)] == frames[:128]
    b.replenish()  # 32 + 32 + 8, then an empty pull ends the gathering
    out = b.next_burst()
    assert out.n == 72 and b.pulls == 4 + 4
    assert [out.batch.frame(i) for i in range(out.n)] == frames[128:]
    b.replenish()  # nothing left: no burst, after one pull
    assert b.next_burst() is None and b.pulls == 9
    # target=1 is the reference's one pull per replenish
    one = B.Poll(None, _rx_bursts(frames), "cpu")
    one.replenish()
    assert one.next_burst().n == 32 and one.pulls == 1


def test_packet_batch_concat_keeps_frames_and_order():
    rng = np.random.default_rng(3)
    parts, want = [], []
    for k in range(3):
        fr = [bytes(rng.integers(0, 256, int(rng.integers(1, 90)), dtype=np.uint8)) for _ in range(5 + k)]
        parts.append(B.packets.PacketBatch.from_frames(fr, "cpu", slot=16))
        want += fr
    cat = B.packets.PacketBatch.concat(parts)
    assert cat.n == len(want)
    assert [cat.frame(i) for i in range(cat.n)] == want


@pytest.mark.gpu
def test_poll_target_parse_matches_oracle(ctx):
    """IMIX arriving as RX bursts of 32 frames, gathered 2048 at a time and
    parsed on the device: every packet's parse equals the oracle's on the
    same frames, in arrival order, the last gather short."""
    from capsule_amd import synth

    import oracle_lib

    a, o, l = synth.imix(5000, seed=12, vlan_frac=0.1)
    frames = [bytes(a[int(x):int(x) + int(n)]) for x, n in zip(o, l)]
    flags = N.F_ACCEPT_ALL | N.F_CSUM_IP | N.F_CSUM_L4 | N.F_FLOW_HASH
    src = B.Poll(ctx, _rx_bursts(frames), "cuda", target=2048)
    got_meta, got_hash, sizes = [], [], []
    while True:
        src.replenish()
        pipe = src.parse(flags)
        out = pipe.next_burst()
        if out is None:
            break
        sizes.append(out.n)
        got_meta.append(out.parsed.meta.cpu().numpy().view(np.uint32))
        got_hash.append(out.parsed.flow_hash.cpu().numpy().view(np.uint64))
    assert sizes == [2048, 2048, 904]
    om, oc, oh, _ = oracle_lib.parse_batch(a, o, l, flags, fields=False)
    assert (np.concatenate(got_meta) == om).all()
    assert (np.concatenate(got_hash) == oh).all()
