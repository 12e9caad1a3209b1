"""Udp/Tcp::set_src_ip / set_dst_ip (udp.rs:174-201, tcp.rs:432-459): the
oracle pinned by the reference's own `set_src_dst_ip` tests (udp.rs:423-445,
tcp.rs:744-766) on its fixture packets, the RFC 1624 update checked against a
full recompute, and cgpu_set_ip bit-exact against the oracle on the GPU."""
import ipaddress
import json
import pathlib

import numpy as np
import pytest

import oracle_lib
from capsule_amd import _native as N
from capsule_amd import synth

GOLD = pathlib.Path(__file__).resolve().parent / "golden"
PACKETS = json.loads((GOLD / "reference_packets.json").read_text())
ALL = N.F_ACCEPT_ALL | N.F_CSUM_IP | N.F_CSUM_L4 | N.F_FLOW_HASH
DEV = "cuda:0"


def _a(s):
    ip = ipaddress.ip_address(s)
    return oracle_lib.ip_addrs([(ip.version, ip.packed)])


def _l4_csum(frame, meta):
    eth = N.meta_eth_len(meta)
    l4 = eth + (40 if N.meta_l3(meta) == N.L3_IPV6 else 20)
    at = l4 + (6 if N.meta_l4(meta) == N.L4_UDP else 16)
    return int.from_bytes(bytes(frame[at : at + 2]), "big")


@pytest.mark.parametrize("name", ["IPV4_UDP_PACKET", "IPV4_TCP_PACKET"])
def test_reference_set_src_dst_ip(name):
    """udp.rs:423-445 / tcp.rs:744-766: set_src_ip(10.0.0.0) changes the
    checksum and the envelope's src; set_dst_ip(20.0.0.0) likewise; a v6
    address on a v4 packet is an error."""
    fr = bytes.fromhex(PACKETS[name]["hex"])
    arena, off, ln = synth.pack_frames([fr])
    meta, *_ = oracle_lib.parse_batch(arena, off, ln, ALL, fields=False)
    eth = N.meta_eth_len(int(meta[0]))
    old = _l4_csum(arena[off[0]:], int(meta[0]))
    a1, st = oracle_lib.set_ip(arena, off, ln, meta, src=_a("10.0.0.0"))
    assert st[0] == N.SETIP_OK
    assert bytes(a1[eth + 12 : eth + 16]) == bytes([10, 0, 0, 0])
    c1 = _l4_csum(a1, int(meta[0]))
    assert c1 != old
    a2, st = oracle_lib.set_ip(a1, off, ln, meta, dst=_a("20.0.0.0"))
    assert st[0] == N.SETIP_OK
    assert bytes(a2[eth + 16 : eth + 20]) == bytes([20, 0, 0, 0])
    assert _l4_csum(a2, int(meta[0])) != c1
    a3, st = oracle_lib.set_ip(a2, off, ln, meta, src=_a("::"))
    assert st[0] == N.SETIP_SRC_MISMATCH and (a3 == a2).all()
    # both in one call = the two calls in sequence
    a4, st = oracle_lib.set_ip(arena, off, ln, meta, src=_a("10.0.0.0"), dst=_a("20.0.0.0"))
    assert st[0] == N.SETIP_OK and (a4 == a2).all()


def test_incremental_equals_recompute():
    """RFC 1624 on a valid checksum gives the full recompute's value: every
    UDP/TCP frame of a reconciled IMIX batch still verifies after its
    addresses change (the v4 header checksum is left stale, like
    Ipv4::set_src)."""
    arena, off, ln = synth.imix(20_000, vlan_frac=0.1, seed=11)
    meta, *_ = oracle_lib.parse_batch(arena, off, ln, ALL, fields=False)
    rng = np.random.default_rng(2)
    n = len(off)
    v6 = N.meta_l3(meta) == N.L3_IPV6
    src = np.zeros(n, oracle_lib.IP_ADDR)
    dst = np.zeros(n, oracle_lib.IP_ADDR)
    for a in (src, dst):
        a["octets"] = rng.integers(0, 256, (n, 16), dtype=np.uint8)
        a["family"] = np.where(v6, 6, 4)
        a["octets"][~v6, 4:] = 0
    out, st = oracle_lib.set_ip(arena, off, ln, meta, src=src, dst=dst)
    assert (st == N.SETIP_OK).all()
    m2, *_ = oracle_lib.parse_batch(out, off, ln, ALL, fields=False)
    assert ((m2 & N.META_L4_CSUM_OK) != 0).all()
    assert not ((m2[~v6] & N.META_IP_CSUM_OK) != 0).all()


def test_skip_and_mismatch_cases():
    """ICMP, extension-header and failed parses are left alone; a family
    mismatch in dst keeps the src update (set_src_ip succeeded)."""
    frames = [bytes.fromhex(PACKETS[k]["hex"]) for k in
              ("ICMPV4_PACKET", "SR_TCP_PACKET", "ARP4_PACKET", "IPV6_TCP_PACKET")]
    arena, off, ln = synth.pack_frames(frames)
    flags = ALL | N.F_ACCEPT_ICMP | N.F_V6_EXT
    meta, *_ = oracle_lib.parse_batch(arena, off, ln, flags, fields=False)
    src = oracle_lib.ip_addrs([(4, b"\x01\x02\x03\x04")] * 3 + [(6, bytes(range(16)))])
    dst = _a("1.1.1.1")
    out, st = oracle_lib.set_ip(arena, off, ln, meta, src=src, dst=dst)
    assert list(st) == [N.SETIP_SKIPPED] * 3 + [N.SETIP_DST_MISMATCH]
    o3 = int(off[3])
    assert (out[: o3] == arena[: o3]).all()
    assert bytes(out[o3 + 22 : o3 + 38]) == bytes(range(16))


def _zero_checksum_frames(k=64):
    """UDP frames whose set_src_ip lands on a computed 0, stored as 0xFFFF."""
    arena, off, ln = synth.uniform(k, kind=synth.V4_UDP, frame_len=64, seed=5)
    meta, *_ = oracle_lib.parse_batch(arena, off, ln, ALL, fields=False)
    src = np.zeros(k, oracle_lib.IP_ADDR)
    src["family"] = 4
    for i in range(k):
        f = arena[off[i] :]
        hc = _l4_csum(f, int(meta[i]))
        m = [int.from_bytes(bytes(f[26 + 2 * w : 28 + 2 * w]), "big") for w in range(2)]
        # want fold(~hc + ~m0 + ~m1 + n0 + n1) == 0xFFFF with n0 = 0
        s = (~hc & 0xFFFF) + (~m[0] & 0xFFFF) + (~m[1] & 0xFFFF)
        s = (s >> 16) + (s & 0xFFFF)
        s = (s >> 16) + (s & 0xFFFF)
        n1 = (0xFFFF - s) % 0xFFFF
        src[i]["octets"][2:4] = [n1 >> 8, n1 & 0xFF]
    return arena, off, ln, meta, src


def test_udp_zero_checksum_stored_as_ffff():
    arena, off, ln, meta, src = _zero_checksum_frames()
    out, st = oracle_lib.set_ip(arena, off, ln, meta, src=src)
    assert (st == 0).all()
    assert all(_l4_csum(out[o:], int(m)) == 0xFFFF for o, m in zip(off, meta))


# ---- GPU parity -------------------------------------------------------------


def _gpu_vs_oracle(ctx, arena, off, ln, flags, src, dst):
    import torch

    from capsule_amd import packets

    b = packets.PacketBatch.from_numpy(arena, off, ln, DEV)
    r = packets.parse(ctx, b, flags)
    st = packets.set_ip(ctx, b, r.meta, src=src, dst=dst)
    torch.cuda.synchronize()
    meta, *_ = oracle_lib.parse_batch(arena, off, ln, flags, fields=False)
    assert (r.meta.cpu().numpy().view(np.uint32) == meta).all()
    want, wst = oracle_lib.set_ip(arena, off, ln, meta, src=src, dst=dst)
    assert (st.cpu().numpy() == wst).all(), "status mismatch"
    assert (b.arena.cpu().numpy() == want).all(), "frame bytes mismatch"
    return wst


@pytest.mark.gpu
def test_set_ip_gpu_per_packet_mixed_families(ctx):
    a, o, l = synth.imix(100_000, vlan_frac=0.1, seed=21)
    fa, fo, fl = synth.fuzz(5_000, seed=22)
    arena, off, ln = synth.pack_frames(
        [bytes(a[x : x + y]) for x, y in zip(o, l)] + [bytes(fa[x : x + y]) for x, y in zip(fo, fl)])
    n = len(off)
    rng = np.random.default_rng(23)
    addrs = []
    for _ in range(2):
        x = np.zeros(n, oracle_lib.IP_ADDR)
        x["octets"] = rng.integers(0, 256, (n, 16), dtype=np.uint8)
        x["family"] = np.where(rng.random(n) < 0.5, 6, 4)
        addrs.append(x)
    st = _gpu_vs_oracle(ctx, arena, off, ln, ALL | N.F_ACCEPT_ICMP | N.F_V6_EXT, *addrs)
    assert len(set(st.tolist())) == 4  # every status occurs


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["src", "dst", "both"])
def test_set_ip_gpu_broadcast(ctx, which):
    arena, off, ln = synth.imix(50_000, v6_frac=0.0, seed=31)
    a = _a("203.0.113.1")
    _gpu_vs_oracle(ctx, arena, off, ln, ALL, a if which != "dst" else None,
                   a if which != "src" else None)


@pytest.mark.gpu
def test_set_ip_gpu_zero_checksum_and_fixtures(ctx):
    arena, off, ln, meta, src = _zero_checksum_frames()
    _gpu_vs_oracle(ctx, arena, off, ln, ALL, src, None)
    frames = [bytes.fromhex(h) for v in PACKETS.values() for h in v.get("packets", [v.get("hex")])]
    arena, off, ln = synth.pack_frames(frames)
    n = len(off)
    _gpu_vs_oracle(ctx, arena, off, ln, ALL | N.F_ACCEPT_ICMP | N.F_V6_EXT,
                   oracle_lib.ip_addrs([(6, bytes(range(16)))] * n), _a("192.0.2.7"))


@pytest.mark.gpu
def test_set_ip_gpu_empty_and_errors(ctx):
    import torch

    from capsule_amd import packets

    b = packets.PacketBatch.from_numpy(np.zeros(64, np.uint8), np.zeros(0, np.uint32),
                                       np.zeros(0, np.uint16), DEV)
    st = packets.set_ip(ctx, b, torch.zeros(0, dtype=torch.int32, device=DEV), src=_a("1.2.3.4"))
    assert st.numel() == 0
    arena, off, ln = synth.imix(10, seed=1)
    b = packets.PacketBatch.from_numpy(arena, off, ln, DEV)
    r = packets.parse(ctx, b, ALL)
    with pytest.raises(ValueError):
        packets.set_ip(ctx, b, r.meta, src=oracle_lib.ip_addrs([(4, b"\0\0\0\0")] * 3))
