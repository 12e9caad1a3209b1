"""Packet::reconcile_all (core/src/packets/mod.rs:297-300) in the CPU oracle.

The oracle's or_reconcile is pinned by the reference's own reconcile tests
(each "no payload change but force a checksum recompute anyway" test leaves
the fixture's checksum unchanged; srh.rs's compute_checksum test fixes the
checksum behind a routing header) and cross-checked against the independent
Python restatement (tests/pyref.py) on fuzzed frames with stale fields.  No
GPU.
"""
import json
import pathlib
import struct

import numpy as np
import pytest

import oracle_lib
import pyref
from capsule_amd import _native as N
from capsule_amd import synth

GOLD = pathlib.Path(__file__).resolve().parent / "golden"
PACKETS = json.loads((GOLD / "reference_packets.json").read_text())
ALL = N.F_ACCEPT_ALL | N.F_ACCEPT_ICMP
ALL_EXT = ALL | N.F_V6_EXT


def fixture(name):
    return bytes.fromhex(PACKETS[name]["hex"])


def reconcile_one(frame, flags, depth):
    arena, off, ln = synth.pack_frames([frame])
    meta, _, _, _ = oracle_lib.parse_batch(arena, off, ln, flags, fields=False)
    out, st = oracle_lib.reconcile(arena, off, ln, meta, flags, depth)
    return bytes(out[: len(frame)]), int(st[0]), int(meta[0])


# (fixture, accept flags, depth, offset of the checksum the test asserts,
#  reference test): udp.rs:446-457, tcp.rs:767-778, ip/v4.rs:718-728,
#  icmp/v4/mod.rs:503-513, icmp/v6/mod.rs:562-572
RECOMPUTE_KATS = [
    ("IPV4_UDP_PACKET", N.F_ACCEPT_V4 | N.F_ACCEPT_UDP, N.LAYER_L4, 14 + 20 + 6, 0x7228,
     "udp.rs:446-457"),
    ("IPV4_TCP_PACKET", N.F_ACCEPT_V4 | N.F_ACCEPT_TCP, N.LAYER_L4, 14 + 20 + 16, 0xA92C,
     "tcp.rs:767-778"),
    ("IPV4_UDP_PACKET", N.F_ACCEPT_V4 | N.F_ACCEPT_UDP, N.LAYER_L3, 14 + 10, 0xF700,
     "ip/v4.rs:718-728"),
    ("ICMPV4_PACKET", N.F_ACCEPT_V4 | N.F_ACCEPT_ICMP, N.LAYER_L4, 14 + 20 + 2, None,
     "icmp/v4/mod.rs:503-513"),
    ("ROUTER_ADVERT_PACKET", N.F_ACCEPT_V6 | N.F_ACCEPT_ICMP, N.LAYER_L4, 14 + 40 + 2, None,
     "icmp/v6/mod.rs:562-572"),
]


@pytest.mark.parametrize("kat", RECOMPUTE_KATS, ids=lambda k: k[5])
def test_reconcile_keeps_reference_checksum(kat):
    """`expected = x.checksum(); x.reconcile_all(); assert_eq!(expected,
    x.checksum())` on the reference's fixture."""
    name, flags, depth, at, want, _ = kat
    fr = fixture(name)
    out, st, meta = reconcile_one(fr, flags, depth)
    assert st == N.RECON_OK and meta & 0xFF == 0
    before = struct.unpack_from(">H", fr, at)[0]
    if want is not None:
        assert before == want
    assert struct.unpack_from(">H", out, at)[0] == before


def test_reconcile_consistent_fixture_unchanged():
    """Every length and checksum of IPV4_UDP_PACKET is already reconciled:
    reconcile_all from the UDP layer writes the same bytes back."""
    fr = fixture("IPV4_UDP_PACKET")
    out, st, _ = reconcile_one(fr, N.F_ACCEPT_V4 | N.F_ACCEPT_UDP, N.LAYER_L4)
    assert st == N.RECON_OK and out == fr


def srh_variant(segments, segments_left, payload_length=None):
    """SR_TCP_PACKET after `srh.set_segments(segments)` (srh.rs:210-233: the
    segment list resized in place, hdr_ext_len = 2 n, last_entry = n - 1)
    and `set_segments_left`, the IPv6 payload_length left as it was."""
    fr = fixture("SR_TCP_PACKET")
    eth_ip6, srh, rest = fr[:54], fr[54:62], fr[62 + 16 * (fr[58] + 1):]
    hdr = bytearray(srh)
    hdr[1] = 2 * len(segments)
    hdr[3] = segments_left
    hdr[4] = len(segments) - 1
    ip6 = bytearray(eth_ip6)
    if payload_length is not None:
        ip6[18:20] = struct.pack(">H", payload_length)
    return bytes(ip6) + bytes(hdr) + b"".join(segments) + rest


def seg(i):
    return bytes(15) + bytes([i])


def test_reconcile_behind_routing_header_srh_kat():
    """srh.rs:603-652 compute_checksum: with segments [::1, ::2, ::3, ::4]
    and segments_left 3 the TCP checksum (0 in the fixture) becomes nonzero
    after reconcile_all, and stays the same with the list cut to [::1] and
    segments_left 0 (the pseudo-header's dst is segments[0] either way)."""
    four = srh_variant([seg(1), seg(2), seg(3), seg(4)], 3)
    one = srh_variant([seg(1)], 0)
    one_fin = srh_variant([seg(1)], 0)
    sums = []
    for fr in (four, one, one_fin):
        t = 54 + 8 + 16 * (fr[58] + 1)
        assert struct.unpack_from(">H", fr, t + 16)[0] == 0
        out, st, meta = reconcile_one(fr, ALL_EXT, N.LAYER_L4)
        assert st == N.RECON_OK and (meta >> 24) & 3 == N.EXT_SRH
        sums.append(struct.unpack_from(">H", out, t + 16)[0])
        # Ipv6::reconcile after the (no-op) SegmentRouting::reconcile
        assert struct.unpack_from(">H", out, 18)[0] == len(fr) - 54
    assert sums[0] != 0 and sums[0] == sums[1] == sums[2]


def test_reconcile_srh_payload_length():
    """srh.rs:655-681: after `srh.reconcile_all()` the IPv6 payload_length
    is the length of the packet behind the IPv6 header (the SRH's len()),
    not what it was before; reconcile from the SRH is reconcile from L3."""
    fr = srh_variant([seg(1), seg(2)], 1, payload_length=7)
    out, st, _ = reconcile_one(fr, ALL_EXT, N.LAYER_L3)
    assert st == N.RECON_OK
    assert struct.unpack_from(">H", out, 18)[0] == len(fr) - 54
    assert out[20:] == fr[20:]  # nothing else moves


def stale_batch(n, seed, max_len=700, flags=ALL):
    arena, off, ln = synth.fuzz(n, seed=seed, max_len=max_len)
    meta, _, _, _ = oracle_lib.parse_batch(arena, off, ln, flags, fields=False)
    synth.stale_fields(arena, off, ln, meta, seed=seed + 100)
    return arena, off, ln, meta


@pytest.mark.parametrize("depth", [N.LAYER_L3, N.LAYER_L4])
@pytest.mark.parametrize("seed", [3, 4])
def test_oracle_reconcile_matches_python_restatement(depth, seed):
    arena, off, ln, meta = stale_batch(400, seed)
    out, st = oracle_lib.reconcile(arena, off, ln, meta, ALL, depth)
    done = 0
    for i in range(len(off)):
        o, L = int(off[i]), int(ln[i])
        want, ok = pyref.reconcile(bytes(arena[o:o + L]), int(meta[i]), depth)
        assert st[i] == (N.RECON_OK if ok else N.RECON_SKIPPED), i
        assert bytes(out[o:o + L]) == want, (i, hex(int(meta[i])))
        done += ok
    assert done > 200
    # bytes outside the frames (junk between them) are untouched
    mask = np.ones(len(arena), bool)
    for o, L in zip(off.astype(np.int64), ln.astype(np.int64)):
        mask[o:o + L] = False
    assert (out[mask] == arena[mask]).all()


def test_reconciled_frames_verify():
    """After reconcile_all from L4 a fresh parse finds every checksum valid
    and UDP length / IPv4 total_length / IPv6 payload_length equal to the
    spans (the invariant reconcile establishes, udp.rs:350-354, v4.rs:486-489,
    v6/mod.rs:331-334)."""
    arena, off, ln, meta = stale_batch(600, 9)
    out, st = oracle_lib.reconcile(arena, off, ln, meta, ALL, N.LAYER_L4)
    m2, _, _, fl = oracle_lib.parse_batch(out, off, ln, ALL | N.F_CSUM_IP | N.F_CSUM_L4)
    rec = fl.view(np.dtype(N.HDR_RECORD_FIELDS)).reshape(-1)
    hit = st == N.RECON_OK
    assert hit.sum() > 300
    assert ((m2[hit] & N.META_L4_CSUM_OK) != 0).all()
    v4 = hit & (((m2 >> 16) & 3) == N.L3_IPV4)
    assert ((m2[v4] & N.META_IP_CSUM_OK) != 0).all()
    hl = (m2 >> 8) & 0xFF
    assert (rec["ip_length"][v4] == (ln[v4] - hl[v4])).all()
    v6 = hit & (((m2 >> 16) & 3) == N.L3_IPV6)
    assert (rec["ip_length"][v6] == (ln[v6] - hl[v6] - 40)).all()
    udp = hit & (((m2 >> 18) & 3) == N.L4_UDP)
    l4o = hl + np.where(((m2 >> 16) & 3) == N.L3_IPV6, 40, 20)
    assert (rec["udp_length_or_window"][udp] == (ln[udp] - l4o[udp])).all()


def test_reconcile_respects_accept_set_and_depth():
    """A packet held at L4 whose parse failed there (an Err in the reference)
    is not touched; one whose layer the accept set lacks is skipped."""
    fr4 = fixture("IPV4_UDP_PACKET")
    bad = bytearray(fr4)
    bad[14 + 2:14 + 4] = b"\x12\x34"  # stale total_length
    arena, off, ln = synth.pack_frames([bytes(bad)])
    meta, _, _, _ = oracle_lib.parse_batch(arena, off, ln, N.F_ACCEPT_V4 | N.F_ACCEPT_TCP)
    assert N.PKT_STATUS[int(meta[0]) & 0xFF] == "NOT_TCP"
    out, st = oracle_lib.reconcile(arena, off, ln, meta, N.F_ACCEPT_V4 | N.F_ACCEPT_TCP, N.LAYER_L4)
    assert st[0] == N.RECON_SKIPPED and (out == arena).all()
    out, st = oracle_lib.reconcile(arena, off, ln, meta, N.F_ACCEPT_V4 | N.F_ACCEPT_TCP, N.LAYER_L3)
    assert st[0] == N.RECON_OK and bytes(out[:len(fr4)]) == fr4
    meta, _, _, _ = oracle_lib.parse_batch(arena, off, ln, N.F_ACCEPT_V4 | N.F_ACCEPT_UDP)
    out, st = oracle_lib.reconcile(arena, off, ln, meta, N.F_ACCEPT_V6 | N.F_ACCEPT_UDP, N.LAYER_L4)
    assert st[0] == N.RECON_SKIPPED and (out == arena).all()
