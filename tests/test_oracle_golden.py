"""Pin the CPU oracle to the reference's own known-answer tests.

Every value comes from tests/golden/reference_kats.json, transcribed from the
asserts of the reference's unit tests (file:line in each entry), applied to
the reference's own fixture packets (core/src/testils/byte_arrays.rs and the
example pcaps).  No GPU.
"""
import json
import pathlib

import numpy as np
import pytest

import oracle_lib
import pyref
from capsule_amd import _native as N
from capsule_amd import synth

GOLD = pathlib.Path(__file__).resolve().parent / "golden"
PACKETS = json.loads((GOLD / "reference_packets.json").read_text())
KATS = json.loads((GOLD / "reference_kats.json").read_text())
REC = np.dtype(N.HDR_RECORD_FIELDS)
ALL = N.F_ACCEPT_ALL | N.F_CSUM_IP | N.F_CSUM_L4 | N.F_FLOW_HASH
PARSE_FLAGS = {  # which typed parse the reference test performed
    None: ALL,
    "v4": N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_ACCEPT_TCP | N.F_CSUM_IP,
    "v6": N.F_ACCEPT_V6 | N.F_ACCEPT_UDP | N.F_ACCEPT_TCP,
    "udp": N.F_ACCEPT_V4 | N.F_ACCEPT_V6 | N.F_ACCEPT_UDP,
    "tcp": N.F_ACCEPT_V4 | N.F_ACCEPT_V6 | N.F_ACCEPT_TCP,
    "icmp": N.F_ACCEPT_V4 | N.F_ACCEPT_V6 | N.F_ACCEPT_ICMP | N.F_CSUM_L4,
    "ext": ALL | N.F_ACCEPT_ICMP | N.F_V6_EXT,
}
EXT = np.dtype(N.EXT_RECORD_FIELDS)


def run_one(name, flags):
    fr = bytes.fromhex(PACKETS[name]["hex"])
    arena, off, ln = synth.pack_frames([fr])
    meta, csum, h, fl, ext = oracle_lib.parse_batch_ext(arena, off, ln, flags)
    return (fr, int(meta[0]), int(csum[0]), int(h[0]), fl.view(REC).reshape(-1)[0],
            ext.view(EXT).reshape(-1)[0])


@pytest.mark.parametrize("kat", KATS["kats"], ids=lambda k: f"{k['packet']}@{k['src']}")
def test_reference_kat(kat):
    fr, meta, csum, h, r, x = run_one(kat["packet"], PARSE_FLAGS[kat.get("parse")])
    if "status" in kat:
        assert N.PKT_STATUS[meta & 0xFF] == kat["status"]
        return
    for key, want in kat.get("expect", {}).items():
        if key == "ext.segment0":
            got = bytes(x["segment0"]).hex()
        elif key == "ext.kind":
            got = int(x["kind"])
            assert got == (meta >> 24) & 3
        elif key.startswith("ext."):
            got = int(x[key[4:]])
        elif key in ("dst_mac", "src_mac", "src_ip", "dst_ip"):
            got = bytes(r[key]).hex()[: len(want)]
        elif key == "dont_fragment":
            got = int(r["ip_flags"]) & 1
        elif key == "more_fragments":
            got = (int(r["ip_flags"]) >> 1) & 1
        elif key in ("udp_length", "window"):
            got = int(r["udp_length_or_window"])
        elif key == "msg_type":
            got = int(r["src_port"])
        elif key == "code":
            got = int(r["dst_port"])
        elif key == "l4":
            got = ["NONE", "UDP", "TCP", "ICMP"][N.meta_l4(meta)]
        elif key == "ip_csum":
            got = csum & 0xFFFF
        elif key == "l4_csum":
            got = csum >> 16
        elif key == "flow":
            src, dst, sp, dp, pr = want
            assert bytes(r["src_ip"]).hex()[: len(src)] == src
            assert bytes(r["dst_ip"]).hex()[: len(dst)] == dst
            assert (int(r["src_port"]), int(r["dst_port"])) == (sp, dp)
            assert N.meta_l4(meta) == (N.L4_UDP if pr == 17 else N.L4_TCP)
            continue
        else:
            got = int(r[key])
        assert got == want, (key, got, want)


def test_compute_inc_kat():
    L = oracle_lib.lib()
    for k in KATS["compute_inc"]:
        old = np.array(k["old_value"], np.uint16)
        new = np.array(k["new_value"], np.uint16)
        assert L.or_compute_inc(k["old"], old.ctypes.data, new.ctypes.data, len(old)) == k["expect"]


def test_siphash_published_vectors():
    """SipHash paper (Aumasson & Bernstein 2012, App. A) 2-4 vectors, key 00..0f,
    and Rust libcore's SipHasher13 vector for the empty message."""
    L = oracle_lib.lib()
    k0, k1 = 0x0706050403020100, 0x0F0E0D0C0B0A0908
    m = np.arange(15, dtype=np.uint8)
    assert L.or_siphash(2, 4, k0, k1, m.ctypes.data, 15) == 0xA129CA6149BE45E5
    assert L.or_siphash(2, 4, k0, k1, m.ctypes.data, 0) == 0x726FDB47DD0E0E31
    assert L.or_siphash(1, 3, k0, k1, m.ctypes.data, 0) == 0xABAC0158050FC4DC
    # the Python restatement agrees with the C one on flow-shaped messages
    rng = np.random.default_rng(5)
    for n in (0, 1, 7, 8, 9, 29, 69, 100):
        msg = rng.integers(0, 256, n, dtype=np.uint8)
        assert L.or_siphash(1, 3, 0, 0, msg.ctypes.data, n) == pyref.siphash13(bytes(msg))


def test_flow_byte_stream_layout():
    """Rust 1.50 #[derive(Hash)] stream of Flow: 29 / 69 bytes."""
    L = oracle_lib.lib()
    src = np.array([139, 133, 217, 110], np.uint8)
    dst = np.array([139, 133, 233, 2], np.uint8)
    out = np.zeros(69, np.uint8)
    n = L.or_flow_bytes(0, src.ctypes.data, dst.ctypes.data, 39376, 1087, 17, out.ctypes.data)
    assert n == 29
    assert bytes(out[:n]) == (bytes(8) + bytes(src) + bytes(8) + bytes(dst)
                              + (39376).to_bytes(2, "little") + (1087).to_bytes(2, "little")
                              + b"\x11")
    s6 = np.arange(16, dtype=np.uint8)
    n = L.or_flow_bytes(1, s6.ctypes.data, s6.ctypes.data, 1, 2, 6, out.ctypes.data)
    assert n == 69
    assert bytes(out[:16]) == (1).to_bytes(8, "little") + (16).to_bytes(8, "little")


def test_pcap_fixtures():
    """examples/pktdump/tcp{4,6}.pcap parse as IPv4/TCP and IPv6/TCP; their
    stored checksums are offload-style zeros."""
    for key, l3, n_expected in (("pktdump_tcp4", N.L3_IPV4, 10), ("pktdump_tcp6", N.L3_IPV6, 10)):
        frames = [bytes.fromhex(h) for h in PACKETS[key]["packets"]]
        assert len(frames) == n_expected
        arena, off, ln = synth.pack_frames(frames)
        meta, csum, h, fl = oracle_lib.parse_batch(arena, off, ln, ALL)
        assert (meta & 0xFF == 0).all()
        assert (((meta >> 16) & 3) == l3).all() and (((meta >> 18) & 3) == N.L4_TCP).all()
        recs = fl.view(REC).reshape(-1)
        assert (recs["l4_checksum"] == 0).all()
    # Appendix B re-derived values for the first tcp4 / tcp6 packet
    frames4 = [bytes.fromhex(h) for h in PACKETS["pktdump_tcp4"]["packets"]]
    m, c, _, _ = oracle_lib.parse_batch(*synth.pack_frames(frames4[:1]), ALL)
    assert (int(c[0]) & 0xFFFF, int(c[0]) >> 16) == (0x66C8, 0x93CE)
    frames6 = [bytes.fromhex(h) for h in PACKETS["pktdump_tcp6"]["packets"]]
    m, c, _, _ = oracle_lib.parse_batch(*synth.pack_frames(frames6[:1]), ALL)
    assert int(c[0]) >> 16 == 0xAAD2


def test_ipv6_tcp_fixture_has_wrong_stored_checksum():
    """IPV6_TCP_PACKET carries the v4 fixture's 0xa92c (byte_arrays.rs:155);
    the recomputed value is 0x1b1c."""
    fr, meta, csum, h, r, _ = run_one("IPV6_TCP_PACKET", ALL)
    assert int(r["l4_checksum"]) == 0xA92C
    assert csum >> 16 == 0x1B1C
    assert not meta & N.META_L4_CSUM_OK


def test_all_fixtures_against_python_restatement():
    """Every reference fixture, every accept/feature flag combination: the C
    oracle and the independent Python restatement agree bit for bit."""
    names = [k for k, v in PACKETS.items() if "hex" in v]
    frames = [bytes.fromhex(PACKETS[k]["hex"]) for k in names]
    for key in ("pktdump_tcp4", "pktdump_tcp6", "ping4d_echo"):
        frames += [bytes.fromhex(h) for h in PACKETS[key]["packets"]]
    arena, off, ln = synth.pack_frames(frames)
    for acc in range(16):
        flags = acc | N.F_CSUM_IP | N.F_CSUM_L4 | N.F_FLOW_HASH
        meta, csum, h, _ = oracle_lib.parse_batch(arena, off, ln, flags)
        for i, fr in enumerate(frames):
            st, m, ipc, l4c, hh = pyref.parse(fr, flags)
            assert int(meta[i]) == (m | st), (i, acc)
            assert int(csum[i]) == (ipc | l4c << 16), (i, acc)
            assert int(h[i]) == hh, (i, acc)
