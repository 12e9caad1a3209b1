"""Parity of the HIP parse/checksum/flow-hash kernel with the CPU oracle.

Bit-exact on every output (meta word, both checksums, flow hash, the 96-byte
header record) for the reference's own fixtures, seeded edge-case batches
and the BASELINE configurations; full-size runs are checked through
size-independent properties (every reconciled packet parses and verifies).
"""
import json
import pathlib

import numpy as np
import pytest
import torch

import oracle_lib
from capsule_amd import _native as N
from capsule_amd import synth

pytestmark = pytest.mark.gpu

GOLD = pathlib.Path(__file__).resolve().parent / "golden"
ALL = N.F_ACCEPT_ALL | N.F_CSUM_IP | N.F_CSUM_L4 | N.F_FLOW_HASH
DEV = "cuda:0"


def gpu_parse(ctx, arena, off, ln, flags, fields=True):
    from capsule_amd import packets

    b = packets.PacketBatch.from_numpy(arena, off, ln, DEV)
    r = packets.parse(ctx, b, flags=flags, fields=fields)
    torch.cuda.synchronize()
    meta = r.meta.cpu().numpy().view(np.uint32)
    csum = r.csum.cpu().numpy().view(np.uint32)
    h = r.flow_hash.cpu().numpy().view(np.uint64)
    fl = r.fields.cpu().numpy() if fields else None
    return meta, csum, h, fl


def assert_ext_parity(ctx, arena, off, ln, flags):
    """Every output including the extension records (CGPU_F_V6_EXT)."""
    from capsule_amd import packets

    b = packets.PacketBatch.from_numpy(arena, off, ln, DEV)
    r = packets.parse(ctx, b, flags=flags, fields=True, ext=True)
    torch.cuda.synchronize()
    om, oc, oh, of, ox = oracle_lib.parse_batch_ext(arena, off, ln, flags)
    gm = r.meta.cpu().numpy().view(np.uint32)
    assert (gm == om).all(), ("meta", np.nonzero(gm != om)[0][:8], gm[gm != om][:4], om[gm != om][:4])
    if flags & (N.F_CSUM_IP | N.F_CSUM_L4):  # outputs that were requested
        gc = r.csum.cpu().numpy().view(np.uint32)
        assert (gc == oc).all(), ("csum", np.nonzero(gc != oc)[0][:8])
    if flags & N.F_FLOW_HASH:
        gh = r.flow_hash.cpu().numpy().view(np.uint64)
        assert (gh == oh).all(), ("hash", np.nonzero(gh != oh)[0][:8])
    assert (r.fields.cpu().numpy() == of).all(), "fields"
    gx = r.ext.cpu().numpy()
    assert (gx == ox).all(), ("ext", np.nonzero((gx != ox).any(axis=1))[0][:8])


def assert_parity(ctx, arena, off, ln, flags, fields=True):
    gm, gc, gh, gf = gpu_parse(ctx, arena, off, ln, flags, fields)
    om, oc, oh, of = oracle_lib.parse_batch(arena, off, ln, flags, fields)
    bad = np.nonzero(gm != om)[0]
    assert not len(bad), f"meta differs at {bad[:8]}: gpu {gm[bad[:4]]} oracle {om[bad[:4]]}"
    if flags & (N.F_CSUM_IP | N.F_CSUM_L4):
        bad = np.nonzero(gc != oc)[0]
        assert not len(bad), f"csum differs at {bad[:8]}: gpu {gc[bad[:4]]} oracle {oc[bad[:4]]}"
    if flags & N.F_FLOW_HASH:
        bad = np.nonzero(gh != oh)[0]
        assert not len(bad), f"hash differs at {bad[:8]}"
    if fields:
        bad = np.nonzero((gf != of).any(axis=1))[0]
        assert not len(bad), f"fields differ at {bad[:8]}"
    return om


def test_reference_fixtures_every_flag_combination(ctx):
    pk = json.loads((GOLD / "reference_packets.json").read_text())
    frames = [bytes.fromhex(v["hex"]) for v in pk.values() if "hex" in v]
    for v in pk.values():
        frames += [bytes.fromhex(h) for h in v.get("packets", [])]
    arena, off, ln = synth.pack_frames(frames)
    for acc in list(range(16)) + [a | N.F_ACCEPT_ICMP for a in range(16)]:
        for feat in (0, N.F_CSUM_IP, N.F_CSUM_L4, N.F_FLOW_HASH, 0x70):
            assert_parity(ctx, arena, off, ln, acc | feat, fields=True)
            if not acc & (N.F_ACCEPT_V6 | N.F_ACCEPT_TCP | N.F_ACCEPT_ICMP):
                # no header record: the monomorphised IPv4/UDP variant
                assert_parity(ctx, arena, off, ln, acc | feat, fields=False)
    assert_parity(ctx, arena, off, ln, ALL, fields=False)


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_fuzz_unaligned_edge_cases(ctx, seed):
    arena, off, ln = synth.fuzz(3000, seed=seed)
    for flags in (ALL, N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_CSUM_L4,
                  N.F_ACCEPT_V6 | N.F_ACCEPT_TCP | N.F_FLOW_HASH, N.F_CSUM_IP | N.F_CSUM_L4,
                  ALL | N.F_ACCEPT_ICMP, N.F_ACCEPT_ICMP | N.F_CSUM_L4 | N.F_CSUM_IP):
        assert_parity(ctx, arena, off, ln, flags, fields=True)
    assert_parity(ctx, arena, off, ln, ALL, fields=False)
    v4u = N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_CSUM_IP | N.F_CSUM_L4 | N.F_FLOW_HASH
    assert_parity(ctx, arena, off, ln, v4u, fields=False)  # the IPv4/UDP variant
    assert_parity(ctx, arena, off, ln, v4u & ~N.F_ACCEPT_UDP, fields=False)


def test_every_length_boundary(ctx):
    """Each kind truncated to every length 0..L, plus jumbo and max-u16 frames,
    at every arena alignment (BadOffset / OutOfBuffer edges, register-window
    edge at 96 B, the streamed tail, odd spans)."""
    rng = np.random.default_rng(9)
    frames = []
    for kind in (synth.V4_UDP, synth.V4_TCP, synth.V6_UDP, synth.V6_TCP, synth.V4_ICMP,
                 synth.V6_ICMP):
        for vlan in (0, 1, 2):
            full = bytes(synth.build_frames(rng, 1, kind, 180, vlan)[0])
            frames += [full[:L] for L in range(0, 181)]
    for L in (2047, 2048, 9000, 65535):
        frames.append(bytes(synth.build_frames(rng, 1, synth.V6_UDP, L, 0)[0]))
        frames.append(bytes(synth.build_frames(rng, 1, synth.V4_TCP, L, 2)[0]))
    for shift in range(4):
        arena, off, ln = synth.pack_frames(frames)
        arena = np.concatenate([np.zeros(shift, np.uint8), arena])
        assert_parity(ctx, arena, off + shift, ln, ALL)
        assert_parity(ctx, arena, off + shift, ln, ALL | N.F_ACCEPT_ICMP)
        assert_parity(ctx, arena, off + shift, ln, N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_CSUM_IP |
                      N.F_CSUM_L4 | N.F_FLOW_HASH, fields=False)


@pytest.mark.parametrize("slot,shift", [(16, 0), (64, 4), (256, 0), (64, 2)])
def test_checksum_tail_lengths(ctx, slot, shift):
    """Every frame length from 60 to 1300 B (and the 2048-B data room), v4/UDP
    and v6/TCP, untagged and QinQ: the window / tail split at byte 64 or 96,
    one- and two-piece slot tails (pieces of 256 B), the long-tail loop past
    two pieces, and a last chunk that ends anywhere in its 16 B, at several
    arena alignments of the frames."""
    rng = np.random.default_rng(slot + shift)
    frames = []
    for kind, vlan in ((synth.V4_UDP, 0), (synth.V6_TCP, 0), (synth.V4_TCP, 2), (synth.V6_UDP, 1)):
        hdr = 14 + 4 * vlan + (40 if kind[0] == 6 else 20) + (20 if kind[1] == 6 else 8)
        lens = list(range(max(60, hdr), 1301)) + [2047, 2048]
        for L in lens:
            frames.append(bytes(synth.build_frames(rng, 1, kind, L, vlan)[0]))
    order = rng.permutation(len(frames))  # mixed lengths within every wave
    arena, off, ln = synth.pack_frames([frames[i] for i in order], slot)
    arena = np.concatenate([np.zeros(shift, np.uint8), arena])
    om = assert_parity(ctx, arena, off + shift, ln, ALL, fields=False)
    assert ((om & 0xFF) == 0).all() and (om & N.META_L4_CSUM_OK).all()
    # the IPv4/UDP variant on the same frames (the others fail NOT_IPV4 / NOT_UDP)
    om = assert_parity(ctx, arena, off + shift, ln, N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_CSUM_IP |
                       N.F_CSUM_L4 | N.F_FLOW_HASH, fields=False)
    assert (om & N.META_L4_CSUM_OK).sum() > 1000


def test_packet_flush_with_arena_end(ctx):
    """Packets that end exactly at the end of the arena, at every alignment
    (the buffer-resource range check must return zeros, not fault)."""
    rng = np.random.default_rng(10)
    for L in (42, 60, 64, 97, 150):
        fr = bytes(synth.build_frames(rng, 1, synth.V4_UDP, L)[0])
        for shift in range(8):
            arena = np.concatenate([np.zeros(shift, np.uint8), np.frombuffer(fr, np.uint8)])
            assert_parity(ctx, arena, np.array([shift], np.uint32), np.array([L], np.uint16), ALL)


def test_config2_uniform_64B_1M(ctx):
    """BASELINE config 2: 1,048,576 x 64-B IPv4/UDP, bit-exact vs the oracle."""
    arena, off, ln = synth.uniform(1 << 20)
    om = assert_parity(ctx, arena, off, ln, N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_CSUM_IP |
                       N.F_CSUM_L4, fields=False)
    assert (om & 0xFF == 0).all() and (om & N.META_IP_CSUM_OK).all()


def test_config3_imix_parity_and_properties(ctx):
    """BASELINE config 3: IMIX, bit-exact on 256k packets; the full 1M batch
    through properties (all parse, all checksums verify, hash never 0)."""
    arena, off, ln = synth.imix(1 << 18, vlan_frac=0.1)
    assert_parity(ctx, arena, off, ln, ALL, fields=True)
    arena, off, ln = synth.imix(1 << 20)
    gm, gc, gh, _ = gpu_parse(ctx, arena, off, ln, ALL, fields=False)
    assert (gm & 0xFF == 0).all()
    assert (gm & N.META_L4_CSUM_OK).all()
    v4 = ((gm >> 16) & 3) == N.L3_IPV4
    assert (gm[v4] & N.META_IP_CSUM_OK).all()
    assert (gh != 0).all()
    # a sample of 4096 packets spread over the batch, bit-exact
    idx = np.linspace(0, len(off) - 1, 4096).astype(np.int64)
    om, oc, oh, _ = oracle_lib.parse_batch(arena, off[idx], ln[idx], ALL, fields=False)
    assert (gm[idx] == om).all() and (gc[idx] == oc).all() and (gh[idx] == oh).all()


def test_parse_is_idempotent_and_stream_ordered(ctx):
    """Two launches on two streams give identical results (no hidden state)."""
    from capsule_amd import packets

    arena, off, ln = synth.imix(50000, seed=77)
    b = packets.PacketBatch.from_numpy(arena, off, ln, DEV)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    r1 = packets.parse(ctx, b, flags=ALL, stream=s1)
    r2 = packets.parse(ctx, b, flags=ALL, stream=s2)
    torch.cuda.synchronize()
    assert torch.equal(r1.meta, r2.meta) and torch.equal(r1.csum, r2.csum)
    assert torch.equal(r1.flow_hash, r2.flow_hash)


def test_host_entry_point_matches_device_entry_point(ctx):
    from capsule_amd import packets

    arena, off, ln = synth.fuzz(2000, seed=21)
    frames = [bytes(arena[o : o + l]) for o, l in zip(off, ln)]
    meta, csum, fh, recs = packets.parse_host(ctx, frames, flags=ALL, fields=True)
    om, oc, oh, of = oracle_lib.parse_batch(arena, off, ln, ALL, True)
    assert (meta == om).all() and (csum == oc).all() and (fh == oh).all()
    assert (recs.view(np.uint8).reshape(-1, 96) == of).all()


def test_empty_batch(ctx):
    from capsule_amd import packets

    b = packets.PacketBatch(torch.zeros(64, dtype=torch.uint8, device=DEV),
                            torch.zeros(0, dtype=torch.int32, device=DEV),
                            torch.zeros(0, dtype=torch.int16, device=DEV))
    r = packets.parse(ctx, b, flags=ALL)
    torch.cuda.synchronize()
    assert r.meta.numel() == 0


def test_status_strings_follow_reference_errors(ctx):
    from capsule_amd import packets

    pk = json.loads((GOLD / "reference_packets.json").read_text())
    frames = [bytes.fromhex(pk["IPV6_TCP_PACKET"]["hex"]), bytes.fromhex(pk["ARP4_PACKET"]["hex"]),
              b"", bytes(10)]
    b = packets.PacketBatch.from_frames(frames, DEV)
    r = packets.parse(ctx, b, flags=N.F_ACCEPT_V4 | N.F_ACCEPT_UDP)
    torch.cuda.synchronize()
    assert r.error(0) == "not an IPv4 packet."
    assert r.error(1) == "not an IPv4 packet."
    assert r.error(2) == "BadOffset"
    assert r.error(3) == "OutOfBuffer"


def test_verify_only_mode_sets_same_meta(ctx):
    """csum=NULL (verify only) gives the same meta word as storing the values."""
    from capsule_amd import packets

    arena, off, ln = synth.fuzz(3000, seed=55)
    b = packets.PacketBatch.from_numpy(arena, off, ln, DEV)
    r1 = packets.parse(ctx, b, flags=ALL)
    r2 = packets.parse(ctx, b, flags=ALL, out=packets.ParseBuffers(b.n, DEV, csum=False))
    torch.cuda.synchronize()
    assert r2.csum is None
    assert torch.equal(r1.meta, r2.meta) and torch.equal(r1.flow_hash, r2.flow_hash)


def ext_batch(seed):
    """IPv6 routing (1..6 segments) and fragment headers before UDP / TCP /
    ICMPv6, every VLAN depth, frames up to 1500 B, plus truncations at every
    length of a few of them, inconsistent segment lists and plain frames."""
    rng = np.random.default_rng(seed)
    frames = []
    for ext, nseg in [("srh", 1), ("srh", 2), ("srh", 3), ("srh", 6), ("frag", 1)]:
        for l4 in (synth.UDP, synth.TCP, synth.ICMP6):
            for vlan in (0, 1, 2):
                need = 14 + 4 * vlan + 40 + (8 + 16 * nseg if ext == "srh" else 8) + \
                    synth.l4_header_len(l4)
                for L in (need, need + 1, need + 37, 300, 1500):
                    frames.append(bytes(synth.build_ext_frames(rng, 1, l4, max(L, need), ext, nseg,
                                                               vlan)[0]))
    full = bytes(synth.build_ext_frames(rng, 1, synth.TCP, 220, "srh", 3, 1)[0])
    frames += [full[:L] for L in range(0, 221)]
    full = bytes(synth.build_ext_frames(rng, 1, synth.UDP, 120, "frag", 1, 0)[0])
    frames += [full[:L] for L in range(0, 121)]
    for _ in range(40):  # inconsistent segment lists (hdr_ext_len != 2 (last_entry + 1))
        f = bytearray(synth.build_ext_frames(rng, 1, synth.TCP, 200, "srh", 2, 0)[0])
        f[14 + 40 + int(rng.integers(1, 5, dtype=np.int64)) % 2 * 3 + 1] ^= 1 + int(rng.integers(0, 255))
        frames.append(bytes(f))
    a, o, l = synth.imix(300, seed=seed)
    frames += [bytes(a[o[i]: o[i] + l[i]]) for i in range(len(o))]
    order = rng.permutation(len(frames))
    return [frames[i] for i in order]


@pytest.mark.parametrize("seed", [1, 2])
def test_ipv6_extension_headers(ctx, seed):
    frames = ext_batch(seed)
    for shift in (0, 1, 2):
        arena, off, ln = synth.pack_frames(frames)
        arena = np.concatenate([np.zeros(shift, np.uint8), arena])
        for flags in (ALL | N.F_V6_EXT | N.F_ACCEPT_ICMP, ALL | N.F_V6_EXT,
                      N.F_ACCEPT_V6 | N.F_ACCEPT_TCP | N.F_V6_EXT | N.F_CSUM_L4 | N.F_FLOW_HASH,
                      ALL):
            assert_ext_parity(ctx, arena, off + shift, ln, flags)


def test_reference_fixtures_with_extensions(ctx):
    pk = json.loads((GOLD / "reference_packets.json").read_text())
    frames = [bytes.fromhex(v["hex"]) for v in pk.values() if "hex" in v]
    arena, off, ln = synth.pack_frames(frames)
    for acc in (N.F_ACCEPT_ALL, N.F_ACCEPT_V6 | N.F_ACCEPT_TCP, N.F_ACCEPT_V6 | N.F_ACCEPT_UDP):
        for feat in (0, N.F_CSUM_L4, N.F_FLOW_HASH, 0x70, 0x70 | N.F_ACCEPT_ICMP):
            assert_ext_parity(ctx, arena, off, ln, acc | feat | N.F_V6_EXT)


@pytest.mark.parametrize("seed", [1, 2])
def test_rows_path_long_frames(ctx, seed):
    """Batches whose mean slot is 128..640 B run the rows variant; its waves
    of aligned frames up to 512 B (at least half of them >= 128 B) read every
    frame in rows and take the checksum span as the frame's word sum minus
    the words before the span.  Every kind, VLAN depth, length 42..512
    (short frames mixed in), corrupted bytes, ICMP, wrong types: bit-exact."""
    rng = np.random.default_rng(seed)
    kinds = [synth.V4_UDP, synth.V4_TCP, synth.V6_UDP, synth.V6_TCP, synth.V4_ICMP,
             synth.V6_ICMP]
    frames = []
    for j in range(6000):
        kind = kinds[int(rng.integers(0, len(kinds)))]
        vlan = int(rng.integers(0, 3))
        need = 14 + 4 * vlan + (20 if kind[0] == 4 else 40) + synth.l4_header_len(kind[1])
        L = int(rng.integers(need, 513)) if rng.random() < 0.75 else int(rng.integers(need, 128))
        fr = synth.build_frames(rng, 1, kind, max(L, need), vlan)[0]
        r = rng.random()
        if r < 0.05:
            fr[int(rng.integers(0, len(fr)))] ^= 0x41
        elif r < 0.08:
            fr = fr[: int(rng.integers(0, len(fr) + 1))]
        frames.append(bytes(fr))
    for slot in (256, 512):
        arena, off, ln = synth.pack_frames(frames, slot)
        for flags in (ALL, ALL | N.F_ACCEPT_ICMP, N.F_ACCEPT_V6 | N.F_ACCEPT_TCP | N.F_CSUM_L4):
            om = assert_parity(ctx, arena, off, ln, flags, fields=True)
        assert_parity(ctx, arena, off, ln, N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_CSUM_IP |
                      N.F_CSUM_L4 | N.F_FLOW_HASH, fields=False)  # IPv4/UDP variant, rows
        assert (om & N.META_L4_CSUM_OK).sum() > 3000


@pytest.mark.parametrize("seed", [3, 4])
def test_rows_path_with_checksum_tail(ctx, seed):
    """Rows waves with frames longer than the rows' 512 B: the rows sum each
    frame's first 512 B and the checksum tail sums the rest (every kind, VLAN
    depth, lengths 42..2048 with short frames in the majority so the batch's
    mean slot stays in the rows range, corruptions, truncations): bit-exact."""
    rng = np.random.default_rng(seed)
    kinds = [synth.V4_UDP, synth.V4_TCP, synth.V6_UDP, synth.V6_TCP, synth.V4_ICMP]
    frames = []
    for j in range(6000):
        kind = kinds[int(rng.integers(0, len(kinds)))]
        vlan = int(rng.integers(0, 3))
        need = 14 + 4 * vlan + (20 if kind[0] == 4 else 40) + synth.l4_header_len(kind[1])
        r = rng.random()
        L = int(rng.integers(513, 2049)) if r < 0.15 else int(rng.integers(max(need, 128), 300))
        fr = synth.build_frames(rng, 1, kind, max(L, need), vlan)[0]
        r = rng.random()
        if r < 0.05:
            fr[int(rng.integers(0, len(fr)))] ^= 0x41
        elif r < 0.08:
            fr = fr[: int(rng.integers(0, len(fr) + 1))]
        frames.append(bytes(fr))
    for slot in (16, 64):
        arena, off, ln = synth.pack_frames(frames, slot)
        assert 128 <= len(arena) // len(off) <= 2200  # the rows variant is launched
        om = assert_parity(ctx, arena, off, ln, ALL | N.F_ACCEPT_ICMP, fields=True)
        assert (om & N.META_L4_CSUM_OK).sum() > 3000
        assert_parity(ctx, arena, off, ln, N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_CSUM_IP |
                      N.F_CSUM_L4 | N.F_FLOW_HASH, fields=False)


def _stream_frames(rng, m, long_frac=0.4, max_len=1500):
    kinds = [synth.V4_UDP, synth.V4_TCP, synth.V6_UDP, synth.V6_TCP, synth.V4_ICMP, synth.V6_ICMP]
    frames = []
    for _ in range(m):
        kind = kinds[int(rng.integers(0, len(kinds)))]
        vlan = int(rng.integers(0, 3)) if rng.random() < 0.2 else 0
        need = 14 + 4 * vlan + (20 if kind[0] == 4 else 40) + synth.l4_header_len(kind[1])
        L = int(rng.integers(97, max_len + 1)) if rng.random() < long_frac else int(rng.integers(need, 97))
        fr = synth.build_frames(rng, 1, kind, max(L, need), vlan)[0]
        r = rng.random()
        if r < 0.04:
            fr[int(rng.integers(0, len(fr)))] ^= 0x41
        elif r < 0.08:
            fr = fr[: int(rng.integers(0, len(fr) + 1))]  # truncated, down to 0 bytes
        frames.append(bytes(fr))
    return frames


def _pack16(frames, gaps, tail):
    """Frames back to back at 16-B granularity with `gaps[i]` extra 16-B
    chunks after frame i; `tail` bytes of arena past the last frame."""
    ln = np.array([len(f) for f in frames], np.int64)
    step = (ln + 15) // 16 * 16 + 16 * np.asarray(gaps, np.int64)
    step = np.maximum(step, 16)  # a 0-byte frame still takes a chunk (offsets strictly ascend)
    off = np.concatenate([[0], np.cumsum(step)[:-1]])
    arena = np.zeros(int(off[-1] + ln[-1] + tail), np.uint8)
    for o, f in zip(off, frames):
        arena[o:o + len(f)] = np.frombuffer(f, np.uint8)
    return arena, off.astype(np.uint32), ln.astype(np.uint16)


@pytest.mark.parametrize("seed", [5, 6])
def test_stream_path_consecutive_frames(ctx, seed):
    """The stream path (parse.hip: waves of ascending 16-B aligned frames
    within 32 KiB, read as one span and summed per frame by a segmented
    scan): frames of 0..1500 B back to back at 16-B granularity, with and
    without padding chunks between them, every kind, VLAN, ICMP, truncated
    and corrupted frames, spans right at the 32 KiB limit, an arena ending
    16 B and 0 B past the last frame (the second falls back), and a batch
    whose waves are not in ascending order (they fall back): bit-exact."""
    rng = np.random.default_rng(seed)
    frames = _stream_frames(rng, 6400)
    n = len(frames)
    cases = [np.zeros(n, np.int64), rng.integers(0, 3, n)]
    for gaps in cases:
        for tail in (16, 0):
            arena, off, ln = _pack16(frames, gaps, tail)
            assert 128 <= len(arena) // n <= 2200  # the variant with the stream path
            for flags in (ALL | N.F_ACCEPT_ICMP, N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_CSUM_IP |
                          N.F_CSUM_L4 | N.F_FLOW_HASH):
                om = assert_parity(ctx, arena, off, ln, flags, fields=bool(flags & N.F_ACCEPT_V6))
            assert (om & N.META_L4_CSUM_OK).sum() > 1000
    # 64 frames of 512 B (32 KiB, the limit) per wave, then 513 B (over it: rows)
    for L in (512 - 16, 512, 513):
        fr = [bytes(x) for x in synth.build_frames(rng, 1024, synth.V6_TCP, L, 0)]
        arena, off, ln = _pack16(fr, np.zeros(1024, np.int64), 16)
        om = assert_parity(ctx, arena, off, ln, ALL)
        assert (om & N.META_L4_CSUM_OK).all()
    # waves whose offsets are not ascending: the window + tail path
    arena, off, ln = _pack16(frames, cases[1], 16)
    perm = np.arange(n)
    for w in range(0, n - 64, 64):
        perm[w + 3], perm[w + 40] = perm[w + 40], perm[w + 3]
    assert_parity(ctx, arena, off[perm], ln[perm], ALL)


def _pack64(frames, gaps, tail, misalign=()):
    """Frames in 64-B slots (the bench's IMIX arena, the ingress gather's
    layout) with `gaps[i]` extra empty slots after frame i; frames whose
    index is in `misalign` start 16 B into their slot."""
    ln = np.array([len(f) for f in frames], np.int64)
    step = (ln + 63) // 64 * 64 + 64 * np.asarray(gaps, np.int64)
    step = np.maximum(step, 64) + 64  # room for a 16-B shift
    off = np.concatenate([[0], np.cumsum(step)[:-1]])
    off[list(misalign)] += 16
    arena = np.full(int(off[-1] + ln[-1] + tail), 0x5a, np.uint8)  # slot padding is not zero
    for o, f in zip(off, frames):
        arena[o:o + len(f)] = np.frombuffer(f, np.uint8)
    return arena, off.astype(np.uint32), ln.astype(np.uint16)


@pytest.mark.parametrize("seed", [7, 8])
def test_stream_path_64b_slots(ctx, seed):
    """The stream path over frames in 64-B slots, the layout of the bench's
    IMIX arena and of the ingress gather: frames of 0..1500 B with non-zero
    slot padding (loaded with the frame's last chunk or skipped, never summed)
    and 0..2 empty slots between them, every kind, VLAN, ICMP, truncated and
    corrupted frames; waves with one frame 16 B into its slot; mixed waves
    just under and just over the 32 KiB span limit: bit-exact."""
    rng = np.random.default_rng(seed)
    frames = _stream_frames(rng, 6400)
    n = len(frames)
    for gaps in (np.zeros(n, np.int64), rng.integers(0, 3, n)):
        for mis in ((), tuple(range(5, n, 128))):
            arena, off, ln = _pack64(frames, gaps, 16, mis)
            assert 128 <= len(arena) // n <= 2200  # the variant with the stream path
            for flags in (ALL | N.F_ACCEPT_ICMP, N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_CSUM_IP |
                          N.F_CSUM_L4 | N.F_FLOW_HASH):
                om = assert_parity(ctx, arena, off, ln, flags, fields=bool(flags & N.F_ACCEPT_V6))
            assert (om & N.META_L4_CSUM_OK).sum() > 1000
    # waves of k 1000-B frames in 1024-B slots and 64 - k 64-B frames (k < 32:
    # not the rows path): k = 29 spans 31,936 B (streamed), k = 31 33,856 B
    # (over the 32 KiB limit: the window + tail path)
    for k in (29, 31):
        fr, off, o = [], [], 0
        for w in range(16):
            longs = set(rng.choice(64, k, replace=False).tolist())
            for j in range(64):
                L = 1000 if j in longs else 64
                kind = synth.V6_TCP if L == 1000 else synth.V4_UDP
                fr.append(bytes(synth.build_frames(rng, 1, kind, L, 0)[0]))
                off.append(o)
                o += 1024 if L == 1000 else 64
        arena = np.full(o + 16, 0x5a, np.uint8)
        for a0, f in zip(off, fr):
            arena[a0:a0 + len(f)] = np.frombuffer(f, np.uint8)
        ln = np.array([len(f) for f in fr], np.uint16)
        om = assert_parity(ctx, arena, np.array(off, np.uint32), ln, ALL)
        assert (om & N.META_L4_CSUM_OK).all()


@pytest.mark.parametrize("k", [32, 48, 55, 56, 64])
def test_stream_rows_threshold(ctx, k):
    """Waves of k 500-B frames (512-B slots) among 64 - k 64-B ones, the long
    frames 64 B into a 128-B line so that spans start mid-line: k < 56 take
    the stream path (its chunk grid starts at the first frame's line), k >= 56
    (7/8 of the wave) the rows path; each wave's frames shuffled: bit-exact."""
    rng = np.random.default_rng(100 + k)
    fr, off, o = [], [], 64
    for w in range(32):
        longs = set(rng.choice(64, k, replace=False).tolist())
        for j in range(64):
            L = 500 if j in longs else 64
            kind = ((synth.V6_TCP, synth.V4_UDP, synth.V4_TCP, synth.V6_UDP)[(w + j) % 4] if L == 500
                    else (synth.V4_UDP, synth.V4_TCP)[(w + j) % 2])
            fr.append(bytes(synth.build_frames(rng, 1, kind, L, 0)[0]))
            off.append(o)
            o += 512 if L == 500 else 64
    arena = np.full(o + 16, 0x5a, np.uint8)
    for a0, f in zip(off, fr):
        arena[a0:a0 + len(f)] = np.frombuffer(f, np.uint8)
    ln = np.array([len(f) for f in fr], np.uint16)
    assert 128 <= len(arena) // len(fr) <= 2200  # the variant with both paths
    om = assert_parity(ctx, arena, np.array(off, np.uint32), ln, ALL)
    assert (om & N.META_L4_CSUM_OK).all()
