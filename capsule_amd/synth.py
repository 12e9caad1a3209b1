"""Seeded synthetic packet batches (host side, numpy).

Mirrors the reference's proptest packet strategies
(core/src/testils/proptest/strategy.rs:209-400): every settable header field
is uniform random (`any::<T>()`), ether_type / protocol are implied by the
layer stack, and the packet is `reconcile_all()`-ed, i.e. length fields and
checksums are consistent (strategy.rs:395-397).  The reference's bench draws
from proptest's deterministic RNG (testils/rvg.rs:40-44), which is not
reproducible outside Rust, so batches here come from numpy's PCG64 with a
fixed seed per configuration.

A batch is (arena u8[], off u32[n], len u16[n]): packets sit at 64-byte
aligned slots of a contiguous arena, the device image of a burst of mbufs.
"""
import numpy as np

ETH_IPV4, ETH_IPV6 = 0x0800, 0x86DD
UDP, TCP, ICMP4, ICMP6 = 17, 6, 1, 58

# kinds: (l3, l4) with l3 in {4, 6}, l4 in {UDP, TCP}
V4_UDP, V4_TCP, V6_UDP, V6_TCP = (4, UDP), (4, TCP), (6, UDP), (6, TCP)
V4_ICMP, V6_ICMP = (4, ICMP4), (6, ICMP6)  # 4-byte generic ICMP header


def l4_header_len(l4):
    return 8 if l4 == UDP else (20 if l4 == TCP else 4)


def _fold(s):
    s = s.astype(np.uint64)
    while True:
        hi = s >> np.uint64(16)
        if not hi.any():
            return s
        s = (s & np.uint64(0xFFFF)) + hi


def _be_word_sum(block):
    """Sum of big-endian u16 words of each row (odd tail padded with 0).

    Rows are summed in chunks of ~16 MiB so a 1 M x 1500-B block needs no
    8-byte-per-byte temporary."""
    m, L = block.shape
    out = np.zeros(m, np.uint64)
    if m == 0 or L == 0:
        return out
    step = max(1, (16 << 20) // L)
    for s in range(0, m, step):
        b = block[s : s + step]
        if L % 2:
            b = np.concatenate([b, np.zeros((b.shape[0], 1), np.uint8)], axis=1)
        else:
            b = np.ascontiguousarray(b)
        out[s : s + step] = b.view(">u2").sum(axis=1, dtype=np.uint64)
    return out


def _put16(a, col, v):
    v = np.asarray(v, dtype=np.uint64)
    a[:, col] = (v >> np.uint64(8)).astype(np.uint8)
    a[:, col + 1] = (v & np.uint64(0xFF)).astype(np.uint8)


def _get16(a, col):
    return a[:, col].astype(np.uint64) * np.uint64(256) + a[:, col + 1]


def build_frames(rng, m, kind, frame_len, vlan=0, hop_limit_min=0):
    """m reconciled frames of one kind and length, as an [m, frame_len] array.

    vlan: 0 none, 1 802.1Q, 2 802.1ad (QinQ) tags (ethernet.rs:164-192).
    """
    l3, l4 = kind
    eth_len = 14 + 4 * vlan
    l3_len = 20 if l3 == 4 else 40
    l4_len = l4_header_len(l4)
    assert frame_len >= eth_len + l3_len + l4_len, (kind, frame_len)
    f = rng.integers(0, 256, size=(m, frame_len), dtype=np.uint8)  # random payload
    # Ethernet (strategy.rs:209-218): random dst/src MACs, ether_type implied.
    et = ETH_IPV4 if l3 == 4 else ETH_IPV6
    if vlan == 0:
        _put16(f, 12, et)
    elif vlan == 1:
        _put16(f, 12, 0x8100)
        _put16(f, 16, et)
    else:
        _put16(f, 12, 0x88A8)
        _put16(f, 16, 0x8100)
        _put16(f, 20, et)
    o = eth_len
    if l3 == 4:  # strategy.rs:220-260, pushed header defaults v4.rs:594-609
        f[:, o] = 0x45
        dscp = rng.integers(0, 256, m, dtype=np.uint16)
        ecn = rng.integers(0, 256, m, dtype=np.uint16)
        f[:, o + 1] = (((dscp << 2) & 0xFC) | (ecn & 0x03)).astype(np.uint8)
        df = rng.integers(0, 2, m, dtype=np.uint16) * 0x4000
        mf = rng.integers(0, 2, m, dtype=np.uint16) * 0x2000
        frag = rng.integers(0, 65536, m, dtype=np.uint32) & 0x1FFF
        _put16(f, o + 6, (df | mf | frag).astype(np.uint64))
        f[:, o + 9] = l4
        _put16(f, o + 2, frame_len - o)  # reconcile: total_length (v4.rs:486-489)
    else:  # ip/v6/mod.rs setters; version 6, random dscp/ecn/flow label
        w = (np.uint64(6) << np.uint64(28)) | rng.integers(0, 1 << 28, m, dtype=np.uint64)
        for b in range(4):
            f[:, o + b] = ((w >> np.uint64(24 - 8 * b)) & np.uint64(0xFF)).astype(np.uint8)
        _put16(f, o + 4, frame_len - o - 40)  # reconcile: payload_length (v6 :331-334)
        f[:, o + 6] = l4
        if hop_limit_min:
            f[:, o + 7] = rng.integers(hop_limit_min, 256, m, dtype=np.uint16).astype(np.uint8)
    t = o + l3_len
    if l4 == UDP:
        _put16(f, t + 4, frame_len - t)  # reconcile: length (udp.rs:350-354)
        cs_at = t + 6
    elif l4 == TCP:
        cs_at = t + 16
    else:  # ICMP checksum at +2 (icmp/v4/mod.rs:88-112)
        cs_at = t + 2
    # L4 checksum over [t, frame_len) with the pseudo-header (checksum.rs).
    _put16(f, cs_at, 0)
    span = frame_len - t
    if l4 == ICMP4:  # Icmpv4::compute_checksum: no pseudo-header
        ph = np.zeros(m, np.uint64)
    elif l3 == 4:
        ph = _be_word_sum(f[:, o + 12 : o + 20]) + np.uint64(l4 + span)
    else:
        ph = _be_word_sum(f[:, o + 8 : o + 40]) + np.uint64(l4 + span)
    s = _fold(_fold(ph) + _be_word_sum(f[:, t:]))
    c = (~s) & np.uint64(0xFFFF)
    if l4 == UDP:
        c = np.where(c == 0, np.uint64(0xFFFF), c)  # udp.rs:137-140
    _put16(f, cs_at, c)
    if l3 == 4:  # header checksum last (reconcile_all order: L4 -> L3)
        _put16(f, o + 10, 0)
        _put16(f, o + 10, (~_fold(_be_word_sum(f[:, o : o + 20]))) & np.uint64(0xFFFF))
    return f


def build_ext_frames(rng, m, l4, frame_len, ext, nseg=1, vlan=0):
    """m reconciled IPv6 frames with one extension header before the L4 layer
    (`l4` in UDP / TCP / ICMP6): ext "srh" = a routing header with `nseg`
    random segments (srh.rs:499-507; hdr_ext_len = 2 nseg, random
    segments_left < nseg, flags and tag), ext "frag" = a fragment header
    (fragment.rs:322-327; random offset, M bit, identification).  The L4
    checksum uses the pseudo-header of the extension's envelope: behind a
    routing header dst = segments[0] (srh.rs:456-470)."""
    eth_len = 14 + 4 * vlan
    xl = 8 + 16 * nseg if ext == "srh" else 8
    t = eth_len + 40 + xl
    assert frame_len >= t + l4_header_len(l4), (frame_len, t)
    f = rng.integers(0, 256, size=(m, frame_len), dtype=np.uint8)
    if vlan == 0:
        _put16(f, 12, ETH_IPV6)
    elif vlan == 1:
        _put16(f, 12, 0x8100)
        _put16(f, 16, ETH_IPV6)
    else:
        _put16(f, 12, 0x88A8)
        _put16(f, 16, 0x8100)
        _put16(f, 20, ETH_IPV6)
    o = eth_len
    w = (np.uint64(6) << np.uint64(28)) | rng.integers(0, 1 << 28, m, dtype=np.uint64)
    for b in range(4):
        f[:, o + b] = ((w >> np.uint64(24 - 8 * b)) & np.uint64(0xFF)).astype(np.uint8)
    _put16(f, o + 4, frame_len - o - 40)
    x = o + 40
    if ext == "srh":
        f[:, o + 6] = 43
        f[:, x] = l4
        f[:, x + 1] = 2 * nseg
        f[:, x + 2] = 4
        f[:, x + 3] = rng.integers(0, nseg, m).astype(np.uint8)
        f[:, x + 4] = nseg - 1
        dst = f[:, x + 8: x + 24]
    else:
        f[:, o + 6] = 44
        f[:, x] = l4
        f[:, x + 1] = 0
        dst = f[:, o + 24: o + 40]
    if l4 == UDP:
        _put16(f, t + 4, frame_len - t)
        cs_at = t + 6
    elif l4 == TCP:
        cs_at = t + 16
    else:
        cs_at = t + 2
    _put16(f, cs_at, 0)
    span = frame_len - t
    ph = _be_word_sum(f[:, o + 8: o + 24]) + _be_word_sum(np.ascontiguousarray(dst)) + \
        np.uint64(l4 + span)
    c = (~_fold(_fold(ph) + _be_word_sum(f[:, t:]))) & np.uint64(0xFFFF)
    if l4 == UDP:
        c = np.where(c == 0, np.uint64(0xFFFF), c)
    _put16(f, cs_at, c)
    return f


def place(groups, order, slot=64):
    """Lay out frames of several same-length groups in `order` into an arena.

    groups: list of [m_g, L_g] arrays; order: array of (group, row) pairs.
    Returns (arena, off, len).  Every frame starts a run of whole `slot`-byte
    blocks, so a group is scattered block-wise (one index per block, not
    per byte), in chunks of rows.
    """
    lens = np.array([groups[g].shape[1] for g, _ in order], dtype=np.uint64)
    slots = (lens + np.uint64(slot - 1)) // np.uint64(slot) * np.uint64(slot)
    off = np.zeros(len(order), dtype=np.uint64)
    if len(order):
        off[1:] = np.cumsum(slots)[:-1]
    total = int(slots.sum()) if len(order) else 0
    assert total < (1 << 32), "arena must stay below 4 GiB (u32 offsets)"
    arena = np.zeros(max(total, slot), dtype=np.uint8)
    blocks = arena[: arena.size // slot * slot].reshape(-1, slot)
    order = np.asarray(order)
    for g, arr in enumerate(groups):
        idx = np.nonzero(order[:, 0] == g)[0] if len(order) else np.zeros(0, np.int64)
        if not len(idx):
            continue
        L = arr.shape[1]
        nb = max(1, -(-L // slot))
        rows = order[idx, 1]
        first = (off[idx] // np.uint64(slot)).astype(np.int64)
        step = max(1, (32 << 20) // (nb * slot))
        for c in range(0, len(idx), step):
            r = rows[c : c + step]
            pad = np.zeros((len(r), nb * slot), np.uint8)
            pad[:, :L] = arr[r]
            bi = first[c : c + step, None] + np.arange(nb)[None, :]
            blocks[bi.reshape(-1)] = pad.reshape(-1, slot)
    return arena, off.astype(np.uint32), lens.astype(np.uint16)


def uniform(n, kind=V4_UDP, frame_len=64, seed=0xC0FFEE, vlan=0, slot=64, hop_limit_min=0):
    """n frames of one kind and size (BASELINE configs 2 and 4)."""
    rng = np.random.default_rng(seed)
    f = build_frames(rng, n, kind, frame_len, vlan, hop_limit_min)
    if slot == frame_len:  # contiguous: no scatter needed
        return f.reshape(-1).copy(), (np.arange(n, dtype=np.uint64) * frame_len).astype(
            np.uint32), np.full(n, frame_len, np.uint16)
    order = np.stack([np.zeros(n, np.int64), np.arange(n)], axis=1)
    return place([f], order, slot)


IMIX_SIZES = (64, 570, 1500)
IMIX_WEIGHTS = (7, 4, 1)


def imix(n, seed=0xC0FFEE + 3, v6_frac=0.5, tcp_frac=0.5, vlan_frac=0.0, slot=64):
    """IMIX 64/570/1500 B at 7:4:1, mixed v4/v6 x UDP/TCP, shuffled (config 3).

    64-B frames cannot hold IPv6/TCP (74 B minimum), so 64-B slots draw from
    {v4/UDP, v4/TCP, v6/UDP}.
    """
    rng = np.random.default_rng(seed)
    w = np.array(IMIX_WEIGHTS, dtype=np.float64)
    size_idx = rng.choice(len(IMIX_SIZES), size=n, p=w / w.sum())
    is6 = rng.random(n) < v6_frac
    istcp = rng.random(n) < tcp_frac
    small = size_idx == 0
    istcp = np.where(small & is6, False, istcp)
    vl = np.where(rng.random(n) < vlan_frac, rng.integers(1, 3, n), 0)
    vl = np.where(small & is6, 0, vl)  # 64-B v6/UDP has no room for a tag
    groups, order_g, order_r = [], np.zeros(n, np.int64), np.zeros(n, np.int64)
    for si, size in enumerate(IMIX_SIZES):
        for l3 in (4, 6):
            for l4 in (UDP, TCP):
                for v in (0, 1, 2):
                    sel = np.nonzero((size_idx == si) & (is6 == (l3 == 6)) &
                                     (istcp == (l4 == TCP)) & (vl == v))[0]
                    if not len(sel):
                        continue
                    groups.append(build_frames(rng, len(sel), (l3, l4), size, v))
                    order_g[sel] = len(groups) - 1
                    order_r[sel] = np.arange(len(sel))
    return place(groups, np.stack([order_g, order_r], axis=1), slot)


def nat64_stream(n, frame_len=256, n_keys=50_000, seed=0xC0FFEE + 4, slot=None,
                 drop_frac=0.0):
    """IPv6/TCP frames for the 6to4 rewrite (config 4).

    Sources come from a pool of `n_keys` distinct (v6 src, tcp src port)
    keys so that NEXT_PORT never wraps for n_keys < 64511; hop_limit is in
    [1, 255] (hop_limit 0 panics in a Rust debug build).  `drop_frac` of the
    packets are IPv6/UDP, which nat_6to4 drops (main.rs:124, 148).
    """
    rng = np.random.default_rng(seed)
    f = build_frames(rng, n, V6_TCP, frame_len, 0, hop_limit_min=1)
    key_src = rng.integers(0, 256, size=(n_keys, 16), dtype=np.uint8)
    key_port = rng.integers(0, 65536, size=n_keys, dtype=np.uint64)
    pick = rng.integers(0, n_keys, size=n)
    f[:, 22:38] = key_src[pick]
    _put16(f, 54, key_port[pick])
    if drop_frac:
        f[rng.random(n) < drop_frac, 20] = UDP
    # re-reconcile the TCP checksum after changing src / port
    o, t = 14, 54
    _put16(f, t + 16, 0)
    span = frame_len - t
    ph = _be_word_sum(f[:, o + 8 : o + 40]) + np.uint64(TCP + span)
    s = _fold(_fold(ph) + _be_word_sum(f[:, t:]))
    _put16(f, t + 16, (~s) & np.uint64(0xFFFF))
    slot = slot or frame_len
    if slot == frame_len:
        return f.reshape(-1).copy(), (np.arange(n, dtype=np.uint64) * frame_len).astype(
            np.uint32), np.full(n, frame_len, np.uint16)
    return place([f], np.stack([np.zeros(n, np.int64), np.arange(n)], axis=1), slot)


def pack_frames(frames, slot=64):
    """Pack arbitrary byte strings at `slot`-aligned offsets."""
    lens = np.array([len(f) for f in frames], dtype=np.uint64)
    slots = np.maximum((lens + np.uint64(slot - 1)) // np.uint64(slot), 1) * np.uint64(slot)
    off = np.zeros(len(frames), np.uint64)
    if len(frames):
        off[1:] = np.cumsum(slots)[:-1]
    arena = np.zeros(max(int(slots.sum()), slot), np.uint8)
    for i, fr in enumerate(frames):
        arena[int(off[i]) : int(off[i]) + len(fr)] = np.frombuffer(bytes(fr), np.uint8)
    return arena, off.astype(np.uint32), lens.astype(np.uint16)


def fuzz(n, seed=1, max_len=1600):
    """Edge-case batch: every kind, VLAN depth, truncations, wrong ether_types
    and protocols, odd lengths and UNALIGNED arena offsets (any byte).

    Returns (arena, off, len) with packets at random byte offsets.
    """
    rng = np.random.default_rng(seed)
    frames = []
    kinds = [V4_UDP, V4_TCP, V6_UDP, V6_TCP, V4_ICMP, V6_ICMP]
    for i in range(n):
        kind = kinds[rng.integers(0, 4) if rng.random() < 0.8 else rng.integers(4, 6)]
        vlan = int(rng.integers(0, 3))
        need = 14 + 4 * vlan + (20 if kind[0] == 4 else 40) + l4_header_len(kind[1])
        L = int(rng.integers(need, max(need + 1, max_len)))
        if rng.random() < 0.5:
            L = int(rng.integers(need, need + 64))
        fr = build_frames(rng, 1, kind, L, vlan)[0]
        r = rng.random()
        if r < 0.15:  # truncate anywhere, including to 0 (BadOffset / OutOfBuffer)
            fr = fr[: int(rng.integers(0, len(fr) + 1))]
        elif r < 0.22:  # wrong ether_type
            et_at = 12 + 4 * vlan
            fr[et_at : et_at + 2] = rng.integers(0, 256, 2, dtype=np.uint8)
        elif r < 0.30:  # wrong L4 protocol
            p_at = 14 + 4 * vlan + (9 if kind[0] == 4 else 6)
            fr[p_at] = rng.choice([0, 1, 6, 17, 58, 132, 255])
        elif r < 0.36:  # corrupt a byte (checksum mismatch)
            j = int(rng.integers(0, len(fr)))
            fr[j] ^= np.uint8(1 + rng.integers(0, 255))
        elif r < 0.40:  # all-zero payload region (checksum 0 / 0xFFFF cases)
            fr[need:] = 0
        frames.append(bytes(fr))
    # unaligned placement with random gaps
    gaps = rng.integers(0, 8, n)
    off = np.zeros(n, np.uint64)
    pos = int(rng.integers(0, 4))
    for i, fr in enumerate(frames):
        off[i] = pos
        pos += len(fr) + int(gaps[i])
    arena = rng.integers(0, 256, size=pos + 16, dtype=np.uint8)  # junk between packets
    for i, fr in enumerate(frames):
        arena[int(off[i]) : int(off[i]) + len(fr)] = np.frombuffer(fr, np.uint8)
    lens = np.array([len(f) for f in frames], np.uint16)
    return arena, off.astype(np.uint32), lens


def nat64_replies(out_arena, off, out_len):
    """IPv4/TCP replies to untagged 6to4 output frames, for the 4to6 rewrite.

    Swapping the IPv4 addresses and the TCP ports turns each output frame
    into the peer's answer, sent to the gateway port the port map assigned;
    both checksums are sums over the swapped words, so they stay valid.
    Frames keep their offsets and lengths (nat_4to6 makes them 20 B longer,
    so the slot must leave that room).
    """
    a = np.array(out_arena, dtype=np.uint8, copy=True)
    o = off.astype(np.int64)
    assert (a[o + 12] == 0x08).all() and (a[o + 13] == 0x00).all(), "untagged IPv4 frames"
    for lo, hi, w in ((26, 30, 4), (34, 36, 2)):
        i = o[:, None] + np.arange(w)[None, :]
        x, y = a[i + lo].copy(), a[i + hi].copy()
        a[i + lo], a[i + hi] = y, x
    return a, off.astype(np.uint32), out_len.astype(np.uint16)


def host_buffer(nbytes):
    """A zeroed u8 array of whole pages of its own (an anonymous mmap, at
    least `nbytes`, rounded up to the page size), for host memory that gets
    registered with the GPU: cgpu_host_register takes whole pages only
    (hipHostRegister pins whole pages: a malloc'd array would pin pages the
    Python heap shares with other allocations).  The mapping lives as long
    as the array."""
    import mmap

    size = (max(int(nbytes), 1) + mmap.PAGESIZE - 1) // mmap.PAGESIZE * mmap.PAGESIZE
    return np.frombuffer(mmap.mmap(-1, size), dtype=np.uint8)


def pinned_buffer(nbytes):
    """(torch pinned tensor, its u8 numpy view): page-locked host memory of
    whole pages (at least `nbytes`), one pinned allocation, as
    cgpu_host_register maps it without registering it again."""
    import mmap

    import torch

    size = (max(int(nbytes), 1) + mmap.PAGESIZE - 1) // mmap.PAGESIZE * mmap.PAGESIZE
    t = torch.zeros(size, dtype=torch.uint8, pin_memory=True)
    assert t.data_ptr() % mmap.PAGESIZE == 0, "pinned allocation not page-aligned"
    return t, t.numpy()


def mbuf_pool(arena, off, length, mem=None, headroom=128, seed=7, room=None):
    """Lay a batch out as a DPDK-style mempool in host memory: one object per
    packet = a 128-B rte_mbuf header (buf_addr @0, data_off @16, pkt_len @36,
    data_len @40, buf_len @54; DPDK 19.11 offsets) followed by its buffer
    (headroom + a data room of `room` bytes, default the longest frame; DPDK's
    default is 2048), object stride a multiple of 64, objects in shuffled
    order (a pool hands out buffers in no particular order).  `mem`: a u8
    array to build in (e.g. a pinned torch tensor's numpy view), else a new
    array of its own pages (host_buffer).  Returns (mem, mbufs u64[n] = the rte_mbuf addresses in
    batch order)."""
    n = len(off)
    length = np.asarray(length, dtype=np.int64)
    if room is None:
        room = int(length.max()) if n else 0
    stride = (128 + headroom + room + 63) // 64 * 64
    need = max(stride * n, 64)
    if mem is None:
        mem = host_buffer(need)
    assert mem.nbytes >= need and mem.dtype == np.uint8
    base = mem.ctypes.data
    objs = np.random.default_rng(seed).permutation(n).astype(np.int64) * stride
    mem[:need] = 0
    buf = (np.uint64(base) + objs.astype(np.uint64) + np.uint64(128))
    for b in range(8):
        mem[objs + b] = ((buf >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.uint8)
    mem[objs + 16] = headroom & 0xFF
    mem[objs + 17] = headroom >> 8
    mem[objs + 40] = (length & 0xFF).astype(np.uint8)
    mem[objs + 41] = (length >> 8).astype(np.uint8)
    for b in range(4):  # pkt_len = data_len (one segment)
        mem[objs + 36 + b] = ((length >> (8 * b)) & 0xFF).astype(np.uint8)
    buf_len = headroom + room
    mem[objs + 54] = buf_len & 0xFF
    mem[objs + 55] = buf_len >> 8
    src0 = np.asarray(off, dtype=np.int64)
    dst0 = objs + 128 + headroom
    for c in range(0, n, 1 << 16):  # frames, 64 Ki packets at a time
        L = length[c:c + (1 << 16)]
        T = int(L.sum())
        if not T:
            continue
        start = np.repeat(np.cumsum(L) - L, L)
        intra = np.arange(T, dtype=np.int64) - start
        mem[np.repeat(dst0[c:c + (1 << 16)], L) + intra] = arena[np.repeat(src0[c:c + (1 << 16)], L) + intra]
    return mem, (np.uint64(base) + objs.astype(np.uint64)).astype(np.uint64)


def mbuf_frames(mem, mbufs):
    """(data_address u64[n], data_len u16[n]) of each mbuf of `mem`, read from
    its header (buf_addr @0 + data_off @16, data_len @40): the pairs an RX
    core hands to cgpu_parse_frames."""
    o = (np.asarray(mbufs, dtype=np.uint64) - np.uint64(mem.ctypes.data)).astype(np.int64)
    buf = np.zeros(len(o), np.uint64)
    for b in range(8):
        buf |= mem[o + b].astype(np.uint64) << np.uint64(8 * b)
    doff = mem[o + 16].astype(np.uint64) | (mem[o + 17].astype(np.uint64) << np.uint64(8))
    dlen = mem[o + 40].astype(np.uint16) | (mem[o + 41].astype(np.uint16) << np.uint16(8))
    return buf + doff, dlen


def mbuf_tailroom(mem, mbufs):
    """Mbuf::tailroom (core/src/dpdk/mbuf.rs:207-213) of each mbuf of `mem`:
    buf_len - data_off - data_len, read from its header; the tailroom a
    4to6 rewrite over (data_address, data_len) pairs needs."""
    o = (np.asarray(mbufs, dtype=np.uint64) - np.uint64(mem.ctypes.data)).astype(np.int64)

    def u16(at):
        return mem[at].astype(np.int64) | (mem[at + 1].astype(np.int64) << 8)

    return (u16(o + 54) - u16(o + 16) - u16(o + 40)).astype(np.uint16)



def stale_fields(arena, off, length, meta, seed=5, frac=1.0):
    """Make the length and checksum fields that Packet::reconcile_all
    rewrites stale, in place, on `frac` of the packets whose parse `meta`
    recorded the layer: random UDP length, L4 checksum, IPv4 total_length and
    header checksum, IPv6 payload_length, plus a new random destination port
    (the `set_dst_port` a pipeline makes before reconciling).  Packets behind
    an IPv6 extension header keep their L4 fields (their L4 offset is not in
    the meta word).  Returns the number of packets changed."""
    rng = np.random.default_rng(seed)
    meta = np.asarray(meta, np.uint32)
    o = np.asarray(off, np.int64)
    n = len(o)
    hit = rng.random(n) < frac
    hl = ((meta >> 8) & 0xFF).astype(np.int64)
    l3 = (meta >> 16) & 3
    l4 = (meta >> 18) & 3
    ext = (meta >> 24) & 3
    ok = (meta & 0xFF) == 0
    ln = np.asarray(length, np.int64)

    def scramble(sel, at):
        at = at[sel]
        arena[at] = rng.integers(0, 256, len(at), dtype=np.uint8)
        arena[at + 1] = rng.integers(0, 256, len(at), dtype=np.uint8)

    v4 = hit & (l3 == 1) & (hl + 20 <= ln)
    v6 = hit & (l3 == 2) & (hl + 40 <= ln)
    scramble(v4, o + hl + 2)
    scramble(v4, o + hl + 10)
    scramble(v6, o + hl + 4)
    t = o + hl + np.where(l3 == 2, 40, 20)
    l4s = hit & ok & (ext == 0) & (l3 != 0)
    udp, tcp, icmp = l4s & (l4 == 1), l4s & (l4 == 2), l4s & (l4 == 3)
    scramble(udp, t + 4)
    scramble(udp, t + 6)
    scramble(udp | tcp, t + 2)  # set_dst_port
    scramble(tcp, t + 16)
    scramble(icmp, t + 2)
    return int(hit.sum())
