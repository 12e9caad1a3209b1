"""Second, independent restatement of the reference parse/checksum path in
plain Python (test infrastructure only), used to cross-check the C oracle on
small batches so the oracle is not trusted on its own say-so.

Follows core/src/packets/{ethernet,ip/v4,ip/v6/mod,udp,tcp,checksum}.rs,
icmp/v4/mod.rs:118-129,205-220, icmp/v6/mod.rs:123-138,217-232 and
core/src/dpdk/mbuf.rs:313-327; the flow hash uses hashlib-free SipHash-1-3.
"""
import struct

ST = {"OK": 0, "ETH_BAD_OFFSET": 1, "ETH_OUT_OF_BUFFER": 2, "NOT_IPV4": 3, "NOT_IPV6": 4,
      "NOT_IP": 5, "L3_BAD_OFFSET": 6, "L3_OUT_OF_BUFFER": 7, "NOT_UDP": 8, "NOT_TCP": 9,
      "NOT_L4": 10, "L4_BAD_OFFSET": 11, "L4_OUT_OF_BUFFER": 12, "NOT_ICMPV4": 15,
      "NOT_ICMPV6": 16}
M64 = (1 << 64) - 1


def compute(ph, data):  # checksum.rs:145-168
    s = ph
    if len(data) % 2:
        s += data[-1] << 8
        data = data[:-1]
    for i in range(0, len(data), 2):
        s += (data[i] << 8) | data[i + 1]
    while s >> 16:
        s = (s >> 16) + (s & 0xFFFF)
    return (~s) & 0xFFFF


def fold(s):
    while s >> 16:
        s = (s >> 16) + (s & 0xFFFF)
    return s


def _rotl(x, b):
    return ((x << b) | (x >> (64 - b))) & M64


def siphash13(msg):
    v0, v1, v2, v3 = 0x736F6D6570736575, 0x646F72616E646F6D, 0x6C7967656E657261, 0x7465646279746573

    def rnd():
        nonlocal v0, v1, v2, v3
        v0 = (v0 + v1) & M64; v1 = _rotl(v1, 13) ^ v0; v0 = _rotl(v0, 32)
        v2 = (v2 + v3) & M64; v3 = _rotl(v3, 16) ^ v2
        v0 = (v0 + v3) & M64; v3 = _rotl(v3, 21) ^ v0
        v2 = (v2 + v1) & M64; v1 = _rotl(v1, 17) ^ v2; v2 = _rotl(v2, 32)

    n = len(msg)
    full = n - n % 8
    for i in range(0, full, 8):
        m = struct.unpack_from("<Q", msg, i)[0]
        v3 ^= m; rnd(); v0 ^= m
    b = (n & 0xFF) << 56
    for t, c in enumerate(msg[full:]):
        b |= c << (8 * t)
    v3 ^= b; rnd(); v0 ^= b
    v2 ^= 0xFF
    rnd(); rnd(); rnd()
    return v0 ^ v1 ^ v2 ^ v3


def flow_bytes(v6, src, dst, sport, dport, proto):
    out = b""
    for a in (src, dst):
        out += struct.pack("<q", 1 if v6 else 0)
        out += (struct.pack("<Q", 16) + a) if v6 else a
    return out + struct.pack("<HHB", sport, dport, proto)


def parse(p, flags):
    """-> (status, meta_without_status, ip_c, l4_c, hash)"""
    acc4, acc6, accu, acct = (flags >> 0) & 1, (flags >> 1) & 1, (flags >> 2) & 1, (flags >> 3) & 1
    acci = (flags >> 7) & 1
    if not flags & 0x3:
        acc4 = acc6 = 1
    if not (accu or acct or acci):
        accu = acct = 1
    n = len(p)
    meta, ip_c, l4_c, h = 0, 0, 0, 0
    if n == 0:
        return ST["ETH_BAD_OFFSET"], meta, ip_c, l4_c, h
    if n < 14:
        return ST["ETH_OUT_OF_BUFFER"], meta, ip_c, l4_c, h
    marker = (p[12] << 8) | p[13]
    vl = 1 if marker == 0x8100 else 2 if marker == 0x88A8 else 0
    hl = 14 + 4 * vl
    if n < hl:
        return ST["ETH_OUT_OF_BUFFER"], meta, ip_c, l4_c, h
    et = (p[hl - 2] << 8) | p[hl - 1]
    meta |= hl << 8 | (vl == 1) << 22 | (vl == 2) << 23
    if acc4 and et == 0x0800:
        l3, l3len = 1, 20
    elif acc6 and et == 0x86DD:
        l3, l3len = 2, 40
    else:
        return (ST["NOT_IP"] if acc4 and acc6 else ST["NOT_IPV4"] if acc4 else ST["NOT_IPV6"],
                meta, ip_c, l4_c, h)
    if not hl < n:
        return ST["L3_BAD_OFFSET"], meta, ip_c, l4_c, h
    if hl + l3len > n:
        return ST["L3_OUT_OF_BUFFER"], meta, ip_c, l4_c, h
    ip = p[hl:hl + l3len]
    meta |= l3 << 16
    if l3 == 1:
        proto = ip[9]
        if flags & 0x10:
            hdr = bytearray(ip); hdr[10:12] = b"\0\0"
            ip_c = compute(0, bytes(hdr))
            if ip_c == ((ip[10] << 8) | ip[11]):
                meta |= 1 << 20
        src, dst = ip[12:16], ip[16:20]
    else:
        proto = ip[6]
        src, dst = ip[8:24], ip[24:40]
    icmp_proto = 1 if l3 == 1 else 58
    if accu and proto == 17:
        l4, l4len, cs = 1, 8, 6
    elif acct and proto == 6:
        l4, l4len, cs = 2, 20, 16
    elif acci and proto == icmp_proto:
        l4, l4len, cs = 3, 4, 2
    elif accu + acct + acci > 1:
        return ST["NOT_L4"], meta, ip_c, l4_c, h
    else:
        return (ST["NOT_UDP"] if accu else ST["NOT_TCP"] if acct else
                ST["NOT_ICMPV4"] if l3 == 1 else ST["NOT_ICMPV6"], meta, ip_c, l4_c, h)
    o = hl + l3len
    if not o < n:
        return ST["L4_BAD_OFFSET"], meta, ip_c, l4_c, h
    if o + l4len > n:
        return ST["L4_OUT_OF_BUFFER"], meta, ip_c, l4_c, h
    meta |= l4 << 18
    pr = {1: 17, 2: 6, 3: icmp_proto}[l4]
    if flags & 0x20:
        span = bytearray(p[o:]); span[cs:cs + 2] = b"\0\0"
        segs = sum(struct.unpack(">%dH" % (len(src) // 2), src)) + \
            sum(struct.unpack(">%dH" % (len(dst) // 2), dst))
        ph = fold(segs + pr + len(span))
        if l4 == 3 and l3 == 1:
            ph = 0  # Icmpv4::compute_checksum: compute(0, data)
        l4_c = compute(ph, bytes(span))
        if l4 == 1 and l4_c == 0:
            l4_c = 0xFFFF
        if l4_c == ((p[o + cs] << 8) | p[o + cs + 1]):
            meta |= 1 << 21
    if flags & 0x40 and l4 != 3:  # ICMP has no Flow
        sport, dport = (p[o] << 8) | p[o + 1], (p[o + 2] << 8) | p[o + 3]
        h = siphash13(flow_bytes(l3 == 2, bytes(src), bytes(dst), sport, dport, pr))
    return 0, meta, ip_c, l4_c, h


def reconcile(p, meta, depth):
    """Packet::reconcile_all (packets/mod.rs:297-300) on one frame, held at
    `depth` (3 = the IP layer, 4 = the L4 layer) with the layers and offsets
    its parse `meta` recorded; no extension headers.  -> (bytes, done)."""
    p = bytearray(p)
    n = len(p)
    hl = (meta >> 8) & 0xFF
    l3, l4 = (meta >> 16) & 3, (meta >> 18) & 3
    if l3 == 0 or (meta >> 24) & 3:
        return bytes(p), False
    l3len = 20 if l3 == 1 else 40
    if hl + l3len > n:
        return bytes(p), False
    o = hl + l3len
    if depth == 4:
        if meta & 0xFF or l4 == 0 or o + {1: 8, 2: 20, 3: 4}[l4] > n:
            return bytes(p), False
        span = n - o
        if l4 == 1:  # Udp::reconcile: set_length, then compute_checksum (udp.rs:350-354)
            p[o + 4:o + 6] = struct.pack(">H", span & 0xFFFF)
        cs = {1: 6, 2: 16, 3: 2}[l4]
        p[o + cs:o + cs + 2] = b"\0\0"
        if l3 == 1:
            src, dst = p[hl + 12:hl + 16], p[hl + 16:hl + 20]
        else:
            src, dst = p[hl + 8:hl + 24], p[hl + 24:hl + 40]
        pr = {1: 17, 2: 6, 3: 1 if l3 == 1 else 58}[l4]
        segs = sum(struct.unpack(">%dH" % (len(src) // 2), bytes(src))) + \
            sum(struct.unpack(">%dH" % (len(dst) // 2), bytes(dst)))
        ph = 0 if (l4 == 3 and l3 == 1) else fold(segs + pr + (span & 0xFFFF))
        c = compute(ph, bytes(p[o:]))
        if l4 == 1 and c == 0:
            c = 0xFFFF
        p[o + cs:o + cs + 2] = struct.pack(">H", c)
    if l3 == 1:  # Ipv4::reconcile (ip/v4.rs:486-489)
        p[hl + 2:hl + 4] = struct.pack(">H", (n - hl) & 0xFFFF)
        p[hl + 10:hl + 12] = b"\0\0"
        p[hl + 10:hl + 12] = struct.pack(">H", compute(0, bytes(p[hl:hl + 20])))
    else:  # Ipv6::reconcile (ip/v6/mod.rs:331-334)
        p[hl + 4:hl + 6] = struct.pack(">H", (n - hl - 40) & 0xFFFF)
    return bytes(p), True
