"""Second, independent restatement of examples/nat64 (nat_6to4, nat_4to6,
assigned_port, assigned_addr) in plain Python -- test infrastructure only,
used to cross-check the C oracle (oracle/oracle.c) so that its nat64 output
is not trusted on its own say-so.  The reference has no nat64 test or
expected output, so two restatements of different shape agreeing byte for
byte is the pin available.

Shape: an Mbuf object over a bytearray with the reference's extend / shrink
/ read_data rules (core/src/dpdk/mbuf.rs:207-270, 313-327), the packet
operations the example calls, in the example's order, and Python dicts for
PORT_MAP / ADDR_MAP with a u16 NEXT_PORT (examples/nat64/main.rs:35-83).
"""
ACT, DROP, ABORT = 0, 1, 2
ST = {"OK": 0, "ETH_BAD_OFFSET": 1, "ETH_OUT_OF_BUFFER": 2, "NOT_IPV4": 3, "NOT_IPV6": 4,
      "L3_BAD_OFFSET": 6, "L3_OUT_OF_BUFFER": 7, "NOT_TCP": 9, "L4_BAD_OFFSET": 11,
      "L4_OUT_OF_BUFFER": 12, "NOT_RESIZED": 13}
V4_ADDR = bytes([203, 0, 113, 1])  # main.rs:35
DEFAULT_IP_TTL = 64                # ip/mod.rs:33


class PacketError(Exception):
    def __init__(self, status):
        super().__init__(status)
        self.status = status


class Mbuf:
    """data_len bytes of frame in a buffer of `room` bytes past data_off."""

    def __init__(self, frame, room=2048):
        self.data = bytearray(frame)
        self.room = room

    def tailroom(self):  # mbuf.rs:207-213
        return self.room - len(self.data)

    def read_data(self, offset, size, bad, oob):  # mbuf.rs:313-327
        if offset >= len(self.data):
            raise PacketError(bad)
        if offset + size > len(self.data):
            raise PacketError(oob)

    def extend(self, offset, n):  # mbuf.rs:224-245
        if n == 0 or offset > len(self.data) or not n < self.tailroom():
            raise PacketError("NOT_RESIZED")
        self.data[offset:offset] = bytes(n)

    def shrink(self, offset, n):  # mbuf.rs:254-270
        if n == 0 or offset + n > len(self.data):
            raise PacketError("NOT_RESIZED")
        del self.data[offset:offset + n]

    def u16(self, at):
        return self.data[at] << 8 | self.data[at + 1]

    def put16(self, at, v):
        self.data[at:at + 2] = (v & 0xFFFF).to_bytes(2, "big")


def csum(data, start=0):
    """checksum::compute (checksum.rs:145-168): one's-complement sum of
    big-endian words plus `start`, folded and complemented."""
    s = start
    for i in range(0, len(data) - 1, 2):
        s += data[i] << 8 | data[i + 1]
    if len(data) & 1:
        s += data[-1] << 8
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return ~s & 0xFFFF


def words(b):
    return sum(b[i] << 8 | b[i + 1] for i in range(0, len(b), 2))


def ethernet(m):
    """Ethernet::try_parse (ethernet.rs:279-300): (header_len, offset of the
    ether_type field the setters address)."""
    m.read_data(0, 14, "ETH_BAD_OFFSET", "ETH_OUT_OF_BUFFER")
    marker = m.u16(12)
    tags = {0x8100: 1, 0x88A8: 2}.get(marker, 0)  # ethernet.rs:164-181
    hl = 14 + 4 * tags
    if len(m.data) < hl:
        raise PacketError("ETH_OUT_OF_BUFFER")
    return hl, 12 + 4 * tags


def tcp_checksum(m, tcp_off, pseudo):
    """Tcp::compute_checksum (tcp.rs:462-477) with the envelope's pseudo-header."""
    m.put16(tcp_off + 16, 0)
    seg = bytes(m.data[tcp_off:])
    m.put16(tcp_off + 16, csum(seg, pseudo(len(seg))))


class Nat64:
    def __init__(self, first_port=1025):
        self.port_map = {}   # (v6 addr bytes, port) -> gateway port
        self.addr_map = {}   # gateway port -> (v6 addr bytes, port)
        self.next_port = first_port

    def assigned_port(self, addr, port):  # main.rs:41-53
        key = (addr, port)
        if key in self.port_map:
            return self.port_map[key]
        p = self.next_port
        self.next_port = (self.next_port + 1) & 0xFFFF  # AtomicU16::fetch_add wraps
        self.port_map.setdefault(key, p)                 # insert_new keeps the first
        self.addr_map.setdefault(p, key)
        return p

    def nat_6to4(self, frame, room=2048):
        """main.rs:121-150 -> (disposition, status, output frame or None)."""
        m = Mbuf(frame, room)
        try:
            hl, et_at = ethernet(m)
            if m.u16(et_at) != 0x86DD:
                raise PacketError("NOT_IPV6")
            m.read_data(hl, 40, "L3_BAD_OFFSET", "L3_OUT_OF_BUFFER")
            v6 = bytes(m.data[hl:hl + 40])
            if v6[6] != 6:
                return DROP, ST["OK"], None
            vtf = int.from_bytes(v6[0:4], "big")
            dscp, ecn = (vtf & 0x0FC00000) >> 22, (vtf & 0x00300000) >> 20
            ttl = (v6[7] - 1) & 0xFF  # hop_limit - 1, wrapping
            protocol, src, dst = v6[6], v6[8:24], v6[36:40]  # map6to4: segments[6..8]
            m.shrink(hl, 40)          # v6.remove() (packets/mod.rs:242-251)
            m.extend(hl, 20)          # ethernet.push::<Ipv4>() (ip/v4.rs:455-469)
            h = bytearray([0x45, 0, 0, 0, 0, 0, 0, 0, DEFAULT_IP_TTL, 0] + [0] * 10)  # v4.rs:594-609
            m.put16(et_at, 0x0800)
            h[1] = (h[1] & 0x03) | ((dscp << 2) & 0xFF)  # set_dscp (v4.rs:189-191)
            h[1] = (h[1] & 0xFC) | (ecn & 0x03)          # set_ecn (v4.rs:201-203)
            h[8], h[9] = ttl, protocol
            h[12:16], h[16:20] = V4_ADDR, dst
            m.data[hl:hl + 20] = h
            tcp = hl + 20
            if m.data[hl + 9] != 6:                        # Tcp::try_parse (tcp.rs:558-573)
                raise PacketError("NOT_TCP")
            m.read_data(tcp, 20, "L4_BAD_OFFSET", "L4_OUT_OF_BUFFER")
            m.put16(tcp, self.assigned_port(bytes(src), m.u16(tcp)))
            # reconcile_all: Tcp::reconcile, then Ipv4::reconcile (v4.rs:486-489)
            tcp_checksum(m, tcp, lambda n: words(V4_ADDR) + words(dst) + 6 + n)
            m.put16(hl + 2, len(m.data) - hl)
            m.put16(hl + 10, 0)
            m.put16(hl + 10, csum(bytes(m.data[hl:hl + 20])))
            return ACT, ST["OK"], bytes(m.data)
        except PacketError as e:
            return ABORT, ST[e.status], None

    def nat_4to6(self, frame, room=2048):
        """main.rs:86-118 -> (disposition, status, output frame or None)."""
        m = Mbuf(frame, room)
        try:
            hl, et_at = ethernet(m)
            if m.u16(et_at) != 0x0800:
                raise PacketError("NOT_IPV4")
            m.read_data(hl, 20, "L3_BAD_OFFSET", "L3_OUT_OF_BUFFER")
            v4 = bytes(m.data[hl:hl + 20])
            ff = v4[6] << 8 | v4[7]
            if not (v4[9] == 6 and ff & 0x1FFF == 0 and not ff & 0x2000):
                return DROP, ST["OK"], None
            m.read_data(hl + 20, 20, "L4_BAD_OFFSET", "L4_OUT_OF_BUFFER")  # v4.peek::<Tcp4>()
            value = self.addr_map.get(m.u16(hl + 22))  # assigned_addr(tcp.dst_port())
            if value is None:
                return DROP, ST["OK"], None
            dst, port = value
            dscp, ecn = v4[1] >> 2, v4[1] & 0x03
            next_header, hop_limit = v4[9], (v4[8] - 1) & 0xFF
            src = bytes([0, 0x64, 0xFF, 0x9B]) + bytes(8) + v4[12:16]  # map4to6 (main.rs:62-75)
            m.shrink(hl, 20)          # v4.remove()
            m.extend(hl, 40)          # ethernet.push::<Ipv6>() (ip/v6/mod.rs:302-318)
            vtf = (6 << 28)           # Ipv6Header::default (v6/mod.rs:453-463)
            vtf = (vtf & ~0x0FC00000) | ((dscp << 22) & 0x0FC00000)  # set_dscp
            vtf = (vtf & ~0x00300000) | ((ecn << 20) & 0x00300000)   # set_ecn
            h = bytearray(vtf.to_bytes(4, "big") + bytes(2) + bytes([next_header, hop_limit])
                          + src + dst)
            m.data[hl:hl + 40] = h
            m.put16(et_at, 0x86DD)
            tcp = hl + 40             # v6.parse::<Tcp6>()
            m.read_data(tcp, 20, "L4_BAD_OFFSET", "L4_OUT_OF_BUFFER")
            m.put16(tcp + 2, port)    # set_dst_port
            # reconcile_all: Tcp::reconcile (v6 pseudo-header, checksum.rs:56-128),
            # then Ipv6::reconcile (v6/mod.rs:331-334)
            tcp_checksum(m, tcp, lambda n: words(src) + words(dst) + (n >> 16) + (n & 0xFFFF) + 6)
            m.put16(hl + 4, len(m.data) - hl - 40)
            return ACT, ST["OK"], bytes(m.data)
        except PacketError as e:
            return ABORT, ST[e.status], None
