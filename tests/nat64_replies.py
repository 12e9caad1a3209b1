"""Reply-frame generator for the nat64 4to6 tests (test infrastructure):
IPv4/TCP frames answering a batch of 6to4 outputs, addressed to the gateway
ports the port map assigned (examples/nat64/main.rs:86-118 reads them)."""
import numpy as np

from capsule_amd import _native as N


def replies(out, out_off, out_len, disp, rng, junk=0.25, max_payload=300):
    """IPv4/TCP reply frames to the 6to4 output frames (dst port = the gateway
    port, so ADDR_MAP hits), plus junk: unknown ports, UDP, fragments,
    truncations, VLAN tags, TTL 0.  Payloads are 0 .. max_payload - 1 B."""
    import struct

    import pyref

    frames = []
    for i in np.nonzero(disp == N.ACT)[0]:
        f = bytes(out[int(out_off[i]) : int(out_off[i]) + int(out_len[i])])
        k = {0x8100: 1, 0x88A8: 2}.get(int.from_bytes(f[12:14], "big"), 0)
        o = 14 + 4 * k
        v4_src, v4_dst = f[o + 12 : o + 16], f[o + 16 : o + 20]
        sport, dport = struct.unpack(">HH", f[o + 20 : o + 24])
        vlan = int(rng.integers(0, 3))
        eth = bytes(rng.integers(0, 256, 12, dtype=np.uint8))
        eth += {0: b"", 1: b"\x81\x00\x00\x07", 2: b"\x88\xa8\x00\x01\x81\x00\x00\x02"}[vlan]
        payload = bytes(rng.integers(0, 256, int(rng.integers(0, max_payload)), dtype=np.uint8))
        ttl = int(rng.integers(0, 256))
        proto, flags_frag, gw = 6, 0x4000 if rng.random() < 0.5 else 0, sport
        r = rng.random()
        if r < junk * 0.3:
            gw = int(rng.integers(0, 65536))  # unknown port (or a hit by chance)
        elif r < junk * 0.5:
            proto = 17
        elif r < junk * 0.7:
            flags_frag = 0x2000 | int(rng.integers(0, 8))  # fragment
        tcp = struct.pack(">HHIIBBHHH", dport, gw, int(rng.integers(0, 2**32)),
                          int(rng.integers(0, 2**32)), 0x50, 0x18, 512, 0, 0) + payload
        ip = bytearray(struct.pack(">BBHHHBBH4s4s", 0x45, int(rng.integers(0, 256)),
                                   20 + len(tcp), 7, flags_frag, ttl, proto, 0, v4_src, v4_dst))
        ph = pyref.fold(sum(struct.unpack(">HHHH", v4_src + v4_dst)) + 6 + len(tcp))
        tcp = bytearray(tcp)
        tcp[16:18] = pyref.compute(ph, bytes(tcp)).to_bytes(2, "big")
        ip[10:12] = pyref.compute(0, bytes(ip)).to_bytes(2, "big")
        fr = eth + b"\x08\x00" + bytes(ip) + bytes(tcp)
        if rng.random() < junk * 0.2:
            fr = fr[: int(rng.integers(0, len(fr)))]
        frames.append(fr)
    return frames
