"""Cross-check the C oracle against the independent Python restatement on
seeded edge-case batches, and the synthetic generators against both."""
import numpy as np
import pytest

import oracle_lib
import pyref
from capsule_amd import _native as N
from capsule_amd import synth

ALL = N.F_ACCEPT_ALL | N.F_CSUM_IP | N.F_CSUM_L4 | N.F_FLOW_HASH


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fuzz_oracle_vs_pyref(seed):
    arena, off, ln = synth.fuzz(300, seed=seed)
    for flags in (ALL, N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_CSUM_L4, N.F_ACCEPT_V6 | N.F_ACCEPT_TCP | 0x70,
                  ALL | N.F_ACCEPT_ICMP, N.F_ACCEPT_ICMP | 0x70, N.F_ACCEPT_V4 | N.F_ACCEPT_ICMP | 0x70):
        meta, csum, h, _ = oracle_lib.parse_batch(arena, off, ln, flags, fields=False)
        for i in range(len(off)):
            fr = bytes(arena[off[i] : off[i] + ln[i]])
            st, m, ipc, l4c, hh = pyref.parse(fr, flags)
            assert int(meta[i]) == (m | st), i
            assert int(csum[i]) == (ipc | l4c << 16), i
            assert int(h[i]) == hh, i


def test_fuzz_covers_every_status():
    arena, off, ln = synth.fuzz(2000, seed=7)
    seen = set()
    for flags in (ALL, N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | 0x70, N.F_ACCEPT_V6 | N.F_ACCEPT_TCP | 0x70,
                  N.F_ACCEPT_ICMP | 0x70):
        meta, _, _, _ = oracle_lib.parse_batch(arena, off, ln, flags, fields=False)
        seen |= set((meta & 0xFF).tolist())
    for s in ("OK", "ETH_BAD_OFFSET", "ETH_OUT_OF_BUFFER", "NOT_IPV4", "NOT_IPV6", "NOT_IP",
              "L3_OUT_OF_BUFFER", "NOT_UDP", "NOT_TCP", "NOT_L4", "L4_OUT_OF_BUFFER",
              "NOT_ICMPV4", "NOT_ICMPV6"):
        assert N.PKT[s] in seen, s


@pytest.mark.parametrize("gen", ["uniform64", "uniform_vlan", "imix", "nat64"])
def test_generators_are_reconciled(gen):
    """Synthetic packets are internally consistent like the proptest strategies
    (strategy.rs:395-397): every layer parses and every checksum verifies."""
    if gen == "uniform64":
        a, o, l = synth.uniform(4096)
    elif gen == "uniform_vlan":
        a, o, l = synth.uniform(4096, kind=synth.V6_TCP, frame_len=300, vlan=2, slot=320)
    elif gen == "imix":
        a, o, l = synth.imix(8192, vlan_frac=0.2)
    else:
        a, o, l = synth.nat64_stream(4096, n_keys=100)
    meta, csum, h, fl = oracle_lib.parse_batch(a, o, l, ALL, fields=True)
    assert (meta & 0xFF == 0).all()
    assert (meta & N.META_L4_CSUM_OK).all()
    v4 = ((meta >> 16) & 3) == N.L3_IPV4
    assert (meta[v4] & N.META_IP_CSUM_OK).all()
    rec = fl.view(np.dtype(N.HDR_RECORD_FIELDS)).reshape(-1)
    assert (rec["ip_length"][v4] == (l[v4] - rec["eth_len"][v4])).all()


def test_multi_parse_udp_counts():
    a, o, l = synth.uniform(1000)
    assert oracle_lib.lib().or_multi_parse_udp(a.ctypes.data, o.ctypes.data, l.ctypes.data, 1000) == 1000
    a, o, l = synth.uniform(1000, kind=synth.V4_TCP, frame_len=64)
    assert oracle_lib.lib().or_multi_parse_udp(a.ctypes.data, o.ctypes.data, l.ctypes.data, 1000) == 0


def test_oracle_under_sanitizers():
    """Run the oracle's parse and nat64 on edge cases under ASan+UBSan in a
    subprocess (the sanitizer runtime must be preloaded into a fresh python)."""
    import os
    import subprocess
    import sys

    san = oracle_lib.ORACLE_DIR / "liboracle_san.so"
    subprocess.run(["make", "-C", str(oracle_lib.ORACLE_DIR), "liboracle_san.so"], check=True,
                   stdout=subprocess.DEVNULL)
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True,
                          text=True).stdout.strip()
    ubsan = subprocess.run(["gcc", "-print-file-name=libubsan.so"], capture_output=True,
                           text=True).stdout.strip()
    code = (
        "import sys; sys.path.insert(0, 'tests'); sys.path.insert(0, '.');"
        "import oracle_lib as o; o._lib = o.load('liboracle_san.so');"
        "from capsule_amd import synth;"
        "a, off, ln = synth.fuzz(400, seed=11); o.parse_batch(a, off, ln, 0x7f);"
        "a, off, ln = synth.nat64_stream(300, n_keys=50, drop_frac=0.2);"
        "pm = o.PortMap(); pm.nat_6to4(a, off, ln); print('clean')"
    )
    env = dict(os.environ, LD_PRELOAD=f"{asan} {ubsan}", ASAN_OPTIONS="detect_leaks=0",
               UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([sys.executable, "-c", code], cwd=str(oracle_lib.ROOT), env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "clean" in r.stdout, r.stderr[-2000:]


def test_oracle_nat64_4to6_drops_unknown_ports():
    """4to6 before any 6to4: ADDR_MAP is empty, every TCP frame is DROP
    (examples/nat64/main.rs:113-114); non-IPv4 frames ABORT."""
    a, o, l = synth.uniform(200, kind=synth.V4_TCP, frame_len=128, seed=5)
    pm = oracle_lib.PortMap()
    out, olen, disp, st = pm.nat_4to6(a, o, l, o + np.uint32(0), len(a) + 64)
    tcp_ok = disp != N.ABORT
    assert (disp[tcp_ok] == N.DROP).all()
    a6, o6, l6 = synth.uniform(50, kind=synth.V6_TCP, frame_len=128, seed=6)
    _, _, disp6, st6 = pm.nat_4to6(a6, o6, l6, o6, len(a6) + 64)
    assert (disp6 == N.ABORT).all() and (st6 == N.PKT["NOT_IPV4"]).all()


def test_oracle_nat64_round_trip():
    """6to4 then 4to6 of reply frames in the oracle alone: each reply goes back
    to the original v6 source / port from 64:ff9b::<v4 src>, checksums valid."""
    import nat64_replies

    rng = np.random.default_rng(3)
    pm = oracle_lib.PortMap()
    a, o, l = synth.nat64_stream(500, n_keys=80, seed=9)
    out, olen, disp, _ = pm.nat_6to4(a, o, l)
    assert (disp == N.ACT).all()
    frames = nat64_replies.replies(out, o, olen, disp, rng, junk=0.0)
    ra, ro, rl = synth.pack_frames(frames)
    out_off = (ro + np.arange(len(ro), dtype=np.uint64) * 64).astype(np.uint32)
    back, blen, bdisp, _ = pm.nat_4to6(ra, ro, rl, out_off, len(ra) + 64 * len(ro) + 64)
    assert (bdisp == N.ACT).all() and (blen == rl + 20).all()
    fr = [bytes(back[int(s):int(s) + int(n)]) for s, n in zip(out_off, blen)]
    ba, bo, bl = synth.pack_frames(fr)
    meta, _, _, fl = oracle_lib.parse_batch(ba, bo, bl, 0x7F, fields=True)
    assert (meta & 0xFF == 0).all() and (meta & N.META_L4_CSUM_OK).all()
    rec = fl.view(np.dtype(N.HDR_RECORD_FIELDS)).reshape(-1)
    a2 = a.reshape(-1, 256)
    for j, f in enumerate(frames):
        assert bytes(rec["dst_ip"][j]) == bytes(a2[j, 22:38])
        assert int(rec["dst_port"][j]) == int.from_bytes(bytes(a2[j, 54:56]), "big")
        k = {0x8100: 1, 0x88A8: 2}.get(int.from_bytes(f[12:14], "big"), 0)
        assert bytes(rec["src_ip"][j]) == bytes.fromhex("0064ff9b") + bytes(8) + f[26 + 4 * k:30 + 4 * k]
    # junk replies: oracle must classify every frame without crashing
    frames = nat64_replies.replies(out, o, olen, disp, rng, junk=1.0)
    ra, ro, rl = synth.pack_frames(frames)
    out_off = (ro + np.arange(len(ro), dtype=np.uint64) * 64).astype(np.uint32)
    _, _, jd, _ = pm.nat_4to6(ra, ro, rl, out_off, len(ra) + 64 * len(ro) + 64)
    assert {N.ACT, N.DROP, N.ABORT} <= set(jd.tolist())


def test_oracle_group_by_is_stable_partition():
    rng = np.random.default_rng(8)
    for n, g in ((0, 3), (1, 1), (5000, 4), (5000, 64)):
        key = rng.integers(0, 70, n, dtype=np.uint8)
        idx, off = oracle_lib.group_by(key, g)
        arm = np.minimum(key, g - 1)
        ref = np.argsort(arm, kind="stable")
        assert (idx == ref).all()
        assert (off == np.concatenate([[0], np.cumsum(np.bincount(arm, minlength=g))])).all()


def test_oracle_group_by_meta_class_arms():
    """CGPU_KEY_META_CLASS: v4/UDP, v4/TCP, v6/UDP, v6/TCP, then everything
    else -- failed parses and ICMP (which is neither Udp nor Tcp)."""
    def meta(status, l3, l4):
        return status | (l3 << 16) | (l4 << 18)

    m = np.array([meta(0, 1, 1), meta(0, 1, 2), meta(0, 2, 1), meta(0, 2, 2),
                  meta(0, 1, 3), meta(0, 2, 3), meta(8, 1, 0), meta(0, 1, 1)], np.uint32)
    idx, off = oracle_lib.group_by(m, 5, N.KEY_META_CLASS)
    assert off.tolist() == [0, 2, 3, 4, 5, 8]
    assert idx.tolist() == [0, 7, 1, 2, 3, 4, 5, 6]


def _nat64_6to4_inputs(rng, m):
    """IPv6 frames for 6to4: the bench's stream shape with UDP drops, VLAN
    tags, hop limits 0 and 1 (the u8 wrap), truncations at every layer,
    non-IPv6 frames and frames near the 2048-B data room."""
    a, o, l = synth.nat64_stream(m, n_keys=m // 8, drop_frac=0.1, seed=int(rng.integers(1 << 30)))
    frames = [bytes(a[int(s):int(s) + int(n)]) for s, n in zip(o, l)]
    for vlan in (1, 2):
        for L in (74 + 4 * vlan, 75 + 4 * vlan, 200, 1500):
            frames += [bytes(x) for x in synth.build_frames(rng, 20, synth.V6_TCP, L, vlan)]
    for f in list(frames[:200]):
        g = bytearray(f)
        r = rng.random()
        if r < 0.3:
            g[21] = int(rng.integers(0, 2))  # hop limit 0 / 1 (no VLAN in the stream)
        elif r < 0.7:
            g = g[: int(rng.integers(0, len(g) + 1))]  # truncated anywhere, down to 0 bytes
        else:
            g[12:14] = b"\x08\x00"  # not an IPv6 packet
        frames.append(bytes(g))
    frames += [bytes(x) for x in synth.build_frames(rng, 5, synth.V6_TCP, 2040, 0)]
    return frames


def test_nat64_oracle_vs_pyref():
    """The C oracle's nat_6to4 / nat_4to6 against an independent Python
    restatement (tests/pyref_nat64.py), byte for byte: every disposition,
    status and ACT frame, NEXT_PORT and the map size, through a 6to4 pass
    over fuzzed IPv6 frames, a second 6to4 pass (committed keys), and the
    replies -- with unknown ports, UDP, fragments, truncations, VLAN tags,
    TTL 0 and frames at the extend tailroom limit -- through 4to6."""
    import nat64_replies
    import pyref_nat64

    rng = np.random.default_rng(21)
    pm = oracle_lib.PortMap()
    ref = pyref_nat64.Nat64()

    def check(direction, frames, out_off=None, out_size=None):
        a, o, l = synth.pack_frames(frames)
        if direction == "6to4":
            out, olen, disp, st = pm.nat_6to4(a, o, l)
            oo = o
        else:
            out, olen, disp, st = pm.nat_4to6(a, o, l, out_off(o), out_size(a, o))
            oo = out_off(o)
        for i, f in enumerate(frames):
            d, s, g = getattr(ref, "nat_" + direction)(f)
            assert (int(disp[i]), int(st[i])) == (d, s), (direction, i, len(f))
            if d == N.ACT:
                got = bytes(out[int(oo[i]):int(oo[i]) + int(olen[i])])
                assert got == g, (direction, i)
        assert pm.next_port() == ref.next_port and pm.size() == len(ref.port_map)
        return out, o, olen, disp

    frames = _nat64_6to4_inputs(rng, 3000)
    out, o, olen, disp = check("6to4", frames)
    check("6to4", frames)  # every key committed now
    assert {N.ACT, N.DROP, N.ABORT} <= set(disp.tolist())
    replies = nat64_replies.replies(out, o, olen, disp, rng, junk=0.4)
    # replies near the tailroom limit (extend(40) needs 40 < tailroom after
    # shrink(20): frames of 2027 B fit in a 2048-B room, 2028 B do not)
    base = next(f for f in replies if ref.nat_4to6(f)[0] == N.ACT)
    for L in (2026, 2027, 2028, 2029):
        g = bytearray(base + bytes(L - len(base)))
        k = {0x8100: 1, 0x88A8: 2}.get(int.from_bytes(g[12:14], "big"), 0)
        g[14 + 4 * k + 2:14 + 4 * k + 4] = (L - 14 - 4 * k).to_bytes(2, "big")
        replies.append(bytes(g))
    _, _, _, d4 = check("4to6", replies,
                        out_off=lambda o: (o + np.arange(len(o), dtype=np.uint64) * 64).astype(np.uint32),
                        out_size=lambda a, o: len(a) + 64 * len(o) + 64)
    assert {N.ACT, N.DROP, N.ABORT} <= set(d4.tolist())
    assert [ref.nat_4to6(f)[:2] for f in replies[-4:]] == [
        (N.ACT, 0), (N.ACT, 0), (N.ABORT, N.PKT["NOT_RESIZED"]), (N.ABORT, N.PKT["NOT_RESIZED"])]
