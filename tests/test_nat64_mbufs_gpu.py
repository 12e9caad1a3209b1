"""examples/nat64 over rte_mbuf bursts (cgpu_nat64_mbufs, the DPDK seam of
SURVEY §8 f2 with egress): the device reads the frames from a registered
DPDK-style mempool, rewrites them and writes every ACT frame back into its own
mbuf.  Checked bit-exactly against the oracle's nat_6to4 / nat_4to6 on the
same frames: dispositions, statuses, and for every mbuf its data_len, pkt_len
and frame bytes (Mbuf::shrink / extend keep data_off, mbuf.rs:225-270);
DROP / ABORT mbufs must be untouched."""
import mmap

import numpy as np
import pytest

import oracle_lib
from capsule_amd import _native as N
from capsule_amd import packets, synth

pytestmark = pytest.mark.gpu


def _u16(mem, at):
    return mem[at].astype(np.int64) | (mem[at + 1].astype(np.int64) << 8)


def _u32(mem, at):
    return sum(mem[at + b].astype(np.int64) << (8 * b) for b in range(4))


def _check_mbufs(mem, mbufs, a, o, l, out, out_off, olen, disp):
    """Every mbuf against the oracle: ACT -> the rewritten frame, else untouched."""
    objs = (mbufs - np.uint64(mem.ctypes.data)).astype(np.int64)
    dlen, plen = _u16(mem, objs + 40), _u32(mem, objs + 36)
    doff = _u16(mem, objs + 16)
    data = objs + 128 + doff
    act = disp == N.ACT
    want = np.where(act, olen.astype(np.int64), l.astype(np.int64))
    assert (dlen == want).all(), np.nonzero(dlen != want)[0][:8]
    assert (plen == want).all()
    for i in range(len(mbufs)):
        d, L = int(data[i]), int(want[i])
        if act[i]:
            s = int(out_off[i])
            assert (mem[d : d + L] == out[s : s + L]).all(), f"frame {i}"
        else:
            s = int(o[i])
            assert (mem[d : d + L] == a[s : s + L]).all(), f"untouched frame {i}"


def _pool(ctx, a, o, l, room):
    mem, mbufs = synth.mbuf_pool(a, o, l, room=room)
    return mem, mbufs, packets.HostRegion.of(ctx, mem)


def test_nat64_mbufs_6to4_then_4to6_replies(ctx):
    a, o, l = synth.nat64_stream(20_000, n_keys=3000, drop_frac=0.05, seed=41)
    mem, mbufs, reg = _pool(ctx, a, o, l, 2048)
    gw = packets.Nat64Gateway(ctx, capacity_log2=14)
    pm = oracle_lib.PortMap()
    try:
        disp, st = gw.nat_mbufs(mbufs, "6to4")
        out, olen, odisp, ost = pm.nat_6to4(a, o, l)
        assert (disp == odisp).all() and (st == ost).all()
        assert (odisp == N.ACT).sum() > 15_000 and (odisp != N.ACT).any()
        _check_mbufs(mem, mbufs, a, o, l, out, o, olen, disp)
        assert gw.next_port() == pm.next_port()
    finally:
        reg.close()

    keep = np.nonzero(odisp == N.ACT)[0]
    ra, ro, rl = synth.nat64_replies(out, o[keep], olen[keep])
    mem2, mb2, reg2 = _pool(ctx, ra, ro, rl, 2048)
    try:
        disp6, st6 = gw.nat_mbufs(mb2, "4to6")
        out6, olen6, odisp6, ost6 = pm.nat_4to6(ra, ro, rl, ro, len(ra))
        assert (disp6 == odisp6).all() and (st6 == ost6).all() and (odisp6 == N.ACT).all()
        _check_mbufs(mem2, mb2, ra, ro, rl, out6, ro, olen6, disp6)
    finally:
        reg2.close()
        gw.close()


@pytest.mark.parametrize("extra", [20, 21])
def test_nat64_mbufs_4to6_tailroom(ctx, extra):
    """extend(20) needs 20 < tailroom (mbuf.rs:228): with exactly 20 bytes of
    room every reply is ABORT / NOT_RESIZED and its mbuf untouched; with 21
    every reply is rewritten."""
    a, o, l = synth.nat64_stream(2_000, n_keys=200, drop_frac=0.0, seed=42)
    gw = packets.Nat64Gateway(ctx, capacity_log2=12)
    pm = oracle_lib.PortMap()
    b = packets.PacketBatch.from_numpy(a, o, l, "cuda:0")
    gw.nat_6to4(b)  # populate the port map (the device and the oracle alike)
    out, olen, odisp, _ = pm.nat_6to4(a, o, l)
    keep = np.nonzero(odisp == N.ACT)[0]
    ra, ro, rl = synth.nat64_replies(out, o[keep], olen[keep])
    room = int(rl.max()) + extra
    assert (rl == rl.max()).all()
    mem, mbufs, reg = _pool(ctx, ra, ro, rl, room)
    try:
        disp, st = gw.nat_mbufs(mbufs, "4to6")
        out6, olen6, odisp6, ost6 = pm.nat_4to6(ra, ro, rl, ro, len(ra))
        if extra <= 20:
            assert (disp == N.ABORT).all() and (st == N.PKT["NOT_RESIZED"]).all()
        else:
            assert (disp == odisp6).all() and (st == ost6).all() and (disp == N.ACT).all()
        _check_mbufs(mem, mbufs, ra, ro, rl, out6, ro, olen6, disp)
    finally:
        reg.close()
        gw.close()


def test_nat64_mbufs_rejects_unregistered_and_empty(ctx):
    gw = packets.Nat64Gateway(ctx, capacity_log2=8)
    a, o, l = synth.nat64_stream(64, n_keys=8, seed=43)
    mem, mbufs, reg = _pool(ctx, a, o, l, 2048)
    try:
        d, s = gw.nat_mbufs(mbufs[:0], "6to4")
        assert d.size == 0
        bad = mbufs.copy()
        bad[5] = np.uint64(0x1000)  # outside every registered region
        with pytest.raises(N.CgpuError):
            gw.nat_mbufs(bad, "6to4")
    finally:
        reg.close()
        gw.close()


def test_nat64_mbufs_bad_pointer_changes_nothing(ctx):
    """A bad mbuf fails the call before anything is rewritten: every mbuf and
    the port map are as they were -- for a one-chunk burst, for a burst of
    two chunks (2^20 mbufs each) whose bad pointer is in the last one, and
    for a frame that runs past its own buffer (data_off + data_len >
    buf_len).  The intact burst then goes through."""
    gw = packets.Nat64Gateway(ctx, capacity_log2=12)
    a, o, l = synth.nat64_stream(4096, n_keys=300, seed=44)
    mem, mbufs, reg = _pool(ctx, a, o, l, 2048)
    before = mem.copy()
    try:
        for burst in (mbufs.copy(), np.tile(mbufs, 257)):
            assert len(burst) in (4096, 4096 * 257)
            burst[-1] = np.uint64(0x1000)  # outside every registered region
            with pytest.raises(N.CgpuError) as e:
                gw.nat_mbufs(burst, "6to4")
            assert e.value.code == N.EINVAL
            assert (mem == before).all()
            assert gw.next_port() == 1025 and gw.size() == 0
        ob = int(mbufs[7]) - mem.ctypes.data
        mem[ob + 40: ob + 42] = np.frombuffer(np.uint16(2049).tobytes(), np.uint8)  # room 2048
        with pytest.raises(N.CgpuError) as e:
            gw.nat_mbufs(mbufs, "6to4")
        assert e.value.code == N.EINVAL
        mem[ob + 40: ob + 42] = before[ob + 40: ob + 42]
        assert (mem == before).all() and gw.next_port() == 1025 and gw.size() == 0
        disp, st = gw.nat_mbufs(mbufs, "6to4")
        out, olen, odisp, ost = oracle_lib.PortMap().nat_6to4(a, o, l)
        assert (disp == odisp).all() and (st == ost).all()
        _check_mbufs(mem, mbufs, a, o, l, out, o, olen, disp)
    finally:
        reg.close()
        gw.close()


def test_nat64_mbufs_custom_data_room(ctx):
    """A mempool with a 4096-B data room: 3000-B IPv6 frames (longer than
    the 2176-B slots the gather assumes, so its arena grows) through 6to4,
    and their 2980-B replies through 4to6, whose extend(20) fits the mbufs'
    real tailroom -- a device batch, modelled on DPDK's 2048-B room, would
    abort them (NotResized).  Oracle with the same data room."""
    room = 4096
    a, o, l = synth.nat64_stream(600, frame_len=3000, n_keys=40, seed=45)
    gw = packets.Nat64Gateway(ctx, capacity_log2=10)
    pm = oracle_lib.PortMap()
    mem, mbufs, reg = _pool(ctx, a, o, l, room)
    try:
        with oracle_lib.data_room(room):
            disp, st = gw.nat_mbufs(mbufs, "6to4")
            out, olen, odisp, ost = pm.nat_6to4(a, o, l)
        assert (odisp == N.ACT).all() and (disp == odisp).all() and (st == ost).all()
        _check_mbufs(mem, mbufs, a, o, l, out, o, olen, disp)
    finally:
        reg.close()
    ra, ro, rl = synth.nat64_replies(out, o, olen)
    mem2, mb2, reg2 = _pool(ctx, ra, ro, rl, room)
    try:
        with oracle_lib.data_room(room):
            disp6, st6 = gw.nat_mbufs(mb2, "4to6")
            out6, olen6, odisp6, ost6 = pm.nat_4to6(ra, ro, rl, ro + 0, len(ra))
        assert (odisp6 == N.ACT).all() and (olen6 == 3000).all()
        assert (disp6 == odisp6).all() and (st6 == ost6).all()
        _check_mbufs(mem2, mb2, ra, ro, rl, out6, ro, olen6, disp6)
    finally:
        reg2.close()
        gw.close()


def _set_lens(mem, mbufs, olen, disp):
    """What the caller of cgpu_nat64_frames does: data_len / pkt_len of each
    ACT mbuf := out_len (the Rust combinator's set of data_len)."""
    objs = (mbufs - np.uint64(mem.ctypes.data)).astype(np.int64)
    act = disp == N.ACT
    v = olen.astype(np.int64)
    for b, off in ((0, 40), (1, 41)):
        mem[objs[act] + off] = ((v[act] >> (8 * b)) & 0xFF).astype(np.uint8)
    for b in range(4):
        mem[objs[act] + 36 + b] = ((v[act] >> (8 * b)) & 0xFF).astype(np.uint8)


def _tailroom(mem, mbufs):
    objs = (mbufs - np.uint64(mem.ctypes.data)).astype(np.int64)
    return (_u16(mem, objs + 54) - _u16(mem, objs + 16) - _u16(mem, objs + 40)).astype(np.uint16)


@pytest.mark.parametrize("extra", [20, 21])
def test_nat64_frames_both_directions(ctx, extra):
    """cgpu_nat64_frames: the same rewrite from (data_address, data_len)
    pairs; the device touches only the frames, the caller sets data_len from
    out_len, and then every mbuf matches the oracle as on the mbuf path.  The
    4to6 replies sit in mbufs with exactly `extra` bytes of room past them."""
    a, o, l = synth.nat64_stream(20_000, n_keys=3000, drop_frac=0.05, seed=47)
    mem, mbufs, reg = _pool(ctx, a, o, l, 2048)
    gw = packets.Nat64Gateway(ctx, capacity_log2=14)
    pm = oracle_lib.PortMap()
    try:
        addrs, lens = synth.mbuf_frames(mem, mbufs)
        olen_g, disp, st = gw.nat_frames(addrs, lens, direction="6to4")
        out, olen, odisp, ost = pm.nat_6to4(a, o, l)
        assert (disp == odisp).all() and (st == ost).all()
        act = odisp == N.ACT
        assert (olen_g[act] == olen[act]).all() and (olen_g[~act] == 0).all()
        objs = (mbufs - np.uint64(mem.ctypes.data)).astype(np.int64)
        assert (_u16(mem, objs + 40) == l).all()  # no mbuf header written by the device
        _set_lens(mem, mbufs, olen_g, disp)
        _check_mbufs(mem, mbufs, a, o, l, out, o, olen, disp)
        assert gw.next_port() == pm.next_port()
    finally:
        reg.close()

    keep = np.nonzero(odisp == N.ACT)[0]
    ra, ro, rl = synth.nat64_replies(out, o[keep], olen[keep])
    mem2, mb2, reg2 = _pool(ctx, ra, ro, rl, int(rl.max()) + extra)
    try:
        addrs, lens = synth.mbuf_frames(mem2, mb2)
        tr = _tailroom(mem2, mb2)
        olen_g, disp6, st6 = gw.nat_frames(addrs, lens, tr, direction="4to6")
        out6, olen6, odisp6, ost6 = pm.nat_4to6(ra, ro, rl, ro, len(ra))
        short = tr <= 20
        assert (disp6[short] == N.ABORT).all() and (st6[short] == N.PKT["NOT_RESIZED"]).all()
        assert (disp6[~short] == odisp6[~short]).all() and (st6[~short] == ost6[~short]).all()
        _set_lens(mem2, mb2, olen_g, disp6)
        _check_mbufs(mem2, mb2, ra, ro, rl, out6, ro, olen6, disp6)
    finally:
        reg2.close()
        gw.close()


def test_nat64_egress_range_checked(ctx):
    """The bytes a 4to6 rewrite may grow into are range-checked with the
    frame: a frame that ends 10 B before its registered region does, but
    whose tailroom says 20 more bytes fit, fails the call (frame pairs with a
    caller-supplied tailroom, and rte_mbufs whose buf_len claims the room)
    before anything is written.  With that frame's true tailroom the call
    goes through, and that frame is NotResized."""
    a, o, l = synth.nat64_stream(512, n_keys=64, seed=48)
    gw = packets.Nat64Gateway(ctx, capacity_log2=12)
    pm = oracle_lib.PortMap()
    gw.nat_6to4(packets.PacketBatch.from_numpy(a, o, l, "cuda:0"))
    out, olen, odisp, _ = pm.nat_6to4(a, o, l)
    keep = np.nonzero(odisp == N.ACT)[0]
    ra, ro, rl = synth.nat64_replies(out, o[keep], olen[keep])
    # the pool laid out once to find where its last frame ends, then again
    # `shift` bytes into a page-aligned buffer so that the end + 10 B falls
    # on a page boundary (regions are whole pages)
    scratch, mb0 = synth.mbuf_pool(ra, ro, rl, room=2048)
    a0, l0 = synth.mbuf_frames(scratch, mb0)
    top = int(np.argmax(a0))
    end0 = int(a0[top]) + int(l0[top]) + 10 - scratch.ctypes.data
    page = mmap.PAGESIZE
    shift = -end0 % page
    buf = synth.host_buffer(shift + end0 + page)
    mem, mbufs = synth.mbuf_pool(ra, ro, rl, mem=buf[shift:], room=2048)
    addrs, lens = synth.mbuf_frames(mem, mbufs)
    assert int(np.argmax(addrs)) == top
    end = shift + end0
    assert end % page == 0
    reg = packets.HostRegion(ctx, buf.ctypes.data, end)
    mem = buf
    before = mem.copy()
    try:
        tr = np.full(len(addrs), 100, np.uint16)
        with pytest.raises(N.CgpuError) as e:
            gw.nat_frames(addrs, lens, tr, direction="4to6")
        assert e.value.code == N.EINVAL and (mem == before).all()
        with pytest.raises(N.CgpuError) as e:
            gw.nat_mbufs(mbufs, "4to6")
        assert e.value.code == N.EINVAL and (mem == before).all()
        tr[top] = 10
        olen_g, disp, st = gw.nat_frames(addrs, lens, tr, direction="4to6")
        assert disp[top] == N.ABORT and st[top] == N.PKT["NOT_RESIZED"]
        rest = np.arange(len(addrs)) != top
        assert (disp[rest] == N.ACT).all()
        assert (mem[end - 10:end] == before[end - 10:end]).all()
    finally:
        reg.close()
        gw.close()
