"""rte_mbuf bursts through cgpu_parse_mbufs (the DPDK seam).

A synthetic DPDK-style mempool in host memory (synth.mbuf_pool: 128-B
rte_mbuf headers at the DPDK 19.11 offsets, shuffled objects, 128-B headroom)
is parsed in both ingress modes -- the calling core gathering into pinned
staging, and the device reading the registered mempool over PCIe -- and every
output is compared bit-exactly with the CPU oracle run on the same frames.
"""
import ctypes
import mmap

import numpy as np
import pytest
import torch

import oracle_lib
from capsule_amd import _native as N
from capsule_amd import packets, synth

pytestmark = pytest.mark.gpu

ALL = N.F_ACCEPT_ALL | N.F_CSUM_IP | N.F_CSUM_L4 | N.F_FLOW_HASH
MODES = [N.INGRESS_STAGE, N.INGRESS_ZERO_COPY]


def edge_batch(seed=11):
    """IMIX with VLAN tags, plus empty, truncated and corrupted frames."""
    a, o, l = synth.imix(3000, seed=seed, vlan_frac=0.2)
    rng = np.random.default_rng(seed)
    l = l.copy()
    cut = rng.choice(len(l), 300, replace=False)
    l[cut] = rng.integers(0, 80, 300).astype(np.uint16)  # truncations, 0-length frames
    a = a.copy()
    bad = rng.choice(len(l), 200, replace=False)
    a[o[bad].astype(np.int64) + rng.integers(0, 60, 200)] ^= 0x5A  # corrupted bytes
    return a, o, l


def check(ctx, a, o, l, mbufs, ingress, fields=True):
    gm, gc, gh, gf = packets.parse_mbufs(ctx, mbufs, ALL, ingress, fields=fields)
    om, oc, oh, of = oracle_lib.parse_batch(a, o, l, ALL, fields=fields)
    assert (gm == om).all(), np.nonzero(gm != om)[0][:8]
    assert (gc == oc).all(), np.nonzero(gc != oc)[0][:8]
    assert (gh == oh).all(), np.nonzero(gh != oh)[0][:8]
    if fields:
        assert (gf.view(np.uint8).reshape(len(o), -1) == of).all()


@pytest.mark.parametrize("ingress", MODES)
def test_pageable_mempool_registered_here(ctx, ingress):
    a, o, l = edge_batch()
    mem, mbufs = synth.mbuf_pool(a, o, l)
    reg = packets.HostRegion.of(ctx, mem)  # hipHostRegister
    try:
        check(ctx, a, o, l, mbufs, ingress)
    finally:
        reg.close()


@pytest.mark.parametrize("ingress", MODES)
def test_pinned_mempool(ctx, ingress):
    a, o, l = synth.imix(4096, seed=3)
    stride = (128 + 128 + int(l.max()) + 63) // 64 * 64
    pinned, pool = synth.pinned_buffer(stride * len(o))
    mem, mbufs = synth.mbuf_pool(a, o, l, mem=pool)
    reg = packets.HostRegion.of(ctx, mem)  # already page-locked: mapped only
    try:
        check(ctx, a, o, l, mbufs, ingress, fields=False)
    finally:
        reg.close()


@pytest.mark.parametrize("headroom", [129, 130, 132])
def test_zero_copy_unaligned_frames(ctx, headroom):
    """Frames that do not start on a 16-B (or 4-B) boundary take the
    dword / byte host loads."""
    a, o, l = synth.imix(1500, seed=headroom)
    mem, mbufs = synth.mbuf_pool(a, o, l, headroom=headroom)
    reg = packets.HostRegion.of(ctx, mem)
    try:
        check(ctx, a, o, l, mbufs, N.INGRESS_ZERO_COPY)
    finally:
        reg.close()


def test_zero_copy_two_regions_and_chunking(ctx):
    """Two mempools, bursts interleaving their mbufs; more than one region."""
    a1, o1, l1 = synth.imix(2000, seed=21)
    a2, o2, l2 = synth.uniform(2000, seed=22)
    m1, b1 = synth.mbuf_pool(a1, o1, l1, seed=1)
    m2, b2 = synth.mbuf_pool(a2, o2, l2, seed=2)
    r1 = packets.HostRegion.of(ctx, m1)
    r2 = packets.HostRegion.of(ctx, m2)
    try:
        mb = np.empty(4000, np.uint64)
        mb[0::2], mb[1::2] = b1, b2
        gm, gc, gh, _ = packets.parse_mbufs(ctx, mb, ALL, N.INGRESS_ZERO_COPY)
        om1, oc1, oh1, _ = oracle_lib.parse_batch(a1, o1, l1, ALL, fields=False)
        om2, oc2, oh2, _ = oracle_lib.parse_batch(a2, o2, l2, ALL, fields=False)
        assert (gm[0::2] == om1).all() and (gm[1::2] == om2).all()
        assert (gc[0::2] == oc1).all() and (gc[1::2] == oc2).all()
        assert (gh[0::2] == oh1).all() and (gh[1::2] == oh2).all()
    finally:
        r2.close()
        r1.close()


def test_zero_copy_rejects_unregistered_pointers(ctx):
    a, o, l = synth.imix(256, seed=5)
    mem, mbufs = synth.mbuf_pool(a, o, l)
    # no region registered at all
    with pytest.raises(N.CgpuError) as e:
        packets.parse_mbufs(ctx, mbufs, ALL, N.INGRESS_ZERO_COPY)
    assert e.value.code == N.EINVAL
    reg = packets.HostRegion.of(ctx, mem)
    try:
        # an mbuf pointer outside the region
        other = np.zeros(4096, np.uint8)
        bad = mbufs.copy()
        bad[17] = np.uint64(other.ctypes.data)
        with pytest.raises(N.CgpuError) as e:
            packets.parse_mbufs(ctx, bad, ALL, N.INGRESS_ZERO_COPY)
        assert e.value.code == N.EINVAL
        # a buf_addr pointing outside the region
        ob = int(mbufs[3]) - mem.ctypes.data
        saved = mem[ob:ob + 8].copy()
        mem[ob:ob + 8] = np.frombuffer(np.uint64(other.ctypes.data).tobytes(), np.uint8)
        with pytest.raises(N.CgpuError):
            packets.parse_mbufs(ctx, mbufs, ALL, N.INGRESS_ZERO_COPY)
        mem[ob:ob + 8] = saved
        check(ctx, a, o, l, mbufs, N.INGRESS_ZERO_COPY, fields=False)  # intact again
    finally:
        reg.close()


def test_stage_rejects_null_mbuf(ctx):
    a, o, l = synth.imix(64, seed=6)
    mem, mbufs = synth.mbuf_pool(a, o, l)
    bad = mbufs.copy()
    bad[5] = 0
    with pytest.raises(N.CgpuError):
        packets.parse_mbufs(ctx, bad, ALL, N.INGRESS_STAGE)
    assert N.lib().cgpu_last_error() == N.EINVAL


def test_register_unregister_bookkeeping(ctx):
    L = N.lib()
    buf = np.zeros(1 << 16, np.uint8)
    assert L.cgpu_host_unregister(ctx.handle, ctypes.c_void_p(buf.ctypes.data)) == N.EINVAL
    bufs = [synth.host_buffer(4096) for _ in range(17)]
    regs = []
    try:
        for b in bufs[:16]:
            regs.append(packets.HostRegion.of(ctx, b))
        with pytest.raises(N.CgpuError):  # 16 regions per context
            packets.HostRegion.of(ctx, bufs[16])
    finally:
        for r in regs:
            r.close()


def test_empty_burst(ctx):
    gm, gc, gh, _ = packets.parse_mbufs(ctx, np.zeros(0, np.uint64), ALL, N.INGRESS_ZERO_COPY)
    assert len(gm) == 0


@pytest.mark.parametrize("ingress", MODES)
def test_jumbo_mempool(ctx, ingress):
    """A 9000-B data room with 9000-B frames: each frame needs more than the
    2176-B slot the zero-copy gather sizes its arena for, so the arena grows
    and the chunk is redone; results bit-exact either way."""
    a, o, l = synth.uniform(700, kind=synth.V4_UDP, frame_len=9000, slot=9024, seed=6)
    mem, mbufs = synth.mbuf_pool(a, o, l, room=9000)
    reg = packets.HostRegion.of(ctx, mem)
    try:
        check(ctx, a, o, l, mbufs, ingress, fields=False)
    finally:
        reg.close()


def test_zero_copy_rejects_frame_past_its_buffer(ctx):
    """data_off + data_len > buf_len is no valid mbuf: the call fails."""
    a, o, l = synth.imix(128, seed=8)
    mem, mbufs = synth.mbuf_pool(a, o, l, room=2048)
    reg = packets.HostRegion.of(ctx, mem)
    try:
        ob = int(mbufs[9]) - mem.ctypes.data
        saved = mem[ob + 40: ob + 42].copy()
        mem[ob + 40: ob + 42] = np.frombuffer(np.uint16(2049).tobytes(), np.uint8)
        with pytest.raises(N.CgpuError) as e:
            packets.parse_mbufs(ctx, mbufs, ALL, N.INGRESS_ZERO_COPY)
        assert e.value.code == N.EINVAL
        mem[ob + 40: ob + 42] = saved
        check(ctx, a, o, l, mbufs, N.INGRESS_ZERO_COPY, fields=False)
    finally:
        reg.close()


@pytest.mark.parametrize("ingress", MODES)
def test_frames_pairs_match_oracle(ctx, ingress):
    """cgpu_parse_frames: the same burst handed over as (data_address,
    data_len) pairs; zero-copy reads the frames alone from the registered
    mempool (no mbuf header)."""
    a, o, l = edge_batch(seed=23)
    mem, mbufs = synth.mbuf_pool(a, o, l)
    addrs, lens = synth.mbuf_frames(mem, mbufs)
    assert (lens == l).all()
    reg = packets.HostRegion.of(ctx, mem)
    try:
        gm, gc, gh, gf = packets.parse_frames(ctx, addrs, lens, ALL, ingress, fields=True)
    finally:
        reg.close()
    om, oc, oh, of = oracle_lib.parse_batch(a, o, l, ALL, fields=True)
    assert (gm == om).all(), np.nonzero(gm != om)[0][:8]
    assert (gc == oc).all() and (gh == oh).all()
    assert (gf.view(np.uint8).reshape(len(o), -1) == of).all()


def test_frames_zero_copy_rejects_unregistered(ctx):
    """A frame address outside every registered region fails the call and is
    never read through."""
    a, o, l = synth.imix(512, seed=5)
    mem, mbufs = synth.mbuf_pool(a, o, l)
    addrs, lens = synth.mbuf_frames(mem, mbufs)
    other = np.zeros(4096, np.uint8)
    addrs = addrs.copy()
    addrs[100] = np.uint64(other.ctypes.data)
    reg = packets.HostRegion.of(ctx, mem)
    try:
        with pytest.raises(N.CgpuError):
            packets.parse_frames(ctx, addrs, lens, ALL, N.INGRESS_ZERO_COPY)
        # the context stays usable
        addrs[100] = synth.mbuf_frames(mem, mbufs)[0][100]
        gm = packets.parse_frames(ctx, addrs, lens, ALL, N.INGRESS_ZERO_COPY)[0]
        assert (gm == oracle_lib.parse_batch(a, o, l, ALL)[0]).all()
    finally:
        reg.close()



def test_register_refuses_partial_pages_overlap_and_straddles(ctx):
    """Whole pages only; no two regions of a context share a page; an
    already page-locked range is mapped only when one pinned allocation
    holds all of it."""
    L = ctx.L
    page = mmap.PAGESIZE
    buf = synth.host_buffer(8 * page)
    base = buf.ctypes.data
    for b, n in ((base + 64, 4 * page), (base, 4 * page + 64), (base, 100)):
        assert L.cgpu_host_register(ctx.handle, ctypes.c_void_p(b), n) == N.EINVAL
    with packets.HostRegion(ctx, base, 4 * page, mem=buf):
        assert L.cgpu_host_register(ctx.handle, ctypes.c_void_p(base + 2 * page), 4 * page) == N.EINVAL
        assert L.cgpu_host_register(ctx.handle, ctypes.c_void_p(base), 4 * page) == N.EINVAL
        with packets.HostRegion(ctx, base + 4 * page, 4 * page):  # the next pages: fine
            pass
    t, pool = synth.pinned_buffer(4 * page)
    pb = pool.ctypes.data
    with packets.HostRegion.of(ctx, pool):  # one pinned allocation: mapped
        pass
    with packets.HostRegion(ctx, pb + page, 2 * page):  # inside it: mapped
        pass
    # a range running past the pinned allocation is refused
    big = 1 << 22
    assert L.cgpu_host_register(ctx.handle, ctypes.c_void_p(pb), big) == N.EINVAL
    del t, pool


def test_register_unregister_free_then_new_mapping_same_range(ctx):
    """The fault of round 5: a pinned mapping must not
    outlive its registration.  A page-aligned pool is registered, read
    zero-copy, unregistered and unmapped; new memory is mapped over exactly
    the same range with new bytes; a pageable host-to-device copy of it and a
    zero-copy read after registering it again must both see the new bytes."""
    libc = ctypes.CDLL(None, use_errno=True)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                          ctypes.c_int, ctypes.c_long]
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    PROT_RW, MAP_PA, MAP_FIXED_NOREPLACE = 0x3, 0x22, 0x100000
    a, o, l = synth.imix(2048, seed=61)
    stride = (128 + 128 + int(l.max()) + 63) // 64 * 64
    size = (stride * len(o) + mmap.PAGESIZE - 1) // mmap.PAGESIZE * mmap.PAGESIZE
    p = libc.mmap(None, size, PROT_RW, MAP_PA, -1, 0)
    assert p not in (None, ctypes.c_void_p(-1).value)
    mem = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(p))
    mem, mbufs = synth.mbuf_pool(a, o, l, mem=mem)
    with packets.HostRegion(ctx, p, size):
        check(ctx, a, o, l, mbufs, N.INGRESS_ZERO_COPY, fields=False)
    del mem
    assert libc.munmap(p, size) == 0
    q = libc.mmap(p, size, PROT_RW, MAP_PA | MAP_FIXED_NOREPLACE, -1, 0)
    if q != p:
        if q not in (None, ctypes.c_void_p(-1).value):
            libc.munmap(q, size)
        pytest.skip("the range was taken before it could be mapped again")
    try:
        mem2 = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(q))
        fresh = np.random.default_rng(62).integers(0, 256, size, dtype=np.uint8)
        mem2[:] = fresh
        got = torch.from_numpy(mem2).to("cuda:0").cpu().numpy()  # pageable H2D
        assert (got == fresh).all()
        a2, o2, l2 = synth.imix(2048, seed=63)
        mem2, mb2 = synth.mbuf_pool(a2, o2, l2, mem=mem2)
        with packets.HostRegion(ctx, q, size):
            check(ctx, a2, o2, l2, mb2, N.INGRESS_ZERO_COPY, fields=False)
        del mem2
    finally:
        libc.munmap(q, size)


def test_frames_submit_wait_double_buffered(ctx):
    """cgpu_parse_frames_submit / _wait: bursts submitted two at a time (the
    next before the previous is waited for), every result against the
    oracle; a third burst in flight is refused (EBUSY), a stale ticket is
    EINVAL, and a burst over two regions (no one-launch path) is parsed
    inside submit and still reported by its wait."""
    a, o, l = edge_batch(seed=31)
    mem, mbufs = synth.mbuf_pool(a, o, l)
    addrs, lens = synth.mbuf_frames(mem, mbufs)
    om, oc, oh, _ = oracle_lib.parse_batch(a, o, l, ALL, fields=False)
    cuts = [0, 1, 33, 600, 1700, 2999, 3000]
    with packets.HostRegion.of(ctx, mem):
        pend, done = [], []
        for s, e in zip(cuts[:-1], cuts[1:]):
            pend.append((s, e, packets.parse_frames_submit(ctx, addrs[s:e], lens[s:e], ALL)))
            if len(pend) == 2:
                with pytest.raises(N.CgpuError) as ex:
                    packets.parse_frames_submit(ctx, addrs[:8], lens[:8], ALL)
                assert ex.value.code == N.EBUSY
                s0, e0, tk = pend.pop(0)
                done.append((s0, e0, packets.parse_frames_wait(ctx, tk)))
        for s0, e0, tk in pend:
            done.append((s0, e0, packets.parse_frames_wait(ctx, tk)))
        for s0, e0, (m, c, h) in done:
            assert (m == om[s0:e0]).all() and (c == oc[s0:e0]).all() and (h == oh[s0:e0]).all()
        with pytest.raises(N.CgpuError) as ex:
            packets.parse_frames_wait(ctx, tk)  # already waited for
        assert ex.value.code == N.EINVAL
        # frames in two regions: parsed inside submit, reported by wait
        a2, o2, l2 = synth.imix(500, seed=32)
        mem2, mb2 = synth.mbuf_pool(a2, o2, l2)
        ad2, ln2 = synth.mbuf_frames(mem2, mb2)
        with packets.HostRegion.of(ctx, mem2):
            mix_a = np.concatenate([addrs[:300], ad2])
            mix_l = np.concatenate([lens[:300], ln2])
            tk = packets.parse_frames_submit(ctx, mix_a, mix_l, ALL)
            m, c, h = packets.parse_frames_wait(ctx, tk)
        om2, oc2, oh2, _ = oracle_lib.parse_batch(a2, o2, l2, ALL, fields=False)
        assert (m == np.concatenate([om[:300], om2])).all()
        assert (h == np.concatenate([oh[:300], oh2])).all()
    ctx.check()
