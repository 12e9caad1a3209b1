"""rte_mbuf bursts through cgpu_parse_mbufs (the DPDK seam).

A synthetic DPDK-style mempool in host memory (synth.mbuf_pool: 128-B
rte_mbuf headers at the DPDK 19.11 offsets, shuffled objects, 128-B headroom)
is parsed in both ingress modes -- the calling core gathering into pinned
staging, and the device reading the registered mempool over PCIe -- and every
output is compared bit-exactly with the CPU oracle run on the same frames.
"""
import ctypes

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
    reg = packets.HostRegion(ctx, mem.ctypes.data, mem.nbytes)  # hipHostRegister
    try:
        check(ctx, a, o, l, mbufs, ingress)
    finally:
        reg.close()


@pytest.mark.parametrize("ingress", MODES)
def test_pinned_mempool(ctx, ingress):
    a, o, l = synth.imix(4096, seed=3)
    stride = (128 + 128 + int(l.max()) + 63) // 64 * 64
    pinned = torch.zeros(stride * len(o), dtype=torch.uint8, pin_memory=True)
    mem, mbufs = synth.mbuf_pool(a, o, l, mem=pinned.numpy())
    reg = packets.HostRegion(ctx, mem.ctypes.data, mem.nbytes)  # already page-locked: mapped only
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
    reg = packets.HostRegion(ctx, mem.ctypes.data, mem.nbytes)
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
    r1 = packets.HostRegion(ctx, m1.ctypes.data, m1.nbytes)
    r2 = packets.HostRegion(ctx, m2.ctypes.data, m2.nbytes)
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
    reg = packets.HostRegion(ctx, mem.ctypes.data, mem.nbytes)
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
            regs.append(packets.HostRegion(ctx, b.ctypes.data, b.nbytes))
        with pytest.raises(N.CgpuError):  # 16 regions per context
            packets.HostRegion(ctx, bufs[16].ctypes.data, bufs[16].nbytes)
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
    reg = packets.HostRegion(ctx, mem.ctypes.data, mem.nbytes)
    try:
        check(ctx, a, o, l, mbufs, ingress, fields=False)
    finally:
        reg.close()


def test_zero_copy_rejects_frame_past_its_buffer(ctx):
    """data_off + data_len > buf_len is no valid mbuf: the call fails."""
    a, o, l = synth.imix(128, seed=8)
    mem, mbufs = synth.mbuf_pool(a, o, l, room=2048)
    reg = packets.HostRegion(ctx, mem.ctypes.data, mem.nbytes)
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
    reg = packets.HostRegion(ctx, mem.ctypes.data, mem.nbytes)
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
    reg = packets.HostRegion(ctx, mem.ctypes.data, mem.nbytes)
    try:
        with pytest.raises(N.CgpuError):
            packets.parse_frames(ctx, addrs, lens, ALL, N.INGRESS_ZERO_COPY)
        # the context stays usable
        addrs[100] = synth.mbuf_frames(mem, mbufs)[0][100]
        gm = packets.parse_frames(ctx, addrs, lens, ALL, N.INGRESS_ZERO_COPY)[0]
        assert (gm == oracle_lib.parse_batch(a, o, l, ALL)[0]).all()
    finally:
        reg.close()

