"""The rows kernels' longest-span-first wave order (parse.hip, "Longest span
first"): a launch of more than one round of waves has its last groups of 64
frames ordered by its first workgroups and handed to the waves through
granules.  The order must change no output.

The bench-size batches (1 Mi frames, 16,384 groups against 8,192 resident
waves) take the schedule in tests/test_bench_parity_gpu.py and
tests/test_reconcile_gpu.py.  Here the test build's hook CGPU_TEST_SCHED_WAVES
(read when a context is created) makes small batches take it: with 256
resident waves, the groups after the first 128 (half a round) are ordered,
in whole lists of 256 groups (one ordering workgroup each): a batch of 600
groups has its last 256 ordered.  Covered:
IMIX (stream path), 256-B and 1500-B frames (rows path), out-of-order
descriptors (window path; the scheduler's lightest class), a partial last
group, reconcile on stale IMIX, more groups than one schedule holds, two
streams of one context at once (one granule buffer per stream), graph
replays (a captured call runs without the schedule, so replays running at
once cannot share granules), and a wave that gives up waiting for its group
(CGPU_TEST_SCHED_SPINS=0): the call must fail loudly, never return stale
outputs.
"""
import os

import numpy as np
import pytest
import torch

import oracle_lib
from capsule_amd import _native as N
from capsule_amd import packets, synth

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
FLAGS = N.F_ACCEPT_ALL | N.F_FLOW_HASH | N.F_CSUM_IP | N.F_CSUM_L4


def _hooked_context(**hooks):
    """A context of the test build with these CGPU_TEST_* hooks (read when
    the context is created)."""
    for k, v in hooks.items():
        os.environ[k] = str(v)
    try:
        return packets.Context(0, test_hooks=True)
    finally:
        for k in hooks:
            del os.environ[k]


@pytest.fixture(scope="module")
def sctx():
    c = _hooked_context(CGPU_TEST_SCHED_WAVES=256)
    yield c
    c.close()


def _check_parse(c, arena, off, ln, flags=FLAGS, stream=None):
    b = packets.PacketBatch.from_numpy(arena, off, ln, DEV)
    r = packets.parse(c, b, flags=flags, stream=stream)
    torch.cuda.synchronize()
    om, oc, oh, _ = oracle_lib.parse_batch(arena, off, ln, flags, fields=False)
    for name, got, want in (("meta", r.meta.cpu().numpy().view(np.uint32), om),
                            ("csum", r.csum.cpu().numpy().view(np.uint32), oc),
                            ("flow hash", r.flow_hash.cpu().numpy().view(np.uint64), oh)):
        bad = np.nonzero(got != want)[0]
        assert not len(bad), f"{name} differs at {bad[:8]} of {len(got)}"
    return om


def _shuffle_groups(arena, off, ln, seed):
    """The same frames with their descriptors' 64-frame groups permuted: the
    groups keep their spans, the batch's order of them changes."""
    g = len(off) // 64
    perm = np.random.default_rng(seed).permutation(g)
    idx = np.concatenate([(perm[:, None] * 64 + np.arange(64)[None, :]).reshape(-1),
                          np.arange(64 * g, len(off))])
    return arena, off[idx].copy(), ln[idx].copy()


@pytest.mark.parametrize("n", [64 * 600, 64 * 600 + 17, 64 * 257 + 1])
def test_imix_stream_path(sctx, n):
    arena, off, ln = synth.imix(n, seed=n)
    om = _check_parse(sctx, arena, off, ln)
    assert (om & 0xFF == 0).all()


@pytest.mark.parametrize("size", [256, 1500])
def test_uniform_rows_path(sctx, size):
    arena, off, ln = synth.uniform(64 * 600, frame_len=size, slot=(size + 63) // 64 * 64, seed=size)
    _check_parse(sctx, arena, off, ln, flags=N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_CSUM_IP
                 | N.F_CSUM_L4 | N.F_FLOW_HASH)


def test_groups_out_of_order(sctx):
    """Groups permuted, and one group's frames reversed (no stream path; the
    scheduler puts it in its lightest class)."""
    arena, off, ln = synth.imix(64 * 600, seed=11)
    arena, off, ln = _shuffle_groups(arena, off, ln, 3)
    off[64 * 500:64 * 501] = off[64 * 500:64 * 501][::-1].copy()
    ln[64 * 500:64 * 501] = ln[64 * 500:64 * 501][::-1].copy()
    _check_parse(sctx, arena, off, ln)


def test_more_groups_than_one_schedule(sctx):
    """256 resident waves, 16,384 ordered at most (from half a round on): a
    batch of 17,000 groups runs groups 0 .. 615 in their own order and
    orders the last 16,384."""
    arena, off, ln = synth.imix(64 * 17000, seed=5)
    _check_parse(sctx, arena, off, ln)


def test_reconcile_stale_imix(sctx):
    arena, off, ln = synth.imix(64 * 600 + 5, seed=9)
    b = packets.PacketBatch.from_numpy(arena, off, ln, DEV)
    flags = N.F_ACCEPT_ALL | N.F_ACCEPT_ICMP
    r = packets.parse(sctx, b, flags=flags)
    meta = r.meta.cpu().numpy().view(np.uint32)
    stale = arena.copy()
    synth.stale_fields(stale, off, ln, meta, seed=4)
    b = packets.PacketBatch.from_numpy(stale, off, ln, DEV)
    st = packets.reconcile(sctx, b, r.meta, flags=flags, depth="l4")
    want, want_st = oracle_lib.reconcile(stale, off, ln, meta, flags, N.LAYER_L4)
    got = b.arena.cpu().numpy()
    bad = np.nonzero(got != want)[0]
    assert not len(bad), f"{len(bad)} bytes differ, first at {bad[:4]}"
    assert (st.cpu().numpy() == want_st).all()


def test_two_streams_at_once(sctx):
    """Two streams of one context, launches interleaved without syncs: each
    stream has its own granule buffer and tag sequence."""
    batches = []
    for seed in (21, 22):
        arena, off, ln = synth.imix(64 * 700, seed=seed)
        batches.append((arena, off, ln, packets.PacketBatch.from_numpy(arena, off, ln, DEV)))
    streams = [torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)]
    outs = []
    for k in range(6):
        s = streams[k & 1]
        arena, off, ln, b = batches[k & 1]
        outs.append((k & 1, packets.parse(sctx, b, flags=FLAGS, stream=s)))
    torch.cuda.synchronize()
    for j, r in outs:
        arena, off, ln, _ = batches[j]
        om, oc, oh, _ = oracle_lib.parse_batch(arena, off, ln, FLAGS, fields=False)
        assert (r.meta.cpu().numpy().view(np.uint32) == om).all()
        assert (r.flow_hash.cpu().numpy().view(np.uint64) == oh).all()


def test_graph_replay_with_new_frames(sctx):
    """A parse captured into a graph runs without the schedule (replays of
    one graph would share its granule buffer and tag); three replays over
    changed frame bytes, each against the oracle, then two graphs of the same
    call replayed on two streams at once."""
    arena, off, ln = synth.imix(64 * 600, seed=31)
    n = len(off)
    b = packets.PacketBatch.from_numpy(arena, off, ln, DEV)
    out = packets.ParseBuffers(n, DEV)
    s = torch.cuda.Stream(DEV)
    with torch.cuda.stream(s):
        packets.parse(sctx, b, flags=FLAGS, out=out, stream=s)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        packets.parse(sctx, b, flags=FLAGS, out=out, stream=s)
    rng = np.random.default_rng(5)
    for _ in range(3):
        ak = arena.copy()
        hit = rng.integers(0, len(ak), 20_000)
        ak[hit] ^= rng.integers(1, 256, len(hit), dtype=np.uint8)
        b.arena.copy_(torch.from_numpy(ak))
        g.replay()
        torch.cuda.synchronize()
        om, oc, oh, _ = oracle_lib.parse_batch(ak, off, ln, FLAGS, fields=False)
        assert (out.meta.cpu().numpy().view(np.uint32) == om).all()
        assert (out.csum.cpu().numpy().view(np.uint32) == oc).all()
        assert (out.flow_hash.cpu().numpy().view(np.uint64) == oh).all()
    # two graphs, replayed concurrently on two streams, each its own outputs
    outs = [packets.ParseBuffers(n, DEV) for _ in range(2)]
    streams = [torch.cuda.Stream(DEV) for _ in range(2)]
    graphs = []
    for o_, st in zip(outs, streams):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=st):
            packets.parse(sctx, b, flags=FLAGS, out=o_, stream=st)
        graphs.append(gr)
    torch.cuda.synchronize()
    for _ in range(4):
        for gr, st in zip(graphs, streams):
            with torch.cuda.stream(st):
                gr.replay()
    torch.cuda.synchronize()
    sctx.check()
    om, oc, oh, _ = oracle_lib.parse_batch(b.arena.cpu().numpy(), off, ln, FLAGS, fields=False)
    for o_ in outs:
        assert (o_.meta.cpu().numpy().view(np.uint32) == om).all()
        assert (o_.flow_hash.cpu().numpy().view(np.uint64) == oh).all()


def test_give_up_is_reported():
    """A wave of the ordered range that gives up waiting for its group
    writes no outputs for it; that must surface as CGPU_EIO: from
    cgpu_ctx_check after an asynchronous parse, and from the synchronous
    entry points themselves (here cgpu_parse_host).  CGPU_TEST_SCHED_SPINS=0
    makes every ordered wave give up at once.  Afterwards the context works
    (and reports nothing) for a batch that takes no schedule."""
    c = _hooked_context(CGPU_TEST_SCHED_WAVES=256, CGPU_TEST_SCHED_SPINS=0)
    try:
        arena, off, ln = synth.imix(64 * 600, seed=41)
        b = packets.PacketBatch.from_numpy(arena, off, ln, DEV)
        out = packets.ParseBuffers(len(off), DEV)
        out.meta.fill_(-1)
        packets.parse(c, b, flags=FLAGS, out=out)
        with pytest.raises(N.CgpuError) as e:
            c.check()
        assert e.value.code == N.EIO
        # the unordered groups were written, the ordered ones (the last 256
        # groups of 64 frames) were not
        meta = out.meta.cpu().numpy().view(np.uint32)
        om = oracle_lib.parse_batch(arena, off, ln, FLAGS, fields=False)[0]
        assert (meta[:64 * 344] == om[:64 * 344]).all()
        assert (meta[64 * 344:] == 0xFFFFFFFF).all()
        c.check()  # read and cleared
        frames = [bytes(arena[o:o + l]) for o, l in zip(off.tolist(), ln.tolist())]
        with pytest.raises(N.CgpuError) as e:
            packets.parse_host(c, frames, flags=FLAGS)
        assert e.value.code == N.EIO
        small = frames[:64 * 200]  # one round of waves: no schedule
        m, _, _, _ = packets.parse_host(c, small, flags=FLAGS)
        assert (m == om[:len(small)]).all()
        c.check()
    finally:
        c.close()


def test_order_range_follows_the_previous_batch(sctx):
    """The host orders from half a round on after a batch whose spans vary,
    from the second round on after one whose groups all have one span (the
    first ordering workgroup's report, capi.hip set_schedule).  Uniform and
    IMIX batches alternating on one stream: every result exact, whichever
    range each call gets."""
    imix = synth.imix(64 * 700, seed=21)
    uni = synth.uniform(64 * 700, frame_len=256, slot=256, seed=22)
    for arena, off, ln in (uni, imix, uni, uni, imix, imix, uni):
        _check_parse(sctx, arena, off, ln)
