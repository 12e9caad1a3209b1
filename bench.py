"""Device-resident packet-path benchmark (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config parse64|...] [--only]

A step is one pass of the hot path over one batch of synthetic packets that
is already resident in HBM.  Default workload = BASELINE config 2 with the
north-star feature set: 1,048,576 x 64-B Ethernet/IPv4/UDP frames, parse +
IPv4 header checksum + UDP checksum verify + 5-tuple flow hash, one
`cgpu_parse_batch` launch per step.  To keep the measurement an HBM one, each
rank keeps R copies of its batch at different HBM addresses (R x 70 MB >
the 256 MiB Infinity Cache) and step k processes copy k mod R.  Every timed
region follows at least W warm-up launches and MIN_WARM_S of device time.

Multi-GPU: one process per GPU, either started by torch.distributed.run or,
when `--gpus N` > 1 arrives without WORLD_SIZE in the environment, by this
script's own launcher (shards.launch_ranks: N child processes; the parent
never touches the GPU).  Every rank owns an independent RX-queue shard (its
own seed, its own HBM) -- no data-path collective, no RCCL, weak scaling;
a gloo process group carries only the barriers, the max-over-ranks of the
elapsed time and the per-rank figures.  value = packets processed by all
ranks / that time.

Rank 0 prints ONE JSON line:
  value / roofline    the --config (default parse64) on every rank; roofline
                      per launch from HIP events on the launch stream, with
                      each rank's fraction in roofline.per_rank;
  shards              BASELINE config 5: IMIX parse + hash, one shard per GPU,
                      aggregate Mpps and per-rank roofline fraction (every N);
  sizes               N=1 only: the metric's other frame sizes (256 B, 1500 B)
                      and configs 3, 3' and 4 (IMIX, IMIX + checksums, nat64),
                      each with its own warm-up and timed loop;
  cpu_baseline        N=1 only: the C oracle restatement of the same workload
                      on a bounded sample, one host core and one per shard.
"""
import argparse
import ctypes
import json
import os
import pathlib
import sys
import time

import numpy as np

from capsule_amd.shards import numa_bind

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
INFINITY_CACHE = 256 << 20


def _cnt(n):
    return "1M" if n == 1 << 20 else str(n)


def make_workload(cfg, seed, n=1 << 20):
    from capsule_amd import _native as N
    from capsule_amd import synth

    if cfg == "parse64":
        arena, off, ln = synth.uniform(n, seed=seed)
        flags = N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_CSUM_IP | N.F_CSUM_L4 | N.F_FLOW_HASH
        desc = f"{_cnt(n)} x 64B Eth/IPv4/UDP: parse + IPv4/UDP checksum verify + 5-tuple hash"
        return dict(arena=arena, off=off, len=ln, flags=flags, kind="parse", desc=desc,
                    algo_bytes=int(ln.astype(np.int64).sum()) + 6 * n, frame="64B")
    if cfg in ("parse256", "parse1500"):  # the metric's other frame sizes, same work as parse64
        size = 256 if cfg == "parse256" else 1500
        arena, off, ln = synth.uniform(n, frame_len=size, seed=seed, slot=(size + 63) // 64 * 64)
        flags = N.F_ACCEPT_V4 | N.F_ACCEPT_UDP | N.F_CSUM_IP | N.F_CSUM_L4 | N.F_FLOW_HASH
        desc = f"{_cnt(n)} x {size}B Eth/IPv4/UDP: parse + IPv4/UDP checksum verify + 5-tuple hash"
        return dict(arena=arena, off=off, len=ln, flags=flags, kind="parse", desc=desc,
                    algo_bytes=int(ln.astype(np.int64).sum()) + 6 * n, frame=f"{size}B")
    if cfg == "imix":
        return imix_header_bytes_workload(seed, n)
    if cfg == "imix_csum":
        arena, off, ln = synth.imix(n, seed=seed)
        flags = N.F_ACCEPT_ALL | N.F_FLOW_HASH | N.F_CSUM_IP | N.F_CSUM_L4
        desc = f"{_cnt(n)} IMIX 64/570/1500 7:4:1 v4/v6 x UDP/TCP: parse + checksums + hash"
        return dict(arena=arena, off=off, len=ln, flags=flags, kind="parse", desc=desc,
                    algo_bytes=int(ln.astype(np.int64).sum()) + 6 * n, frame="IMIX",
                    line_floor=line_floor_bytes(off, ln))
    if cfg in ("nat64", "nat64_cold"):
        arena, off, ln = synth.nat64_stream(n, seed=seed)
        desc = (f"{_cnt(n)} x 256B IPv6/TCP -> IPv4 6to4 rewrite + TCP/IPv4 checksums (examples/nat64), "
                "236-B output frames packed back to back")
        # The egress buffer is packed (a TX ring / DMA-out image): with the
        # frames left in 256-B slots every frame's last output line would be
        # written partially.
        new_len = ln.astype(np.int64) - 20
        out_off = np.zeros(n, np.int64)
        out_off[1:] = np.cumsum(new_len)[:-1]
        if cfg == "nat64_cold":
            desc = (f"first pass of the {_cnt(n)} x 256B IPv6/TCP stream over a fresh port map "
                    "(every key new: ordered NEXT_PORT assignment, main.rs:45-51), 6to4 "
                    "rewrite + checksums, packed egress")
        return dict(arena=arena, off=off, len=ln, flags=0, kind=cfg, desc=desc,
                    out_off=out_off.astype(np.uint32), out_size=int(new_len.sum()) + 64,
                    algo_bytes=int(ln.astype(np.int64).sum()) + 6 * n, frame="256B")
    if cfg in ("reconcile64", "reconcile_imix"):
        return reconcile_workload(cfg, seed, n)
    if cfg == "nat64_4to6":
        # the v6 stream that populates the port map; the timed replies are
        # built from its 6to4 output on the device (main())
        arena, off, ln = synth.nat64_stream(n, seed=seed)
        desc = (f"{_cnt(n)} x 236B IPv4/TCP replies -> IPv6 4to6 rewrite + TCP checksum "
                "(examples/nat64), port map populated by a 6to4 pass")
        return dict(arena=arena, off=off, len=ln, flags=0, kind="nat64_4to6", desc=desc,
                    frame="236B")
    raise SystemExit(f"unknown config {cfg}")


def reconcile_workload(cfg, seed, n):
    """Packet::reconcile_all from the L4 layer (packets/mod.rs:297-300) on a
    parsed burst whose length and checksum fields went stale (a pipeline
    that rewrote ports, then reconciles before transmit); the parse and the
    staling are reconcile_setup's (untimed).  Algorithmic bytes: every frame
    byte (the L4 checksum spans to the frame end) + the 6-B descriptor + the
    4-B meta word read, plus the fields written (UDP length + checksum, TCP
    checksum, IPv4 total_length + header checksum, IPv6 payload_length)."""
    from capsule_amd import _native as N
    from capsule_amd import synth

    if cfg == "reconcile64":
        arena, off, ln = synth.uniform(n, seed=seed)
        flags = N.F_ACCEPT_V4 | N.F_ACCEPT_UDP
        frame, desc = "64B", f"{_cnt(n)} x 64B Eth/IPv4/UDP"
    else:
        arena, off, ln = synth.imix(n, seed=seed)
        flags = N.F_ACCEPT_ALL
        frame, desc = "IMIX", f"{_cnt(n)} IMIX 64/570/1500 7:4:1 v4/v6 x UDP/TCP"
    return dict(arena=arena, off=off, len=ln, flags=flags, kind="reconcile", frame=frame,
                seed=seed, desc=desc + ": reconcile_all from L4 in place (UDP length + L4 "
                "checksum, IPv4 total_length + header checksum / IPv6 payload_length); the "
                "resident copies are staled once, so the timed launches re-reconcile frames "
                "an earlier pass already reconciled (the kernel's work does not depend on it)")


def reconcile_setup(w, ctx, dev):
    """Parse the burst on the device (its meta words, as a pipeline has
    them), then make its length / checksum fields stale (host side) and set
    the algorithmic bytes from the layers the parse found.  Returns the
    device meta tensor; w["arena"] becomes the stale arena."""
    import torch

    from capsule_amd import _native as N
    from capsule_amd import packets, synth

    b = packets.PacketBatch.from_numpy(w["arena"], w["off"], w["len"], dev)
    meta_d = packets.parse(ctx, b, flags=w["flags"]).meta.clone()
    torch.cuda.synchronize(dev)
    del b
    meta = meta_d.cpu().numpy().view(np.uint32)
    w["arena"] = w["arena"].copy()
    synth.stale_fields(w["arena"], w["off"], w["len"], meta, seed=w["seed"] + 1)
    l3, l4 = (meta >> 16) & 3, (meta >> 18) & 3
    written = np.where(l3 == N.L3_IPV4, 4, 2) + np.where(l4 == N.L4_UDP, 4, 2)
    n = len(w["off"])
    w["meta"] = meta
    w["algo_bytes"] = int(w["len"].astype(np.int64).sum()) + 10 * n + int(written.sum())
    return meta_d


def nat64_4to6_setup(w, ctx, dev):
    """Run the 6to4 pass (untimed) and turn its output into reply frames."""
    import torch

    from capsule_amd import packets
    from capsule_amd import synth

    gw = packets.Nat64Gateway(ctx, capacity_log2=PORTMAP_LOG2)
    b = packets.PacketBatch.from_numpy(w["arena"], w["off"], w["len"], dev)
    ob, disp, _ = gw.nat_6to4(b)
    torch.cuda.synchronize(dev)
    assert (disp.cpu().numpy() == 0).all()
    w["setup"] = (w["arena"], w["off"], w["len"])
    w["arena"], w["off"], w["len"] = synth.nat64_replies(
        ob.arena.cpu().numpy(), w["off"], ob.len.cpu().numpy().view(np.uint16))
    w["algo_bytes"] = int(w["len"].astype(np.int64).sum()) + 6 * len(w["off"])
    return gw


def line_floor_bytes(off, span):
    """Bytes of the distinct 128-B lines that [off, off + span) of every
    packet touches, plus the descriptor arrays (u32 off, u16 len): the HBM
    read floor of a kernel that reads exactly those bytes, since HBM and L2
    move whole lines (TCC_EA0_RDREQ_64B ~ 0 on these kernels)."""
    o = off.astype(np.int64)
    e = o + np.maximum(span.astype(np.int64), 1) - 1
    first, last = o >> 7, e >> 7
    cnt = last - first + 1
    lines = np.repeat(first, cnt) + (np.arange(int(cnt.sum())) -
                                     np.repeat(np.cumsum(cnt) - cnt, cnt))
    n = len(off)
    return 128 * (len(np.unique(lines)) + -(-4 * n // 128) + -(-2 * n // 128))


def imix_header_bytes_workload(seed, n=1 << 20):
    """IMIX parse+hash: algorithmic bytes = headers touched + 6 B descriptor."""
    from capsule_amd import _native as N
    from capsule_amd import synth

    arena, off, ln = synth.imix(n, seed=seed)
    eth = np.full(n, 14, np.int64)
    l3 = np.zeros(n, np.int64)
    l4 = np.zeros(n, np.int64)
    # decode the synthetic frames' layer kinds from their bytes (host-side bookkeeping)
    o = off.astype(np.int64)
    et = arena[o + 12].astype(np.int64) * 256 + arena[o + 13]
    v6 = et == 0x86DD
    l3 = np.where(v6, 40, 20)
    proto = np.where(v6, arena[o + 14 + 6], arena[o + 14 + 9])
    l4 = np.where(proto == 17, 8, 20)
    algo = int((eth + l3 + l4 + 6).sum())
    flags = N.F_ACCEPT_ALL | N.F_FLOW_HASH
    return dict(arena=arena, off=off, len=ln, flags=flags, kind="parse", frame="IMIX",
                desc=f"{_cnt(n)} IMIX 64/570/1500 7:4:1 v4/v6 x UDP/TCP: parse + 5-tuple hash",
                algo_bytes=algo, line_floor=line_floor_bytes(off, eth + l3 + l4))


def cpu_baseline(w, seconds):
    """The C oracle (CPU restatement of the reference path, test infra) on
    the same batch, time-bounded samples: one host core, then one thread per
    core on independent shards (capsule's RSS model: one core per RX queue,
    shared nothing; nat64 keeps one port map per shard)."""
    import threading

    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib

    L = oracle_lib.lib()
    arena, off, ln = w["arena"], w["off"], w["len"]
    n = len(off)
    p = lambda a: a.ctypes.data  # noqa: E731

    def make_run():
        if w["kind"] == "parse":
            meta = np.zeros(n, np.uint32)
            csum = np.zeros(n, np.uint32)
            h = np.zeros(n, np.uint64)
            return lambda: L.or_parse_batch(p(arena), p(off), p(ln), n, w["flags"], p(meta),
                                            p(csum), p(h), None)
        if w["kind"] == "reconcile":
            work = arena.copy()
            meta = w["meta"]
            return lambda: L.or_reconcile(p(work), len(work), p(off), p(ln), p(meta), n, w["flags"], 4, None)
        pm = oracle_lib.PortMap()
        out = np.zeros(len(arena), np.uint8)
        olen = np.zeros(n, np.uint16)
        disp = np.zeros(n, np.uint8)
        st = np.zeros(n, np.uint8)
        fn = L.or_nat64_6to4
        if w["kind"] == "nat64_4to6":
            pm.nat_6to4(*w["setup"])  # same port map as the device side
            fn = L.or_nat64_4to6
        if w["kind"] == "nat64_cold":  # every pass over a fresh map (the map's
            # construction is inside the sample, as the device's reset is not)
            def cold():
                m = oracle_lib.PortMap()
                return fn(m.h, p(arena), p(off), p(ln), n, p(out), p(off), p(olen), p(disp),
                          p(st))
            return cold
        return lambda: (pm, fn(pm.h, p(arena), p(off), p(ln), n, p(out), p(off),
                               p(olen), p(disp), p(st)))

    def timed(run, secs):
        run()  # warm
        passes, t0 = 0, time.perf_counter()
        while True:
            run()
            passes += 1
            el = time.perf_counter() - t0
            if el >= secs:
                return passes, el

    passes, el = timed(make_run(), seconds)
    res = {"value": round(passes * n / el / 1e6, 3), "unit": "Mpps", "cores": 1,
           "kind": "port",
           "sample": f"C oracle (oracle/oracle.c) over the same {n}-packet batch, "
                     f"{passes} passes, {el:.1f} s, 1 thread"}
    # one shard per core: ctypes drops the GIL for the duration of each call
    threads = min(16, os.cpu_count() or 1)  # the GPU box's CPU share is 16
    runs = [make_run() for _ in range(threads)]
    got = [None] * threads

    def worker(t):
        got[t] = timed(runs[t], min(5.0, seconds))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    res["all_cores"] = {"threads": threads,
                        "value": round(sum(pp * n / e for pp, e in got) / 1e6, 3),
                        "sample": f"{threads} threads, each its own shard replica of the "
                                  f"{n}-packet batch, ~{min(5.0, seconds):.0f} s"}
    if w["kind"] == "parse" and w["frame"] == "64B":
        # the reference bench's own routine (bench/packets.rs:65-69 multi_parse_udp),
        # batches of 500 like bench/packets.rs:31
        passes, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < min(3.0, seconds):
            for s in range(0, n, 500):
                e = min(n, s + 500)
                L.or_multi_parse_udp(p(arena), p(off[s:e]), p(ln[s:e]), e - s)
            passes += 1
        el = time.perf_counter() - t0
        res["multi_parse_udp_mpps"] = round(passes * n / el / 1e6, 3)
        # ... and on the reference bench's own input shape: v4_udp() builds
        # 42-B header-only Eth/IPv4/UDP packets (testils/proptest/strategy.rs:
        # 446-448), each in its own mbuf (128-B rte_mbuf + 128-B headroom,
        # 2304-B objects), parsed in batches of 500 (bench/packets.rs:31).
        from capsule_amd import synth

        m, stride = 500 * 64, 2304
        frames = synth.build_frames(np.random.default_rng(7), m, synth.V4_UDP, 42)
        a42 = np.zeros(m * stride, np.uint8)
        a42.reshape(m, stride)[:, 256:298] = frames
        o42 = (np.arange(m, dtype=np.uint32) * stride + 256).astype(np.uint32)
        l42 = np.full(m, 42, np.uint16)
        assert L.or_multi_parse_udp(p(a42), p(o42), p(l42), m) == m
        passes, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < min(3.0, seconds):
            for s in range(0, m, 500):
                L.or_multi_parse_udp(p(a42), p(o42[s:s + 500]), p(l42[s:s + 500]), 500)
            passes += 1
        el = time.perf_counter() - t0
        res["multi_parse_udp_42B"] = {
            "value": round(passes * m / el / 1e6, 3), "unit": "Mpps", "cores": 1,
            "sample": f"{m} 42-B v4_udp() packets in 2304-B mbuf objects, batches of 500, "
                      f"{passes} passes, {el:.1f} s"}
    try:
        res["host_cpu"] = next(x.split(":", 1)[1].strip() for x in
                               open("/proc/cpuinfo") if x.startswith("model name"))
    except Exception:
        pass
    return res


SEEDS = {"parse64": 2, "parse256": 2, "parse1500": 2, "imix": 3, "imix_csum": 3, "nat64": 4,
         "nat64_4to6": 4, "nat64_cold": 4, "reconcile64": 5, "reconcile_imix": 5}
CONFIGS = tuple(SEEDS)
METRIC = "Mpps device-resident parse+cksum+hash @64/256/1500B; % HBM-read roofline"
# the metric's other sizes and BASELINE's other single-GPU configs, timed in
# the same N=1 run (the `sizes` object of the line)
SIZES = ("parse256", "parse1500", "imix", "imix_csum", "nat64", "nat64_4to6", "nat64_cold",
         "reconcile64", "reconcile_imix")
# BASELINE config 5: IMIX shards, one per GPU (the `shards` object)
SHARD_CONFIG = "imix"
MIN_WARM_S = 0.15  # device time of warm-up before any timed region (steady clocks)
PORTMAP_LOG2 = int(os.environ.get("CGPU_BENCH_PORTMAP_LOG2", "20"))  # Nat64Gateway default


def pmc_traffic(cfg):
    """HBM bytes per launch from profiles/pmc_<cfg>.json, when that profile
    was taken on the current kernel sources (scripts/summarize_prof.py)."""
    pmc = ROOT / "profiles" / f"pmc_{cfg}.json"
    if not pmc.exists():
        return None
    sys.path.insert(0, str(ROOT / "scripts"))
    from summarize_prof import source_hash

    p = json.loads(pmc.read_text())
    if p.get("src_hash") == source_hash(cfg) and "traffic_bytes" in p:
        return int(p["traffic_bytes"])
    return None


def bench_config(cfg, g, ctx, dev, steps, warmup, w=None, queues=1, n_pkts=1 << 20):
    """Time one config on this rank.

    Builds the rank's shard of the workload, keeps R copies resident in HBM
    (R x batch > 2 x the 256 MiB Infinity Cache; launch k processes copy
    k mod R), warms up for at least `warmup` launches AND MIN_WARM_S of
    device time, then times `steps` launches between a sync + barrier on
    each side (ShardGroup.timed: max over ranks).  HIP events recorded on the
    launch stream around the same launches give the per-launch device time.

    queues > 1 (parse configs): the rank serves that many RX queues, each on
    its own HIP stream with its own outputs, launch k on queue k mod queues;
    consecutive launches then overlap, so there is no per-launch device time
    and the rate comes from the wall clock alone.
    """
    import torch

    from capsule_amd import packets

    w = w or make_workload(cfg, g.shard_seed(0xC0FFEE + SEEDS[cfg]), n=n_pkts)
    n = len(w["off"])
    if w["kind"] == "nat64_cold":
        return bench_nat64_cold(cfg, g, ctx, dev, steps, warmup, w)
    gw = nat64_4to6_setup(w, ctx, dev) if w["kind"] == "nat64_4to6" else None
    meta_d = reconcile_setup(w, ctx, dev) if w["kind"] == "reconcile" else None
    batch_bytes = len(w["arena"]) + 6 * n
    copies = max(2, -(-2 * INFINITY_CACHE // batch_bytes))
    b0 = packets.PacketBatch.from_numpy(w["arena"], w["off"], w["len"], dev)
    batches = [b0] + [packets.PacketBatch(b0.arena.clone(), b0.off.clone(), b0.len.clone())
                      for _ in range(copies - 1)]
    stream = torch.cuda.current_stream(dev)
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(queues - 1)]
    if w["kind"] == "parse":
        # checksum verify: CSUM_OK bits in meta, computed values not stored
        outs = [packets.ParseBuffers(n, dev, csum=False) for _ in range(max(2, queues))]
        launchers = [packets.ParseLauncher(ctx, batches[k % copies], outs[k % len(outs)], w["flags"],
                                           streams[k % queues]) for k in range(2 * copies * queues)]
    elif w["kind"] == "reconcile":
        assert queues == 1
        outs = meta_d
        launchers = [packets.ReconcileLauncher(ctx, batches[k], meta_d, w["flags"], "l4", stream)
                     for k in range(copies)]
    else:
        assert queues == 1, "one port map, one queue"
        direction = "4to6" if gw is not None else "6to4"
        gw = gw or packets.Nat64Gateway(ctx, capacity_log2=PORTMAP_LOG2)
        if "out_off" in w:
            oo = torch.from_numpy(w["out_off"].view(np.int32)).to(dev)
            outs = [(torch.empty(w["out_size"], dtype=torch.uint8, device=dev), oo,
                     torch.empty(n, dtype=torch.int16, device=dev),
                     torch.empty(n, dtype=torch.uint8, device=dev),
                     torch.empty(n, dtype=torch.uint8, device=dev)) for _ in range(2)]
        else:
            outs = [(torch.empty_like(b.arena), b.off, torch.empty(n, dtype=torch.int16, device=dev),
                     torch.empty(n, dtype=torch.uint8, device=dev),
                     torch.empty(n, dtype=torch.uint8, device=dev)) for b in batches[:2]]
        launchers = [packets.Nat64Launcher(gw, batches[k % copies], outs[k & 1], stream,
                                           direction) for k in range(2 * copies)]
    cycle = len(launchers)

    # HIP events on the launch stream: eva behind the first timed launch, ev1
    # behind the last; (ev1 - eva) / (K - 1) is the per-launch device time of
    # launches 2..K (kernel plus the back-to-back dispatch gap), which the
    # host keeps queued ahead of the device.  Nothing is recorded before the
    # first launch, so the region starts with the launch itself; the first
    # launch's submission latency is in ms_per_step, not in the kernel time.
    # Both are recorded once here first: torch creates an event's HIP object
    # at its first record, which must not happen inside the timed region.
    eva, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for e in (eva, ev1):
        e.record(stream)

    # warm-up: >= `warmup` launches and >= MIN_WARM_S of device time, in
    # bursts of 64 back-to-back launches (a sync after each keeps the
    # runtime's launch queue short), so the clocks are at their steady state;
    # then two untimed rehearsals of the timed region's own shape (`steps`
    # launches between syncs)
    k = 0
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    done = 0
    while done < warmup or time.perf_counter() - t0 < MIN_WARM_S:
        for _ in range(64):
            launchers[k % cycle]()
            k += 1
        done += 64
        torch.cuda.synchronize(dev)
    for _ in range(2):
        for _ in range(steps):
            launchers[k % cycle]()
            k += 1
        torch.cuda.synchronize(dev)

    state = {"k": k, "left": steps}

    def one():
        launchers[state["k"] % cycle]()
        if state["left"] == steps:
            eva.record(stream)
        state["k"] += 1
        state["left"] -= 1
        if state["left"] == 0:
            ev1.record(stream)

    elapsed = g.timed(one, steps, sync=lambda: torch.cuda.synchronize(dev))
    if queues > 1:  # launches overlap across the queues: wall clock only
        kern_us = elapsed / steps * 1e6
    elif steps > 1:
        kern_us = eva.elapsed_time(ev1) / (steps - 1) * 1e3
    else:  # one launch: eva and ev1 both follow it; fall back to the wall time
        kern_us = elapsed / steps * 1e6
    res = dict(cfg=cfg, n=n, desc=w["desc"], frame=w["frame"], copies=copies, elapsed=elapsed, queues=queues,
               steps=steps, kern_us=kern_us, algo_bytes=w["algo_bytes"],
               achieved=w["algo_bytes"] / (kern_us * 1e-6) / 1e9, w=w,
               line_floor=w.get("line_floor"))
    del launchers, outs, batches, b0
    if gw is not None:
        gw.close()
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    return res


# per-rank device identity (ordinal, PCI address), gathered once in main():
# a scaling line then shows which GPU each rank's figures come from
DEVICES = [None]


def summarize(r, g):
    """Aggregate of one config over the ranks (collective: every rank calls
    it in the same order)."""
    fr = g.gather(r["achieved"] / HBM_PEAK_GBS)
    us = g.gather(r["kern_us"])
    total = g.sum(r["n"] * r["steps"])
    devs = DEVICES if len(DEVICES) == len(us) else [None] * len(us)
    s = {
        "workload": r["desc"], "packets_per_step": r["n"], "steps": r["steps"],
        "mpps": round(total / r["elapsed"] / 1e6, 2),
        "ms_per_step": round(r["elapsed"] / r["steps"] * 1e3, 5),
        "kernel_us": round(r["kern_us"], 3),
        "achieved_GBps": round(r["achieved"], 1),
        "frac": round(r["achieved"] / HBM_PEAK_GBS, 4),
        "algo_bytes_per_launch": r["algo_bytes"],
        "traffic": r["traffic"] if "traffic" in r else pmc_traffic(r["cfg"]),
        "per_rank": [{"rank": i, "kernel_us": round(u, 3), "frac": round(f, 4), "device": d}
                     for i, (u, f, d) in enumerate(zip(us, fr, devs))],
    }
    if r.get("line_floor"):
        # HBM and L2 move 128-B lines: the bytes of the distinct lines the
        # kernel must touch in this layout, and the fraction of the peak the
        # kernel reaches on them
        lf = r["line_floor"]
        s["line_floor_bytes"] = lf
        s["frac_of_line_floor"] = round(lf / (r["kern_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
    for k in ("note",):
        if r.get(k):
            s[k] = r[k]
    return s


def device_identity(ordinal):
    import torch

    p = torch.cuda.get_device_properties(ordinal)
    return {"ordinal": ordinal, "name": p.name,
            "pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"}


def check_devices(devs, one_device):
    """Each rank on its own GPU (distinct PCI addresses), unless the N-rank
    path is being rehearsed on one card (CGPU_BENCH_ONE_DEVICE=1)."""
    pcis = [d["pci"] for d in devs]
    if not one_device and len(set(pcis)) != len(pcis):
        raise SystemExit(f"bench.py: ranks share a GPU ({pcis}); set CGPU_BENCH_ONE_DEVICE=1 "
                         "to rehearse N ranks on one device")


def bench_nat64_cold(cfg, g, ctx, dev, steps, warmup, w):
    """The cold port map: every timed call is the first pass of the stream
    over a freshly reset map (cgpu_portmap_reset, enqueued on the stream
    before the call), so every key is new and its port comes from the
    ordered NEXT_PORT assignment (assigned_port's miss path, main.rs:45-51:
    the fused kernel defers every frame, the tail kernel orders the keys and
    rewrites them).  kernel_us = device time of the call alone (HIP events
    after the reset and after the tail); the wall-clock rate includes the
    resets."""
    import torch

    from capsule_amd import packets

    n = len(w["off"])
    stream = torch.cuda.current_stream(dev)
    gw = packets.Nat64Gateway(ctx, capacity_log2=PORTMAP_LOG2)
    b = packets.PacketBatch.from_numpy(w["arena"], w["off"], w["len"], dev)
    oo = torch.from_numpy(w["out_off"].view(np.int32)).to(dev)
    out = (torch.empty(w["out_size"], dtype=torch.uint8, device=dev), oo,
           torch.empty(n, dtype=torch.int16, device=dev),
           torch.empty(n, dtype=torch.uint8, device=dev),
           torch.empty(n, dtype=torch.uint8, device=dev))
    launch = packets.Nat64Launcher(gw, b, out, stream, "6to4")
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    for a, z in evs:  # create the HIP events outside the timed region
        a.record(stream)
        z.record(stream)
    for _ in range(max(3, min(warmup, 20))):
        gw.reset(stream=stream)
        launch()
    torch.cuda.synchronize(dev)
    keys = gw.size()  # every call starts over: the map holds exactly one pass's keys
    assert 0 < keys <= n and gw.next_port() == (1025 + keys) & 0xFFFF, "cold pass"
    state = {"j": 0}

    def one():
        j = state["j"]
        gw.reset(stream=stream)
        evs[j][0].record(stream)
        launch()
        evs[j][1].record(stream)
        state["j"] = j + 1

    elapsed = g.timed(one, steps, sync=lambda: torch.cuda.synchronize(dev))
    kern_us = sum(a.elapsed_time(z) for a, z in evs) / steps * 1e3
    keys = gw.size()
    gw.close()
    del launch, out, b
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    return dict(cfg=cfg, n=n, desc=w["desc"], frame=w["frame"], copies=1, elapsed=elapsed,
                queues=1, steps=steps, kern_us=kern_us, algo_bytes=w["algo_bytes"],
                achieved=w["algo_bytes"] / (kern_us * 1e-6) / 1e9, w=w,
                note=f"{keys} new keys per call; mpps and ms_per_step include the map reset "
                     "before each call, kernel_us and frac do not")


def stub_worker(args):
    """GPU-free stand-in for one rank (--stub, for CPU tests of the launcher
    and of the line's shape): the same ShardGroup control plane and the same
    JSON line, with a sleep in place of each launch."""
    from capsule_amd.shards import ShardGroup

    g = ShardGroup()
    same = os.environ.get("CGPU_BENCH_STUB_SAME_DEVICE") == "1"  # (test of check_devices)
    pci = "0000:00:00" if same else f"0000:{g.local_rank + 1:02x}:00"
    # no GPU: the binding runs against a sysfs without these devices
    DEVICES[:] = g.gather_obj({"ordinal": g.local_rank, "name": "stub", "pci": pci,
                               "numa": numa_bind(pci, sysfs="/nonexistent")})
    check_devices(DEVICES, os.environ.get("CGPU_BENCH_ONE_DEVICE") == "1")

    def fake(cfg, steps):
        el = g.timed(lambda: time.sleep(1e-4 * (1 + g.rank)), steps)
        return dict(cfg=cfg, n=1 << 20, desc=f"stub {cfg}", frame="-", copies=0, elapsed=el,
                    steps=steps, kern_us=100.0 * (1 + g.rank), algo_bytes=70 << 20,
                    achieved=(70 << 20) / (1e-4 * (1 + g.rank)) / 1e9, w=None, traffic=None,
                    line_floor=(108 << 20) if cfg.startswith("imix") else None)

    main = fake(args.config, args.steps)
    extra = {} if args.only else {"shards": dict(summarize(fake(SHARD_CONFIG, args.steps), g),
                                                  config=SHARD_CONFIG)}
    if not args.only and g.world == 1:
        extra["sizes"] = {c: summarize(fake(c, args.steps), g) for c in SIZES}
    emit(args, g, main, extra, stub=True)
    g.close()


def emit(args, g, m, extra, cpu=None, stub=False):
    s = summarize(m, g)
    total = g.sum(m["n"] * m["steps"])
    result = {
        "metric": METRIC,
        "value": round(total / m["elapsed"] / 1e6, 2),
        "unit": "Mpps",
        "n_gpus": g.world,
        "steps": m["steps"],
        "warmup": args.warmup,
        "ms_per_step": round(m["elapsed"] / m["steps"] * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded proptest-style reconciled frames, one shard per rank)",
        "config": {"workload": m["desc"], "config": m["cfg"], "packets_per_step": m["n"],
                   "global_batch": m["n"] * g.world, "resident_copies": m["copies"],
                   "launch": "direct",
                   "parallelism": f"{g.world} independent RX-queue shards, one per GPU "
                                  "(no collective; gloo control plane only)"},
        "roofline": {"bound": "hbm", "achieved": s["achieved_GBps"], "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": s["frac"], "traffic": s["traffic"],
                     "kernel_us": s["kernel_us"], "algo_bytes_per_launch": m["algo_bytes"],
                     "per_rank": s["per_rank"],
                     "mean_frac_over_ranks": round(sum(r["frac"] for r in s["per_rank"]) /
                                                   g.world, 4)},
        "parity": {"parse_and_checksums": "bit-exact vs the C oracle, which is pinned by the "
                                          "reference's own KATs (tests/golden)",
                   "flow_hash": "bit-exact vs the C oracle; parity unpinned vs the reference "
                                "(convention: SipHash-1-3(0,0) over Rust-1.50 derive(Hash) "
                                "of Flow, no reference vector exists)",
                   "nat64_bytes": "bit-exact vs the C oracle, which a second, independent "
                                  "restatement (tests/pyref_nat64.py) matches byte for byte; "
                                  "parity unpinned vs the reference (examples/nat64 has no "
                                  "test or expected output)"},
    }
    result.update(extra)
    if cpu is not None:
        result["cpu_baseline"] = cpu
    if stub:
        result["stub"] = True
    if g.rank == 0:
        print(json.dumps(result), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--config", default="parse64", choices=list(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--only", action="store_true",
                    help="time the --config only (no `shards` / `sizes` objects; for profiling)")
    ap.add_argument("--sub-steps", type=int, default=300,
                    help="timed launches of each `shards` / `sizes` config (at least --steps)")
    ap.add_argument("--n", type=int, default=1 << 20,
                    help="packets per batch (default 1 Mi, the BASELINE configs; smaller for "
                         "the bench-mode tests)")
    ap.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--e2e", action="store_true",
                    help="host-resident batches: pinned H2D + parse + D2H, pipelined (DESIGN.md §8)")
    ap.add_argument("--ingress", choices=["stage", "zero_copy", "frames"],
                    help="with --e2e: rte_mbuf bursts from a host mempool through cgpu_parse_mbufs "
                         "(stage / zero_copy) or as (address, length) pairs through "
                         "cgpu_parse_frames (frames, zero-copy)")
    ap.add_argument("--burst", type=int, default=1 << 18,
                    help="with --ingress: mbufs per cgpu_parse_mbufs call")
    ap.add_argument("--inflight", type=int, default=1, choices=[1, 2],
                    help="with --ingress frames: bursts in flight (2: cgpu_parse_frames_submit "
                         "/ _wait, the next burst submitted before the previous one is waited for)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # Not started by torch.distributed.run: start one rank process per GPU
        # (children of this process, which never touches the GPU).
        from capsule_amd.shards import launch_ranks

        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}; "
              "using WORLD_SIZE", file=sys.stderr)
    if args.stub:
        return stub_worker(args)

    import torch

    from capsule_amd import packets
    from capsule_amd.shards import ShardGroup

    if args.e2e:  # one rank: its host thread on the GPU's node, then the pinned buffers
        torch.cuda.set_device(0)
        numa_bind(device_identity(0)["pci"])
    if args.e2e and args.ingress:
        return e2e_mbufs(args)
    if args.e2e:
        return e2e(args)
    g = ShardGroup()
    # CGPU_BENCH_ONE_DEVICE=1: every rank on GPU 0 (rehearsing the N-rank
    # path on a one-GPU box; the ranks then share the card)
    one_device = os.environ.get("CGPU_BENCH_ONE_DEVICE") == "1"
    ordinal = 0 if one_device else g.local_rank
    dev = torch.device("cuda", ordinal)
    torch.cuda.set_device(dev)
    ident = device_identity(ordinal)
    # the rank's host thread on its GPU's NUMA node before any host buffer
    ident["numa"] = numa_bind(ident["pci"])
    DEVICES[:] = g.gather_obj(ident)
    check_devices(DEVICES, one_device)
    ctx = packets.Context(ordinal)

    main_r = bench_config(args.config, g, ctx, dev, args.steps, args.warmup, n_pkts=args.n)
    extra = {}
    if not args.only:
        sub = max(args.steps, args.sub_steps)
        # BASELINE config 5: this rank's IMIX shard, all ranks at once
        shard_r = (main_r if args.config == SHARD_CONFIG else
                   bench_config(SHARD_CONFIG, g, ctx, dev, sub, args.warmup, n_pkts=args.n))
        extra["shards"] = dict(summarize(shard_r, g), config=SHARD_CONFIG,
                               roofline_basis="header bytes the reference touches + 6-B "
                                              "descriptor (SURVEY.md §8d)")
        if g.world == 1:  # the metric's other sizes and configs 3'/4 (N=1 only)
            sizes = {}
            for c in SIZES:
                r = shard_r if c == SHARD_CONFIG else bench_config(c, g, ctx, dev, sub,
                                                                     args.warmup, n_pkts=args.n)
                sizes[c] = summarize(r, g)
                if r is not shard_r:
                    r["w"] = None
            extra["sizes"] = sizes
        shard_r["w"] = None if shard_r is not main_r else shard_r["w"]
        if g.world == 1 and main_r["w"]["kind"] == "parse":
            # the same workload served as two RX queues of this GPU (two
            # streams, launches alternating): the chip's rate when launches
            # overlap instead of draining one by one (context for `value`,
            # which stays one queue per GPU)
            q = bench_config(args.config, g, ctx, dev, sub, args.warmup, w=main_r["w"], queues=2,
                             n_pkts=args.n)
            extra["rx_queues"] = {
                "queues": 2, "mpps": round(q["n"] * q["steps"] / q["elapsed"] / 1e6, 2),
                "us_per_launch_wall": round(q["kern_us"], 3),
                "achieved_GBps": round(q["achieved"], 1),
                "frac": round(q["achieved"] / HBM_PEAK_GBS, 4),
                "basis": "algorithmic bytes per launch / wall time per launch (launches overlap)"}
    cpu = None
    if g.world == 1 and not args.no_cpu:
        cpu = cpu_baseline(main_r["w"], args.cpu_seconds)
    emit(args, g, main_r, extra, cpu)
    ctx.close()
    g.close()


def bench_nat64_mbufs(args, w):
    """End-to-end nat64 over rte_mbuf bursts (cgpu_nat64_mbufs, or
    cgpu_nat64_frames over (data_address, data_len) pairs): the device reads
    the frames from the registered mempool, rewrites them and writes the ACT
    frames back into their mbufs, one synchronous call per burst.  6to4 for
    --config nat64; 4to6 for --config nat64_4to6, over the replies to the
    6to4 stream, whose pass (untimed, device-resident) populates the map.
    The call rewrites the mempool in place, so the pool is restored between
    calls, outside the timed region (only the calls are timed).  Prints one
    JSON line."""
    import torch

    from capsule_amd import packets, synth

    ctx = packets.Context(0)
    to6 = args.config == "nat64_4to6"
    direction = "4to6" if to6 else "6to4"
    if to6:  # the replies (host arrays), the map populated by their 6to4 pass
        gw = nat64_4to6_setup(w, ctx, torch.device("cuda", 0))
    n = len(w["off"])
    room = 2048  # DPDK's default data room: 4to6 needs the tailroom
    stride = (128 + 128 + room + 63) // 64 * 64
    pinned, pool = synth.pinned_buffer(stride * n)
    mem, mbufs = synth.mbuf_pool(w["arena"], w["off"], w["len"], mem=pool, room=room)
    orig = mem.copy()
    reg = packets.HostRegion.of(ctx, mem)
    if not to6:
        gw = packets.Nat64Gateway(ctx, capacity_log2=PORTMAP_LOG2)
    B = min(args.burst, n)
    bursts = [mbufs[s:s + B] for s in range(0, n - B + 1, B)]
    frames = args.ingress == "frames"
    if frames:  # (data_address, data_len) pairs, as the RX core hands them over
        fa, fl = synth.mbuf_frames(mem, mbufs)
        tr = synth.mbuf_tailroom(mem, mbufs)
        pairs = [(fa[s:s + B].copy(), fl[s:s + B].copy(), tr[s:s + B].copy())
                 for s in range(0, n - B + 1, B)]

    def call(k):
        if frames:
            a, ln, t = pairs[k % len(pairs)]
            _, d, _ = gw.nat_frames(a, ln, t if to6 else None, direction=direction)
            return d
        return gw.nat_mbufs(bursts[k % len(bursts)], direction)[0]

    # Each call rewrites its burst's objects in place; they are restored
    # between calls, outside the timed region: for bursts of up to 8 Ki
    # mbufs only the burst's own objects (header line + frame), so the
    # restore does not sweep the whole pool through the CPU caches before
    # each call (whose host-side work it would then slow down)
    mb_off = (mbufs.astype(np.int64) - mem.ctypes.data)
    nobj = 128 + 128 + int(w["len"].max()) + 20
    restore = None
    if B <= 8192 and n * nobj <= 1 << 26:
        rel = np.arange(nobj, dtype=np.int64)
        restore = [(mb_off[s:s + B, None] + rel[None, :]).ravel().astype(np.int32)
                   for s in range(0, n - B + 1, B)]

    def reset(k):
        if restore is None:
            np.copyto(mem, orig)
        else:
            idx = restore[k % len(restore)]
            mem[idx] = orig[idx]

    call(0)  # 6to4: first sight of the keys (deferred path), untimed
    reset(0)
    calls, el, acts = 0, 0.0, 0
    while calls < max(4, args.steps // 50) or el < 1.0:
        reset(calls)
        t0 = time.perf_counter()
        disp = call(calls)
        el += time.perf_counter() - t0
        acts += int((disp == 0).sum())
        calls += 1
    print(json.dumps({
        "metric": f"end-to-end Mpps, nat64 {direction} over rte_mbuf bursts (" +
                  ("cgpu_nat64_frames: (data_address, data_len) pairs, frames rewritten in "
                   "place, data_len left to the caller" if frames else
                   "cgpu_nat64_mbufs: zero-copy gather, rewrite, frames written back into the "
                   "mbufs") + ")",
        "value": round(calls * B / el / 1e6, 2), "unit": "Mpps", "config": args.config,
        "ingress": args.ingress, "burst": B, "calls": calls, "act_frac": round(acts / (calls * B), 4),
        "us_per_burst": round(el / calls * 1e6, 1),
        "mempool": f"{n} objects x {stride} B, page-locked, shuffled; 128-B rte_mbuf headers"}),
        flush=True)
    gw.close()
    reg.close()
    ctx.close()


def e2e_mbufs(args):
    """End-to-end rate of rte_mbuf bursts: a DPDK-style mempool of the parse
    workload's frames in page-locked host memory, bursts of --burst mbuf
    pointers through cgpu_parse_mbufs (synchronous: gather -> parse -> results
    in host arrays), one core, one stream.  Prints one JSON line."""
    import torch

    from capsule_amd import _native as N
    from capsule_amd import packets, synth

    torch.cuda.set_device(0)
    w = make_workload(args.config, 0xC0FFEE + 2, n=args.n)
    if args.config in ("nat64", "nat64_4to6") and args.ingress in ("zero_copy", "frames"):
        return bench_nat64_mbufs(args, w)
    if w["kind"] != "parse":
        raise SystemExit("--ingress applies to the parse configs, and zero_copy / frames to "
                         "nat64 and nat64_4to6")
    n = len(w["off"])
    ctx = packets.Context(0)
    stride = (128 + 128 + int(w["len"].max()) + 63) // 64 * 64
    pinned, pool = synth.pinned_buffer(stride * n)
    mem, mbufs = synth.mbuf_pool(w["arena"], w["off"], w["len"], mem=pool)
    reg = packets.HostRegion.of(ctx, mem)
    ingress = {"stage": N.INGRESS_STAGE, "zero_copy": N.INGRESS_ZERO_COPY,
               "frames": N.INGRESS_ZERO_COPY}[args.ingress]
    B = min(args.burst, n)
    bursts = [mbufs[s:s + B] for s in range(0, n - B + 1, B)]
    outs = [(np.zeros(B, np.uint32), np.zeros(B, np.uint32), np.zeros(B, np.uint64))
            for _ in range(2)]
    L = N.lib()
    if args.ingress == "frames":
        # the RX core hands over (data_address, data_len) pairs, read from the
        # mbuf headers it has just written (outside the timed calls)
        fa, fl = synth.mbuf_frames(mem, mbufs)
        pairs = [(fa[s:s + B].copy(), fl[s:s + B].copy()) for s in range(0, n - B + 1, B)]

    def call(k):  # the device-resident config's work: parse + checksums + hash
        meta, cs, fh = outs[k & 1]
        if args.ingress == "frames":
            a, ln = pairs[k % len(pairs)]
            N.check(L.cgpu_parse_frames(ctx.handle, a.ctypes.data, ln.ctypes.data, B, w["flags"],
                                        ingress, meta.ctypes.data, cs.ctypes.data, fh.ctypes.data,
                                        None), "cgpu_parse_frames")
            return
        mb = bursts[k % len(bursts)]
        N.check(L.cgpu_parse_mbufs(ctx.handle, mb.ctypes.data, B, w["flags"], ingress,
                                   meta.ctypes.data, cs.ctypes.data, fh.ctypes.data, None),
                "cgpu_parse_mbufs")

    if args.inflight == 2:
        if args.ingress != "frames":
            raise SystemExit("--inflight 2 applies to --ingress frames")
        pend = []

        def call(k):  # submit burst k, then wait for burst k - 1 (double buffering)
            a, ln = pairs[k % len(pairs)]
            pend.append(packets.parse_frames_submit(ctx, a, ln, w["flags"], out=outs[k & 1]))
            if len(pend) == 2:
                packets.parse_frames_wait(ctx, pend.pop(0))

    for k in range(3):
        call(k)
    calls, t0 = 0, time.perf_counter()
    while calls < max(4, args.steps // 10) or time.perf_counter() - t0 < 2.0:
        call(calls)
        calls += 1
    if args.inflight == 2:
        while pend:
            packets.parse_frames_wait(ctx, pend.pop(0))
    el = time.perf_counter() - t0
    print(json.dumps({
        "metric": "end-to-end Mpps, rte_mbuf bursts from a host mempool ("
                  + ("cgpu_parse_frames: (data_address, data_len) pairs, zero-copy"
                     if args.ingress == "frames" else "cgpu_parse_mbufs") + ")",
        "value": round(calls * B / el / 1e6, 2), "unit": "Mpps", "config": args.config,
        "ingress": args.ingress, "burst": B, "calls": calls, "inflight": args.inflight,
        "us_per_burst": round(el / calls * 1e6, 1),
        "mempool": f"{n} objects x {stride} B, page-locked, shuffled; 128-B rte_mbuf headers"}),
        flush=True)
    reg.close()
    ctx.close()


def numa_report(dev, tensors):
    """NUMA placement for the end-to-end rates: the GPU's node (sysfs) and the
    nodes of a sample of pages of each pinned host tensor (move_pages(2) with
    no target nodes reports where each page lives).  A pinned buffer on the
    node away from the GPU's PCIe root crosses the socket link on every DMA."""
    import ctypes
    import torch

    out = {}
    try:
        p = torch.cuda.get_device_properties(dev)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            out["gpu_node"] = int(f.read())
    except (OSError, ValueError, RuntimeError):
        out["gpu_node"] = None
    libc = ctypes.CDLL(None, use_errno=True)
    page = os.sysconf("SC_PAGE_SIZE")
    for name, t in tensors.items():
        nb = t.numel() * t.element_size()
        k = max(1, min(64, nb // page))
        addrs = (ctypes.c_void_p * k)(*[(t.data_ptr() + (nb * j // k)) & ~(page - 1) for j in range(k)])
        status = (ctypes.c_int * k)()
        if libc.syscall(279, 0, ctypes.c_ulong(k), addrs, None, status, 0) != 0:  # SYS_move_pages
            out[name] = f"move_pages errno {ctypes.get_errno()}"
            continue
        hist = {}
        for v in status:
            hist[str(v)] = hist.get(str(v), 0) + 1
        out[name] = hist
    return out


def e2e(args):
    """End-to-end rate with the batch starting and ending in host memory.

    The burst sits in a pinned host arena (where a NIC would have DMA'd it);
    each step copies arena + descriptors host->device on one stream, parses on
    a second, copies meta/hash (and the nat64 output frames) device->host on a
    third, with three batches in flight.  Prints one JSON line (not the
    driver's metric line).
    """
    import torch

    from capsule_amd import packets

    if args.config == "nat64_cold":
        raise SystemExit("--e2e: nat64_cold is a device-resident timing of the map's first pass")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # the pipeline's streams first, before the library's context stream and
    # any setup work (the order in which streams are created and first used
    # decides which of them share a hardware queue)
    # Two streams: the upload and the kernel share one (the kernel is 1-2 % of
    # a batch's upload), the download has its own.  With three, the box's 4
    # hardware queues (GPU_MAX_HW_QUEUES, HIP's default) could put two of
    # the pipeline's streams on one queue: 4to6 then ran its uploads and
    # downloads one after the other, 107 against 182 Mpps.
    nstreams = int(os.environ.get("CGPU_E2E_STREAMS", "2"))
    h2d, d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    comp = h2d if nstreams == 2 else torch.cuda.Stream(dev)
    if os.environ.get("CGPU_E2E_STREAMS_LATE") == "1":  # the round-3 order (A/B only)
        h2d = comp = d2h = None
    w = make_workload(args.config, 0xC0FFEE + 2, n=args.n)
    n = len(w["off"])
    ctx = packets.Context(0)
    gw = nat64_4to6_setup(w, ctx, dev) if w["kind"] == "nat64_4to6" else None
    host = dict(arena=torch.from_numpy(w["arena"]).pin_memory(),
                off=torch.from_numpy(w["off"].view(np.int32)).pin_memory(),
                len=torch.from_numpy(w["len"].view(np.int16)).pin_memory())
    D = 3
    bufs = [packets.PacketBatch(torch.empty_like(host["arena"], device=dev),
                                torch.empty_like(host["off"], device=dev),
                                torch.empty_like(host["len"], device=dev)) for _ in range(D)]
    if h2d is None:
        h2d, d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        comp = h2d if nstreams == 2 else torch.cuda.Stream(dev)
    if w["kind"] == "parse":
        outs = [packets.ParseBuffers(n, dev, csum=False) for _ in range(D)]
        host_out = [(torch.empty(n, dtype=torch.int32, pin_memory=True),
                     torch.empty(n, dtype=torch.int64, pin_memory=True)) for _ in range(D)]
        launch = [packets.ParseLauncher(ctx, bufs[d], outs[d], w["flags"], comp) for d in range(D)]

        def back(d):
            host_out[d][0].copy_(outs[d].meta, non_blocking=True)
            host_out[d][1].copy_(outs[d].flow_hash, non_blocking=True)
        down_bytes = 12 * n
    else:
        direction = "4to6" if gw is not None else "6to4"
        gw = gw or packets.Nat64Gateway(ctx, capacity_log2=PORTMAP_LOG2)
        nat = [(torch.empty_like(bufs[d].arena), bufs[d].off,
                torch.empty(n, dtype=torch.int16, device=dev),
                torch.empty(n, dtype=torch.uint8, device=dev),
                torch.empty(n, dtype=torch.uint8, device=dev)) for d in range(D)]
        host_out = [(torch.empty_like(host["arena"], pin_memory=True),
                     torch.empty(n, dtype=torch.int16, pin_memory=True)) for _ in range(D)]
        launch = [packets.Nat64Launcher(gw, bufs[d], nat[d], comp, direction) for d in range(D)]

        def back(d):
            host_out[d][0].copy_(nat[d][0], non_blocking=True)
            host_out[d][1].copy_(nat[d][2], non_blocking=True)
        down_bytes = len(w["arena"]) + 2 * n
    up_bytes = len(w["arena"]) + 6 * n
    ev_up = [torch.cuda.Event() for _ in range(D)]
    ev_comp = [torch.cuda.Event() for _ in range(D)]
    ev_down = [torch.cuda.Event() for _ in range(D)]
    # phase clocks of the timed steps (start / end of each stream's part):
    # how long each copy and the kernel take, and whether they overlap
    T = 10
    ph = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(T)]
    tr = {"k0": None}

    def mark(k, j, s):
        if tr["k0"] is not None and 0 <= k - tr["k0"] < T:
            ph[k - tr["k0"]][j].record(s)

    def step(k):
        d = k % D
        with torch.cuda.stream(h2d):
            h2d.wait_event(ev_down[d])  # buffer d free again (its results went home)
            mark(k, 0, h2d)
            bufs[d].arena.copy_(host["arena"], non_blocking=True)
            bufs[d].off.copy_(host["off"], non_blocking=True)
            bufs[d].len.copy_(host["len"], non_blocking=True)
            mark(k, 1, h2d)
            ev_up[d].record(h2d)
        comp.wait_event(ev_up[d])
        mark(k, 2, comp)
        launch[d]()
        mark(k, 3, comp)
        ev_comp[d].record(comp)
        with torch.cuda.stream(d2h):
            d2h.wait_event(ev_comp[d])
            mark(k, 4, d2h)
            back(d)
            mark(k, 5, d2h)
            ev_down[d].record(d2h)

    for d in range(D):
        ev_down[d].record(d2h)
    for t in ph:  # create the timing events' HIP objects before the timed region
        for e in t:
            e.record(comp)
    kw = max(3, args.warmup // 10)
    for k in range(kw):
        step(k)
    torch.cuda.synchronize(dev)
    steps = max(10, args.steps // 10)
    tr["k0"] = kw + steps // 2
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    n_tr = min(T, steps - steps // 2)

    def mean_ms(j0, j1):
        return round(sum(ph[t][j0].elapsed_time(ph[t][j1]) for t in range(n_tr)) / n_tr, 3)

    phases = {"h2d_ms": mean_ms(0, 1), "kernel_ms": mean_ms(2, 3), "d2h_ms": mean_ms(4, 5),
              "h2d_start_to_next_ms": round(sum(ph[t][0].elapsed_time(ph[t + 1][0])
                                                for t in range(n_tr - 1)) / max(1, n_tr - 1), 3)}
    print(json.dumps({
        "metric": "end-to-end Mpps, host-resident batches (pinned H2D + kernel + D2H)",
        "value": round(n * steps / el / 1e6, 2), "unit": "Mpps", "config": args.config,
        "steps": steps, "packets_per_step": n, "ms_per_step": round(el / steps * 1e3, 3),
        "h2d_GBps": round(up_bytes * steps / el / 1e9, 2),
        "d2h_GBps": round(down_bytes * steps / el / 1e9, 2),
        "batches_in_flight": D, "streams": nstreams, "phases": phases,
        "numa": numa_report(dev, {"h2d_src": host["arena"], "d2h_dst": host_out[0][0]})}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
