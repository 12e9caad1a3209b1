"""Burst-level mirror of capsule's batch combinators over the device path.

The reference pulls one packet at a time through a chain of closures
(`Batch::next`, core/src/batch/mod.rs:122-135); each step returns a
`Disposition` -- Act (keep going), Drop, or Abort (an `Err`) (mod.rs:54-107).
Here a step sees a whole burst: the device image of the packets
(`PacketBatch`) plus per-packet dispositions, and a closure returns
per-packet tensors instead of one value.  The semantics are the reference's:

- only Act packets reach a step; Drop and Abort pass through untouched
  (mod.rs:137-160, filter_map.rs:73-81);
- a failing typed parse (`p.parse::<Ipv4>()?`) aborts the packet with the
  reference's error (`status`, CGPU_PKT_*);
- `group_by` routes Act packets to arms by a selector key, in batch order,
  with a catch-all arm (group_by.rs:143-200); without one, unmatched packets
  pass through as Act (group_by.rs:186-200);
- `replace` follows each Act packet with its replacement and drops the
  original (replace.rs); inside a group_by arm the outputs stay after the
  input packet they came from (group_by_fanout, mod.rs:672-696);
- `send` counts what leaves the pipeline: processed (transmitted + emitted),
  dropped, errors (send.rs:95-118), and hands the Act packets to the
  transmit side.

Device work: `parse` runs cgpu_parse_batch, `group_by` cgpu_group_by;
dispositions and the arm merge are plain tensor plumbing.
"""
import torch

from . import _native as N
from . import packets

ACT, DROP, ABORT = N.ACT, N.DROP, N.ABORT
EMIT = 3  # Disposition::Emit: already sent through another PacketTx (mod.rs:60)


def _u32_to_i32(x):
    x = x & 0xFFFFFFFF
    return torch.where(x >= 1 << 31, x - (1 << 32), x).to(torch.int32)


class Burst:
    """One burst in flight: `batch` (device PacketBatch), `disp` (u8 [n]
    Disposition), `status` (u8 [n], why an Abort happened: CGPU_PKT_*, 0
    otherwise), `parsed` (the last ParsedBatch, or None) and `origin` (int64
    [n], the index of the input packet each one descends from -- replace
    emits two packets for one)."""

    def __init__(self, batch, disp=None, status=None, parsed=None, origin=None):
        n, dev = batch.n, batch.arena.device
        self.batch = batch
        self.disp = disp if disp is not None else torch.full((n,), ACT, dtype=torch.uint8, device=dev)
        self.status = status if status is not None else torch.zeros(n, dtype=torch.uint8, device=dev)
        self.parsed = parsed
        self.origin = origin if origin is not None else torch.arange(n, device=dev)

    @property
    def n(self):
        return self.batch.n

    def act(self):
        return self.disp == ACT

    def dispositions(self):
        return self.disp.cpu().tolist()

    def take(self, idx):
        """The sub-burst of packets `idx` (a device index tensor), in that order."""
        idx = idx.long()
        parsed = None
        if self.parsed is not None:
            r = self.parsed
            parsed = packets.ParsedBatch(*(t[idx] if t is not None else None for t in
                                           (r.meta, r.csum, r.flow_hash, r.fields, r.ext)))
        return Burst(packets.PacketBatch(self.batch.arena, self.batch.off[idx], self.batch.len[idx]),
                     self.disp[idx], self.status[idx], parsed, self.origin[idx])

    @staticmethod
    def concat(bursts):
        """One burst holding `bursts` back to back; distinct arenas are
        appended into one (64-B aligned), their offsets rebased."""
        arenas, offs, base = [], [], 0
        seen = {}
        for b in bursts:
            a = b.batch.arena
            key = (a.data_ptr(), a.numel())
            if key not in seen:
                seen[key] = base
                arenas.append(a)
                pad = (-a.numel()) % 64
                if pad:
                    arenas.append(torch.zeros(pad, dtype=torch.uint8, device=a.device))
                base += a.numel() + pad
            offs.append(_u32_to_i32(b.batch.off.long() + seen[key]) if seen[key] else b.batch.off)
        arena = arenas[0] if len(arenas) == 1 else torch.cat(arenas)
        parsed = None
        rs = [b.parsed for b in bursts]
        if all(r is not None for r in rs):
            cols = []
            for name in ("meta", "csum", "flow_hash", "fields", "ext"):
                ts = [getattr(r, name) for r in rs]
                cols.append(torch.cat(ts) if all(t is not None for t in ts) else None)
            parsed = packets.ParsedBatch(*cols)
        return Burst(packets.PacketBatch(arena, torch.cat(offs), torch.cat([b.batch.len for b in bursts])),
                     torch.cat([b.disp for b in bursts]), torch.cat([b.status for b in bursts]),
                     parsed, torch.cat([b.origin for b in bursts]))


class Batch:
    """Base of the combinators: `next_burst()` yields Bursts, or None when
    the source is exhausted (`Batch::next` returning None)."""

    def __init__(self, ctx, upstream=None):
        self.ctx = ctx
        self.upstream = upstream

    def replenish(self):
        if self.upstream is not None:
            self.upstream.replenish()

    def next_burst(self):
        b = self.upstream.next_burst()
        return None if b is None else self.apply(b)

    def apply(self, burst):  # pragma: no cover - the combinators override it
        return burst

    # --- combinators (core/src/batch/mod.rs:137-300) ---------------------------
    def parse(self, flags=None, fields=False, upto="l4"):
        return Parse(self, flags, fields, upto)

    def map(self, fn):
        return Map(self, fn)

    def filter(self, pred):
        return Filter(self, pred)

    def filter_map(self, fn):
        return FilterMap(self, fn)

    def group_by(self, selector, arms, catch_all=None, n_keys=256):
        return GroupBy(self, selector, arms, catch_all, n_keys)

    def inspect(self, fn):
        return Inspect(self, fn)

    def for_each(self, fn):
        return ForEach(self, fn)

    def replace(self, fn):
        return Replace(self, fn)

    def emit(self, tx):
        return Emit(self, tx)

    def send(self, tx):
        return Send(self, tx)


class Channel:
    """An in-process PacketTx / PacketRx pair (the mpsc channel of the
    reference's tests, rxtx.rs): `transmit` queues a burst, `receive` takes
    the oldest one (an empty list when nothing is queued)."""

    def __init__(self):
        self.q = []

    def transmit(self, packets_):
        self.q.append(packets_)

    append = transmit  # so a Channel can be a Send / Emit target

    def receive(self):
        return self.q.pop(0) if self.q else []


def _size(burst):
    if burst is None:
        return 0
    return burst.n if isinstance(burst, packets.PacketBatch) else len(burst)


class Poll(Batch):
    """`Poll::new(rx)` / `poll_fn(f)` (batch/poll.rs:47-62): `replenish`
    pulls the next burst from the receive side -- a PacketRx (anything with
    `receive()`), a function returning a burst, or an iterator of bursts.
    A burst is a PacketBatch or a list of frames (bytes).

    `target`: packets to gather per replenish.  The reference pulls one
    burst (at most RX_BURST_MAX = 32 mbufs, dpdk/port.rs:149-171) per
    replenish, which is `target=1`; a device call costs a fixed ~20 us
    (DESIGN.md §8), so the GPU seam keeps pulling until it holds `target`
    packets or a pull brings nothing (the queue is drained: nothing waits for
    packets that have not arrived), and runs the pulled bursts as one, in
    arrival order."""

    def __init__(self, ctx, rx, device="cuda:0", target=1):
        super().__init__(ctx)
        if hasattr(rx, "receive"):
            self.pull = rx.receive
        elif callable(rx):
            self.pull = rx
        else:
            it = iter(rx)
            self.pull = lambda: next(it, None)
        self.device = device
        self.target = max(1, int(target))
        self.pending = None
        self.pulls = 0  # receive() calls so far

    def replenish(self):
        parts, total = [], 0
        while total < self.target:
            nxt = self.pull()
            self.pulls += 1
            if _size(nxt) == 0:
                break
            parts.append(nxt)
            total += _size(nxt)
        if not parts:
            self.pending = None
            return
        if all(not isinstance(p, packets.PacketBatch) for p in parts):
            nxt = packets.PacketBatch.from_frames([f for p in parts for f in p], self.device)
        else:
            nxt = packets.PacketBatch.concat(
                [p if isinstance(p, packets.PacketBatch) else
                 packets.PacketBatch.from_frames(p, self.device) for p in parts])
        self.pending = Burst(nxt)

    def next_burst(self):
        b, self.pending = self.pending, None
        return b


# the layer each failing status belongs to (include/capsule_gpu.h)
_LAYER = {**{s: 2 for s in ("ETH_BAD_OFFSET", "ETH_OUT_OF_BUFFER")},
          **{s: 3 for s in ("NOT_IPV4", "NOT_IPV6", "NOT_IP", "L3_BAD_OFFSET", "L3_OUT_OF_BUFFER",
                            "EXT_BAD_OFFSET", "EXT_OUT_OF_BUFFER", "SRH_INCONSISTENT")}}


class Parse(Batch):
    """The typed parse chain `p.parse::<Ethernet>()?.parse::<Ipv4|Ipv6>()?
    .parse::<Udp|Tcp|...>()?` for every Act packet; a failing step aborts
    the packet with its status (the `?` of a map / filter_map closure).
    upto = "l2" / "l3" / "l4": the chain stops after Ethernet, IP or L4,
    so only failures of those layers abort."""

    def __init__(self, upstream, flags, fields, upto):
        super().__init__(upstream.ctx, upstream)
        self.flags = packets.parse_flags() if flags is None else flags
        self.fields = fields
        depth = {"l2": 2, "l3": 3, "l4": 4}[upto]
        lut = torch.zeros(256, dtype=torch.bool)
        for code, name in enumerate(N.PKT_STATUS):
            lut[code] = code != 0 and _LAYER.get(name, 4) <= depth
        self.aborts = lut

    def apply(self, b):
        r = packets.parse(self.ctx, b.batch, flags=self.flags, fields=self.fields)
        st = (r.meta & 0xFF).to(torch.uint8)
        fail = b.act() & self.aborts.to(st.device)[st.long()]
        b.status = torch.where(fail, st, b.status)
        b.disp = torch.where(fail, torch.full_like(b.disp, ABORT), b.disp)
        b.parsed = r
        return b


def _acting(b):
    """(indices, sub-burst) of the Act packets: closures see only those, like
    `Disposition::map` (mod.rs:74-86).  (None, None) when there are none."""
    idx = torch.nonzero(b.act()).flatten()
    return (idx, b.take(idx)) if idx.numel() else (None, None)


def _abort(b, idx, st):
    """Abort b's packets idx where the u8 status st (one per idx) is nonzero."""
    st = st.to(torch.uint8)
    bad = st != 0
    b.status[idx[bad]] = st[bad]
    b.disp[idx[bad]] = ABORT


class Map(Batch):
    """`map(|p| -> Result<T>)` (map.rs): fn(burst of the Act packets) may
    change them in place (their bytes live in the shared arena) and returns
    None or a u8 status per packet; a nonzero status aborts it."""

    def __init__(self, upstream, fn):
        super().__init__(upstream.ctx, upstream)
        self.fn = fn

    def apply(self, b):
        idx, sub = _acting(b)
        if idx is not None:
            st = self.fn(sub)
            if st is not None:
                _abort(b, idx, st)
        return b


class Filter(Batch):
    """`filter(|p| bool)` (filter.rs): pred(burst of the Act packets) returns
    a bool per packet; False drops it."""

    def __init__(self, upstream, pred):
        super().__init__(upstream.ctx, upstream)
        self.pred = pred

    def apply(self, b):
        idx, sub = _acting(b)
        if idx is not None:
            keep = torch.as_tensor(self.pred(sub), device=idx.device).to(torch.bool).expand(idx.numel())
            b.disp[idx[~keep]] = DROP
        return b


class FilterMap(Batch):
    """`filter_map(|p| -> Result<Either<T>>)` (filter_map.rs:73-81): fn(burst
    of the Act packets) returns a u8 Disposition per packet (Keep -> ACT,
    Drop -> DROP, Err -> ABORT), or (dispositions, status) to say why."""

    def __init__(self, upstream, fn):
        super().__init__(upstream.ctx, upstream)
        self.fn = fn

    def apply(self, b):
        idx, sub = _acting(b)
        if idx is None:
            return b
        out = self.fn(sub)
        d, st = out if isinstance(out, tuple) else (out, None)
        d = d.to(torch.uint8)
        b.disp[idx] = d
        if st is not None:
            ab = d == ABORT
            b.status[idx[ab]] = st.to(torch.uint8)[ab]
        return b


class Inspect(Batch):
    """`inspect(|p| ...)` (inspect.rs): a side effect on the Act packets."""

    def __init__(self, upstream, fn):
        super().__init__(upstream.ctx, upstream)
        self.fn = fn

    def apply(self, b):
        idx, sub = _acting(b)
        if idx is not None:
            self.fn(sub)
        return b


class ForEach(Inspect):
    """`for_each(|p| -> Result<()>)` (for_each.rs): like inspect, but a
    nonzero status aborts the packet."""

    def apply(self, b):
        idx, sub = _acting(b)
        if idx is not None:
            st = self.fn(sub)
            if st is not None:
                _abort(b, idx, st)
        return b


class _Arm(Batch):
    """The source of one group_by arm: the arm's sub-burst."""

    def __init__(self, ctx):
        super().__init__(ctx)
        self.burst = None

    def replenish(self):
        pass

    def next_burst(self):
        b, self.burst = self.burst, None
        return b


class GroupBy(Batch):
    """`group_by(selector, compose!{ k => |group| ..., _ => |group| ... })`
    (group_by.rs:143-200).  selector(burst) returns a u8 key per packet;
    `arms` maps a key (or a tuple of keys: `k1, k2 => ...`) to a function
    building the arm's pipeline from its source; `catch_all` builds the `_`
    arm (None: unmatched packets pass through as Act).  Act packets are
    partitioned on the device (cgpu_group_by, stable) and each arm runs on
    its sub-burst; the dispositions are merged back in batch order."""

    def __init__(self, upstream, selector, arms, catch_all, n_keys):
        super().__init__(upstream.ctx, upstream)
        self.selector = selector
        self.n_keys = n_keys
        self.routes = []  # (keys, source, pipeline)
        for keys, build in arms.items():
            keys = keys if isinstance(keys, tuple) else (keys,)
            src = _Arm(self.ctx)
            self.routes.append((keys, src, build(src)))
        self.catch_all = None
        if catch_all is not None:
            src = _Arm(self.ctx)
            self.catch_all = (src, catch_all(src))

    def apply(self, b):
        key = self.selector(b).to(torch.uint8)
        # arm number per packet: routes in order, then the catch-all /
        # pass-through arm; packets that are not Act go to a final arm of their own
        n_arms = len(self.routes) + 2
        lut = torch.full((self.n_keys,), len(self.routes), dtype=torch.uint8, device=key.device)
        for a, (keys, _, _) in enumerate(self.routes):
            for k in keys:
                lut[int(k)] = a
        arm = lut[key.long()]
        arm = torch.where(b.act(), arm, torch.full_like(arm, n_arms - 1))
        g = packets.group_by(self.ctx, arm, n_arms, by="key")
        off = g.off.cpu().tolist()
        pipes = [p for _, _, p in self.routes] + [self.catch_all[1] if self.catch_all else None, None]
        srcs = [s for _, s, _ in self.routes] + [self.catch_all[0] if self.catch_all else None, None]
        outer = b.origin
        b.origin = torch.arange(b.n, device=outer.device)
        outs = []
        for a in range(n_arms):
            if off[a] == off[a + 1]:
                continue
            sub = b.take(g.idx[off[a]:off[a + 1]])
            if pipes[a] is not None:
                srcs[a].burst = sub
                sub = pipes[a].next_burst()
            outs.append(sub)
        if not outs:
            b.origin = outer
            return b
        # back into batch order: every output after the packet it came from,
        # an arm's outputs for one packet in the order the arm produced them
        merged = Burst.concat(outs)
        order = torch.sort(merged.origin, stable=True).indices
        r = merged.take(order)
        r.origin = outer[r.origin]
        return r


class Replace(Batch):
    """`replace(|p| -> Result<T>)` (replace.rs): every Act packet is followed
    by a new packet built from it; the original becomes Drop.  fn(burst)
    returns the new frames, one per packet of the burst it is given (a list
    of bytes or a PacketBatch); it sees only the Act packets.  An error is
    expressed as (frames, status) with a nonzero status aborting that packet
    instead (no replacement)."""

    def __init__(self, upstream, fn):
        super().__init__(upstream.ctx, upstream)
        self.fn = fn

    def apply(self, b):
        act, sub = _acting(b)
        if act is None:
            return b
        out = self.fn(sub)
        frames, st = out if isinstance(out, tuple) else (out, None)
        if not isinstance(frames, packets.PacketBatch):
            frames = packets.PacketBatch.from_frames(frames, b.batch.arena.device)
        rep = Burst(frames, origin=b.origin[act])
        orig = Burst(b.batch, b.disp.clone(), b.status.clone(), None, b.origin)
        orig.disp[act] = DROP
        pos = torch.arange(b.n, device=act.device)
        rkey, okey = 2 * act, 2 * pos + 1
        if st is not None:  # failed replacements: the original aborts, nothing new
            st = st.to(torch.uint8)
            bad = st != 0
            orig.disp[act[bad]] = ABORT
            orig.status[act[bad]] = st[bad]
            keep = torch.nonzero(~bad).flatten()
            rep, rkey = rep.take(keep), rkey[keep]
        merged = Burst.concat([rep, orig])
        return merged.take(torch.sort(torch.cat([rkey, okey]), stable=True).indices)


class Emit(Batch):
    """`emit(tx)` (emit.rs): the Act packets are sent to `tx` right away and
    become Emit."""

    def __init__(self, upstream, tx):
        super().__init__(upstream.ctx, upstream)
        self.tx = tx

    def apply(self, b):
        act = torch.nonzero(b.act()).flatten()
        if act.numel():
            s = b.take(act).batch
            self.tx.append(s)
            b.disp[act] = EMIT
        return b


class Send(Batch):
    """`send(tx)` (send.rs:85-119): the Act packets go to `tx` (a list the
    transmitted PacketBatches are appended to), Drop packets are freed, and
    the counters are updated like the reference's metrics (send.rs:104-110):
    processed = transmitted + emitted, dropped, errors (= aborted)."""

    def __init__(self, upstream, tx):
        super().__init__(upstream.ctx, upstream)
        self.tx = tx
        self.transmitted = self.emitted = self.dropped = self.aborted = 0

    @property
    def processed(self):
        return self.transmitted + self.emitted

    @property
    def errors(self):
        return self.aborted

    def apply(self, b):
        counts = torch.bincount(b.disp.long(), minlength=4).cpu().tolist()
        self.transmitted += counts[ACT]
        self.dropped += counts[DROP]
        self.aborted += counts[ABORT]
        self.emitted += counts[EMIT]
        keep = torch.nonzero(b.act()).flatten()
        if keep.numel():
            self.tx.append(b.take(keep).batch)
        return b

    def run_once(self):
        """One burst: replenish, then consume it (Pipeline::run_once).
        Returns False when the source is exhausted."""
        self.replenish()
        return self.next_burst() is not None

    def run(self):
        """Drain the source."""
        while self.run_once():
            pass
