"""Host-side mirror of the reference's packet API for the GPU hot path.

The reference processes one `Mbuf` at a time through typed parses
(`packet.parse::<Ethernet>()?.parse::<Ipv4>()?.parse::<Udp4>()?`,
core/src/packets/mod.rs:178) inside batch combinators (core/src/batch/).
Here the unit is a *burst*: a `PacketBatch` is the device image of many
single-segment mbufs (an arena of frame bytes plus per-packet offset and
data_len, core/src/dpdk/mbuf.rs:196-205), and one call runs the whole chain
for every packet on the GPU.  Per-packet `Result`s become a status code per
packet carrying the same distinctions as the reference's errors
(`BufferError::{BadOffset, OutOfBuffer}` mbuf.rs:85-98, "not an IPv4
packet." v4.rs:430, ...), see `ParsedBatch.error()`.

Device memory and streams come from torch (plumbing only); every byte of
packet work runs in the HIP kernels behind include/capsule_gpu.h.
"""
import ctypes

import numpy as np
import torch

from . import _native as N

_STATUS_MSG = {
    N.PKT["ETH_BAD_OFFSET"]: "BadOffset",
    N.PKT["ETH_OUT_OF_BUFFER"]: "OutOfBuffer",
    N.PKT["L3_BAD_OFFSET"]: "BadOffset",
    N.PKT["L3_OUT_OF_BUFFER"]: "OutOfBuffer",
    N.PKT["L4_BAD_OFFSET"]: "BadOffset",
    N.PKT["L4_OUT_OF_BUFFER"]: "OutOfBuffer",
}


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream_handle(stream):
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


class Context:
    """`cgpu_ctx`: one per core thread / RX queue (runtime/core_map.rs:236-293)."""

    def __init__(self, device=0, test_hooks=False):
        if not torch.cuda.is_available():
            raise RuntimeError("capsule_amd: no HIP device visible")
        self.device = torch.device("cuda", device)
        # test_hooks=True: a context of the test build (tests only), whose
        # objects all go through that library
        self.L = N.lib(test=test_hooks)
        self._h = ctypes.c_void_p()
        N.check(self.L.cgpu_ctx_create(device, ctypes.byref(self._h)), "cgpu_ctx_create")

    @property
    def handle(self):
        return self._h

    def check(self, stream=None):
        """`cgpu_ctx_check`: synchronise `stream` (torch's current one by
        default) and raise CgpuError(EIO) if a kernel of this context set the
        device error word since the last check."""
        N.check(self.L.cgpu_ctx_check(self._h, _stream_handle(stream)), "cgpu_ctx_check")

    def close(self):
        if self._h:
            self.L.cgpu_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PacketBatch:
    """Device image of a burst of mbufs: arena (u8), off (u32), len (u16)."""

    def __init__(self, arena, off, length):
        assert arena.dtype == torch.uint8 and off.dtype == torch.int32
        assert length.dtype == torch.int16 and off.numel() == length.numel()
        self.arena, self.off, self.len = arena, off, length

    @property
    def n(self):
        return self.off.numel()

    @classmethod
    def from_numpy(cls, arena, off, length, device):
        """Copy a host batch (np.uint8 arena, np.uint32 off, np.uint16 len)."""
        a = torch.from_numpy(np.ascontiguousarray(arena, dtype=np.uint8)).to(device)
        o = torch.from_numpy(np.ascontiguousarray(off, dtype=np.uint32).view(np.int32)).to(device)
        ln = torch.from_numpy(np.ascontiguousarray(length, dtype=np.uint16).view(np.int16)).to(device)
        return cls(a, o, ln)

    @classmethod
    def from_frames(cls, frames, device, slot=64):
        """Pack a list of byte strings at `slot`-aligned offsets."""
        from .synth import pack_frames

        return cls.from_numpy(*pack_frames(frames, slot), device)

    @classmethod
    def concat(cls, parts):
        """Bursts laid end to end (arenas concatenated, offsets moved), in
        order: the device image of the mbufs of several RX bursts."""
        if len(parts) == 1:
            return parts[0]
        arenas, offs, base = [], [], 0
        for p in parts:
            arenas.append(p.arena)
            o = p.off.to(torch.int64) & 0xFFFFFFFF
            offs.append(o + base)
            base += p.arena.numel()
        if base > 0xFFFF0000:
            raise ValueError("concatenated arena past 4 GiB")
        off = torch.cat(offs)
        off = torch.where(off >= 1 << 31, off - (1 << 32), off).to(torch.int32)
        return cls(torch.cat(arenas), off, torch.cat([p.len for p in parts]))

    def cbatch(self):
        b = N.Batch()
        b.arena = self.arena.data_ptr()
        b.arena_len = self.arena.numel()
        b.off = self.off.data_ptr()
        b.len = self.len.data_ptr()
        b.n = self.n
        return b

    def frame(self, i):
        o = int(self.off[i].item()) & 0xFFFFFFFF
        ln = int(self.len[i].item()) & 0xFFFF
        return bytes(self.arena[o : o + ln].cpu().numpy())


class ParsedBatch:
    """SoA result of `parse`: meta, csum, flow_hash, fields (device tensors)."""

    def __init__(self, meta, csum, flow_hash, fields, ext=None):
        self.meta, self.csum, self.flow_hash, self.fields = meta, csum, flow_hash, fields
        self.ext = ext  # [n, 48] uint8 extension records (CGPU_F_V6_EXT), or None

    def status(self):
        return self.meta & 0xFF

    def ok(self):
        return self.status() == 0

    def ip_csum(self):
        return self.csum & 0xFFFF

    def l4_csum(self):
        return (self.csum >> 16) & 0xFFFF

    def error(self, i):
        """Reference error text of packet i (None when every layer parsed)."""
        s = int(self.meta[i].item()) & 0xFF
        if s == 0:
            return None
        msg = N.lib().cgpu_pkt_status_str(s).decode()
        return _STATUS_MSG.get(s, msg) if s in _STATUS_MSG else msg

    def fields_numpy(self):
        if self.fields is None:
            return None
        raw = self.fields.cpu().numpy()
        return raw.view(np.dtype(N.HDR_RECORD_FIELDS)).reshape(-1)


def parse_flags(accept=N.F_ACCEPT_ALL, csum_ip=True, csum_l4=True, flow_hash=True):
    f = accept
    if csum_ip:
        f |= N.F_CSUM_IP
    if csum_l4:
        f |= N.F_CSUM_L4
    if flow_hash:
        f |= N.F_FLOW_HASH
    return f


class ParseBuffers:
    """Preallocated outputs for repeated `parse` calls on same-sized bursts.

    csum=False: verify-only checksums (the CSUM_OK bits of meta are still
    set; the computed values are not stored)."""

    def __init__(self, n, device, fields=False, csum=True, ext=False):
        self.ext = (torch.empty((n, N.EXT_RECORD_SIZE), dtype=torch.uint8, device=device)
                    if ext else None)
        self.meta = torch.empty(n, dtype=torch.int32, device=device)
        self.csum = torch.empty(n, dtype=torch.int32, device=device) if csum else None
        self.flow_hash = torch.empty(n, dtype=torch.int64, device=device)
        self.fields = (torch.empty((n, N.HDR_RECORD_SIZE), dtype=torch.uint8, device=device)
                       if fields else None)


def parse(ctx, batch, flags=None, fields=False, out=None, stream=None, ext=False):
    """Batched Ethernet -> Ipv4/Ipv6 -> Udp/Tcp parse + checksums + flow hash.

    Mirrors `parse::<Ethernet>()` (ethernet.rs:279) -> `parse::<Ipv4|Ipv6>()`
    (v4.rs:427, v6/mod.rs:274) -> `parse::<Udp|Tcp>()` (udp.rs:287, tcp.rs:558),
    plus `compute_checksum` evaluated on the bytes as they are and the hash of
    `flow()`.  Asynchronous on `stream` (torch's current stream by default).
    ext=True (with N.F_V6_EXT in flags): also the IPv6 extension records.
    """
    if flags is None:
        flags = parse_flags()
    n = batch.n
    if out is None:
        out = ParseBuffers(n, batch.arena.device, fields, ext=ext)
    po = N.ParseOut()
    po.meta = out.meta.data_ptr()
    po.csum = out.csum.data_ptr() if out.csum is not None else None
    po.flow_hash = out.flow_hash.data_ptr()
    po.fields = out.fields.data_ptr() if (fields and out.fields is not None) else None
    po.ext = out.ext.data_ptr() if (ext and out.ext is not None) else None
    cb = batch.cbatch()
    rc = ctx.L.cgpu_parse_batch(ctx.handle, ctypes.byref(cb), flags, ctypes.byref(po),
                                  _stream_handle(stream))
    N.check(rc, "cgpu_parse_batch")
    return ParsedBatch(out.meta[:n], out.csum[:n] if out.csum is not None else None,
                       out.flow_hash[:n],
                       out.fields[:n] if (fields and out.fields is not None) else None,
                       out.ext[:n] if (ext and out.ext is not None) else None)


def parse_host(ctx, frames, flags=None, fields=False):
    """Host-memory variant (the DPDK seam): frames is a list of bytes."""
    if flags is None:
        flags = parse_flags()
    n = len(frames)
    bufs = [ctypes.create_string_buffer(bytes(f), max(1, len(f))) for f in frames]
    ptrs = (ctypes.c_void_p * n)(*[ctypes.cast(b, ctypes.c_void_p).value for b in bufs])
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    meta = np.zeros(n, np.uint32)
    csum = np.zeros(n, np.uint32)
    fh = np.zeros(n, np.uint64)
    fl = np.zeros((n, N.HDR_RECORD_SIZE), np.uint8) if fields else None
    rc = ctx.L.cgpu_parse_host(
        ctx.handle, ptrs, lens.ctypes.data, n, flags, meta.ctypes.data, csum.ctypes.data,
        fh.ctypes.data, fl.ctypes.data if fields else None)
    N.check(rc, "cgpu_parse_host")
    recs = fl.view(np.dtype(N.HDR_RECORD_FIELDS)).reshape(-1) if fields else None
    return meta, csum, fh, recs


class HostRegion:
    """A host memory range registered for zero-copy ingress (a mempool's
    memzone): whole pages (cgpu_host_register refuses anything else).
    Unregistered on close(), on leaving a `with` block, or when collected;
    the caller keeps the memory mapped until then (`mem`, if given, is held
    here so that it cannot be freed first)."""

    def __init__(self, ctx, base, nbytes, mem=None):
        self.ctx, self.base, self.nbytes, self._mem = ctx, None, nbytes, mem
        N.check(ctx.L.cgpu_host_register(ctx.handle, base, nbytes), "cgpu_host_register")
        self.base = base

    @classmethod
    def of(cls, ctx, mem):
        """Register a numpy u8 array of whole pages (synth.host_buffer,
        synth.pinned_buffer) and keep it alive with the registration."""
        return cls(ctx, mem.ctypes.data, mem.nbytes, mem=mem)

    def close(self):
        if self.base is not None and self.ctx.handle:
            N.check(self.ctx.L.cgpu_host_unregister(self.ctx.handle, self.base),
                    "cgpu_host_unregister")
        self.base = None
        self._mem = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def parse_mbufs(ctx, mbufs, flags=None, ingress=N.INGRESS_STAGE, fields=False):
    """A burst of rte_mbufs (u64 numpy array of their addresses, the
    Vec<Mbuf> of PacketRx::receive) parsed into host arrays.  ingress:
    INGRESS_STAGE (the calling core gathers into pinned staging) or
    INGRESS_ZERO_COPY (the device reads the registered mempool)."""
    if flags is None:
        flags = parse_flags()
    mbufs = np.ascontiguousarray(mbufs, dtype=np.uint64)
    n = len(mbufs)
    meta = np.zeros(n, np.uint32)
    csum = np.zeros(n, np.uint32)
    fh = np.zeros(n, np.uint64)
    fl = np.zeros((n, N.HDR_RECORD_SIZE), np.uint8) if fields else None
    rc = ctx.L.cgpu_parse_mbufs(
        ctx.handle, mbufs.ctypes.data, n, flags, ingress, meta.ctypes.data, csum.ctypes.data,
        fh.ctypes.data, fl.ctypes.data if fields else None)
    N.check(rc, "cgpu_parse_mbufs")
    recs = fl.view(np.dtype(N.HDR_RECORD_FIELDS)).reshape(-1) if fields else None
    return meta, csum, fh, recs


def parse_frames(ctx, addrs, lens, flags=None, ingress=N.INGRESS_STAGE, fields=False):
    """A burst handed over as host (data_address, data_len) pairs (u64 and
    u16 numpy arrays) parsed into host arrays.  INGRESS_ZERO_COPY: the device
    reads the frames alone from registered host memory."""
    if flags is None:
        flags = parse_flags()
    addrs = np.ascontiguousarray(addrs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    n = len(addrs)
    meta = np.zeros(n, np.uint32)
    csum = np.zeros(n, np.uint32)
    fh = np.zeros(n, np.uint64)
    fl = np.zeros((n, N.HDR_RECORD_SIZE), np.uint8) if fields else None
    rc = ctx.L.cgpu_parse_frames(
        ctx.handle, addrs.ctypes.data, lens.ctypes.data, n, flags, ingress, meta.ctypes.data,
        csum.ctypes.data, fh.ctypes.data, fl.ctypes.data if fields else None)
    N.check(rc, "cgpu_parse_frames")
    recs = fl.view(np.dtype(N.HDR_RECORD_FIELDS)).reshape(-1) if fields else None
    return meta, csum, fh, recs


class FramesTicket:
    """A burst in flight through `parse_frames_submit`: its host result
    arrays (valid once `parse_frames_wait` has returned)."""

    def __init__(self, ticket, meta, csum, flow_hash, keep):
        self.ticket, self.meta, self.csum, self.flow_hash = ticket, meta, csum, flow_hash
        self._keep = keep


def parse_frames_submit(ctx, addrs, lens, flags=None, out=None):
    """`cgpu_parse_frames_submit`: start the zero-copy parse of a burst of
    (data_address, data_len) pairs and return at once (at most two bursts in
    flight per context; CgpuError EBUSY past that).  `out`: (meta, csum,
    flow_hash) host arrays to fill, else new ones."""
    if flags is None:
        flags = parse_flags()
    addrs = np.ascontiguousarray(addrs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    n = len(addrs)
    if out is None:
        out = (np.zeros(n, np.uint32), np.zeros(n, np.uint32), np.zeros(n, np.uint64))
    meta, cs, fh = out
    t = ctypes.c_uint32()
    N.check(ctx.L.cgpu_parse_frames_submit(ctx.handle, addrs.ctypes.data, lens.ctypes.data, n,
                                           flags, meta.ctypes.data, cs.ctypes.data,
                                           fh.ctypes.data, ctypes.byref(t)),
            "cgpu_parse_frames_submit")
    return FramesTicket(t.value, meta, cs, fh, out)


def parse_frames_wait(ctx, tk):
    """`cgpu_parse_frames_wait`: the burst's results are in tk's arrays."""
    N.check(ctx.L.cgpu_parse_frames_wait(ctx.handle, tk.ticket), "cgpu_parse_frames_wait")
    return tk.meta, tk.csum, tk.flow_hash


class Groups:
    """Result of `group_by`: `idx[off[k]:off[k+1]]` are arm k's packets."""

    def __init__(self, idx, off):
        self.idx = idx
        self.off = off

    def arm(self, k, host_off=None):
        o = host_off if host_off is not None else self.off.cpu().tolist()
        return self.idx[o[k]:o[k + 1]]

    def counts(self):
        o = self.off.cpu().tolist()
        return [o[k + 1] - o[k] for k in range(len(o) - 1)]


# arms of group_by(..., by="class") (include/capsule_gpu.h CGPU_KEY_META_CLASS)
CLASS_ARMS = ("v4_udp", "v4_tcp", "v6_udp", "v6_tcp", "other")


def group_by(ctx, key, n_groups=None, by="key", idx=None, stream=None):
    """`batch.group_by(selector, compose!{..})` (core/src/batch/group_by.rs:
    143-172) over a whole burst: a stable partition of packet indices into
    arms.  `by="key"`: `key` is a u8 tensor of arm numbers (e.g. a nat64
    disposition array, whose arm sizes are the Emitted/Dropped/Aborted
    counters of send.rs:104-110); keys >= n_groups - 1 fall into the last,
    catch-all arm.  `by="class"`: `key` is the parse meta tensor and the arms
    are CLASS_ARMS.  Asynchronous on `stream`."""
    n = key.numel()
    if by == "class":
        kind, n_groups = N.KEY_META_CLASS, n_groups or len(CLASS_ARMS)
        if key.dtype != torch.int32:
            raise TypeError("group_by(by='class') takes the int32 parse meta tensor")
    elif by == "key":
        kind = N.KEY_U8
        if key.dtype != torch.uint8 or n_groups is None:
            raise TypeError("group_by(by='key') takes a uint8 key tensor and n_groups")
    else:
        raise ValueError(by)
    if idx is None:
        idx = torch.empty(n, dtype=torch.int32, device=key.device)
    off = torch.empty(n_groups + 1, dtype=torch.int32, device=key.device)
    rc = ctx.L.cgpu_group_by(ctx.handle, _ptr(key.contiguous()), kind, n, n_groups, _ptr(idx),
                               _ptr(off), _stream_handle(stream))
    N.check(rc, "cgpu_group_by")
    return Groups(idx[:n], off)


def ip_addrs(addrs):
    """Host cgpu_ip_addr array from `ipaddress` objects (or (family, bytes))."""
    a = np.zeros(len(addrs), np.dtype(N.IP_ADDR_FIELDS))
    for i, x in enumerate(addrs):
        fam, b = (x.version, x.packed) if hasattr(x, "packed") else x
        if fam not in (4, 6) or len(b) != (4 if fam == 4 else 16):
            raise ValueError(f"bad address {x!r}")
        a[i]["family"] = fam
        a[i]["octets"][: len(b)] = np.frombuffer(bytes(b), np.uint8)
    return a


def _addr_tensor(addrs, n, device):
    if addrs is None:
        return None, 0
    if isinstance(addrs, np.ndarray):
        addrs = torch.from_numpy(addrs.view(np.uint8).reshape(-1, N.IP_ADDR_SIZE)).to(device)
    elif not isinstance(addrs, torch.Tensor):
        addrs = torch.from_numpy(ip_addrs(addrs).view(np.uint8).reshape(-1, N.IP_ADDR_SIZE)).to(device)
    if addrs.dtype != torch.uint8 or addrs.numel() % N.IP_ADDR_SIZE:
        raise TypeError("addresses: cgpu_ip_addr records (uint8 [k, 20])")
    k = addrs.numel() // N.IP_ADDR_SIZE
    if k not in (1, n):
        raise ValueError(f"{k} addresses for {n} packets (need 1 or n)")
    return addrs.contiguous(), (0 if k == 1 else 1)


def set_ip(ctx, batch, meta, src=None, dst=None, stream=None, status=None):
    """`udp.set_src_ip(src)?; udp.set_dst_ip(dst)?` (udp.rs:174-201,
    tcp.rs:432-459) for every packet the parse accepted as UDP/TCP, in place
    in `batch.arena`: the address store plus the RFC 1624 incremental update
    of the L4 checksum (checksum::compute_with_ipaddr, checksum.rs:202-220).
    `src`/`dst`: one address for the whole burst or one per packet, as
    `ipaddress` objects, a cgpu_ip_addr numpy array or a device uint8
    [k, 20] tensor.  Returns the per-packet status (SETIP_*; a family
    mismatch is the reference's "cannot mix IPv4 and IPv6 addresses.").
    Asynchronous on `stream`."""
    n = batch.n
    dev = batch.arena.device
    if meta.dtype != torch.int32 or meta.numel() != n:
        raise TypeError("set_ip takes the int32 parse meta tensor of this batch")
    s, ss = _addr_tensor(src, n, dev)
    d, ds = _addr_tensor(dst, n, dev)
    if status is None:
        status = torch.empty(n, dtype=torch.uint8, device=dev)
    rc = ctx.L.cgpu_set_ip(ctx.handle, _ptr(batch.arena), batch.arena.numel(), _ptr(batch.off),
                             _ptr(batch.len), _ptr(meta), n, _ptr(s), ss, _ptr(d), ds,
                             _ptr(status), _stream_handle(stream))
    N.check(rc, "cgpu_set_ip")
    if stream is not None:  # address copies made here must outlive the launch
        for t in (s, d):
            if t is not None:
                t.record_stream(stream)
    return status


_DEPTH = {"l2": N.LAYER_L2, "l3": N.LAYER_L3, "l4": N.LAYER_L4}


def reconcile(ctx, batch, meta, flags=None, depth="l4", stream=None, status=None):
    """`packet.reconcile_all()` (packets/mod.rs:297-300) for every packet of
    a parsed burst, in place in `batch.arena`, each held at `depth` ("l4",
    "l3" or "l2") with the layers its parse `meta` recorded: L4 (Udp: length
    := span, then the checksum, udp.rs:350-354; Tcp / Icmp: the checksum),
    then L3 (Ipv4: total_length, header checksum, v4.rs:486-489; Ipv6:
    payload_length, v6/mod.rs:331-334).  `flags`: the accept set the parse
    ran with.  Returns the per-packet status (RECON_OK / RECON_SKIPPED: the
    parse did not reach `depth`).  Asynchronous on `stream`."""
    n = batch.n
    dev = batch.arena.device
    if meta.dtype != torch.int32 or meta.numel() != n:
        raise TypeError("reconcile takes the int32 parse meta tensor of this batch")
    if flags is None:
        flags = parse_flags()
    if status is None:
        status = torch.empty(n, dtype=torch.uint8, device=dev)
    rc = ctx.L.cgpu_reconcile(ctx.handle, _ptr(batch.arena), batch.arena.numel(), _ptr(batch.off),
                                _ptr(batch.len), _ptr(meta), n, flags, _DEPTH[depth], _ptr(status),
                                _stream_handle(stream))
    N.check(rc, "cgpu_reconcile")
    return status


def reconcile_frames(ctx, addrs, lens, meta, flags=None, depth="l4"):
    """`reconcile_all` over a burst handed over as host (data_address,
    data_len) pairs in registered host memory (cgpu_reconcile_frames), in
    place; `meta` the host parse words of those bytes (e.g. from
    `parse_frames`).  Returns the status per frame (RECON_OK / _SKIPPED)."""
    if flags is None:
        flags = parse_flags()
    addrs = np.ascontiguousarray(addrs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    meta = np.ascontiguousarray(meta, dtype=np.uint32)
    n = len(addrs)
    if len(lens) != n or len(meta) != n:
        raise ValueError("addrs, lens and meta must have one entry per frame")
    st = np.zeros(n, np.uint8)
    rc = ctx.L.cgpu_reconcile_frames(ctx.handle, addrs.ctypes.data, lens.ctypes.data,
                                       meta.ctypes.data, n, flags, _DEPTH[depth], st.ctypes.data)
    N.check(rc, "cgpu_reconcile_frames")
    return st


class ReconcileLauncher:
    """A `reconcile` call with prebuilt ctypes arguments (bench loops)."""

    def __init__(self, ctx, batch, meta, flags, depth="l4", stream=None, status=None):
        self._keep = (batch, meta, status)
        self._fn = ctx.L.cgpu_reconcile
        self._args = [ctx.handle, _ptr(batch.arena), batch.arena.numel(), _ptr(batch.off),
                      _ptr(batch.len), _ptr(meta), batch.n, flags, _DEPTH[depth], _ptr(status),
                      _stream_handle(stream)]

    def __call__(self):
        rc = self._fn(*self._args)
        if rc:
            N.check(rc, "cgpu_reconcile")


class Nat64Gateway:
    """examples/nat64 6to4 direction with its PORT_MAP on the device.

    `NEXT_PORT` starts at `first_port` (1025 in examples/nat64/main.rs:42) and
    wraps modulo 2^16 like `AtomicU16::fetch_add`.  Packets are assigned
    gateway ports in batch order, so a stream cut into consecutive batches
    gets exactly the ports the reference's single-core pipeline would.
    """

    def __init__(self, ctx, capacity_log2=20, first_port=1025):
        self.ctx = ctx
        self._h = ctypes.c_void_p()
        N.check(self.ctx.L.cgpu_portmap_create(ctx.handle, capacity_log2, first_port,
                                            ctypes.byref(self._h)), "cgpu_portmap_create")

    def next_port(self):
        v = ctypes.c_uint16()
        N.check(self.ctx.L.cgpu_portmap_next_port(self._h, ctypes.byref(v)), "next_port")
        return v.value

    def size(self):
        v = ctypes.c_uint32()
        N.check(self.ctx.L.cgpu_portmap_size(self._h, ctypes.byref(v)), "size")
        return v.value

    def reset(self, first_port=1025, stream=None):
        """Empty the map (as a fresh gateway), asynchronously on `stream`."""
        N.check(self.ctx.L.cgpu_portmap_reset(self._h, first_port, _stream_handle(stream)),
                "cgpu_portmap_reset")

    def _call(self, fn, what, grow, batch, out_arena, out_off, stream, out):
        n = batch.n
        dev = batch.arena.device
        if out is None:
            if out_arena is None:
                out_arena = torch.zeros(batch.arena.numel() + grow * n, dtype=torch.uint8,
                                        device=dev)
            if out_off is None:
                out_off = batch.off
            out_len = torch.zeros(n, dtype=torch.int16, device=dev)
            disp = torch.empty(n, dtype=torch.uint8, device=dev)
            status = torch.empty(n, dtype=torch.uint8, device=dev)
        else:
            out_arena, out_off, out_len, disp, status = out
        cb = batch.cbatch()
        rc = fn(self.ctx.handle, self._h, ctypes.byref(cb), _ptr(out_arena), out_arena.numel(),
                _ptr(out_off), _ptr(out_len), _ptr(disp), _ptr(status), _stream_handle(stream))
        N.check(rc, what)
        return PacketBatch(out_arena, out_off, out_len), disp, status

    def nat_6to4(self, batch, out_arena=None, out_off=None, stream=None, out=None):
        """`nat_6to4` (examples/nat64/main.rs:121-150) on a device batch.

        Returns (out PacketBatch, disposition u8, status u8).  Output frame i
        is written at out_off[i] (default: its input slot offset in a fresh
        arena of the same size); out_len[i] is the new data_len for ACT
        packets and 0 otherwise.
        """
        return self._call(self.ctx.L.cgpu_nat64_6to4, "cgpu_nat64_6to4", 0, batch, out_arena,
                          out_off, stream, out)

    def nat_4to6(self, batch, out_arena, out_off, stream=None, out=None):
        """`nat_4to6` (examples/nat64/main.rs:86-118): output frames are 20 B
        longer, so out_off[i] must leave room for len[i] + 20 bytes."""
        return self._call(self.ctx.L.cgpu_nat64_4to6, "cgpu_nat64_4to6", 20, batch, out_arena,
                          out_off, stream, out)

    def nat_mbufs(self, mbufs, direction="6to4"):
        """`install_6to4` / `install_4to6` (examples/nat64/main.rs:152-165)
        on a burst of rte_mbufs (u64 numpy array of their addresses, from a
        mempool registered with HostRegion): the device reads the frames,
        rewrites them and writes every ACT frame back into its own mbuf
        (data_len / pkt_len -20 or +20).  Returns host (disposition, status)."""
        mbufs = np.ascontiguousarray(mbufs, dtype=np.uint64)
        n = len(mbufs)
        disp = np.zeros(n, np.uint8)
        st = np.zeros(n, np.uint8)
        d = {"6to4": N.NAT64_6TO4, "4to6": N.NAT64_4TO6}[direction]
        rc = self.ctx.L.cgpu_nat64_mbufs(self.ctx.handle, self._h, d, mbufs.ctypes.data, n,
                                      disp.ctypes.data, st.ctypes.data)
        N.check(rc, "cgpu_nat64_mbufs")
        return disp, st

    def nat_frames(self, addrs, lens, tailroom=None, direction="6to4"):
        """`nat_mbufs` over (data_address, data_len) pairs (u64 / u16 numpy
        arrays; tailroom u16, needed for 4to6): the device rewrites the
        frames in place in registered memory and touches no mbuf header.
        Returns host (out_len, disposition, status); out_len is each ACT
        frame's new data_len."""
        addrs = np.ascontiguousarray(addrs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        tr = None if tailroom is None else np.ascontiguousarray(tailroom, dtype=np.uint16)
        n = len(addrs)
        olen = np.zeros(n, np.uint16)
        disp = np.zeros(n, np.uint8)
        st = np.zeros(n, np.uint8)
        d = {"6to4": N.NAT64_6TO4, "4to6": N.NAT64_4TO6}[direction]
        rc = self.ctx.L.cgpu_nat64_frames(self.ctx.handle, self._h, d, addrs.ctypes.data,
                                       lens.ctypes.data, tr.ctypes.data if tr is not None else None,
                                       n, olen.ctypes.data, disp.ctypes.data, st.ctypes.data)
        N.check(rc, "cgpu_nat64_frames")
        return olen, disp, st

    def close(self):
        if self._h:
            self.ctx.L.cgpu_portmap_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ParseLauncher:
    """A `parse` call with every ctypes argument prebuilt: calling it costs one
    foreign call (for launch-bound loops such as bench.py; the batch and
    output tensors must stay alive and unchanged in size)."""

    def __init__(self, ctx, batch, out, flags, stream=None):
        self._keep = (batch, out)
        self._fn = ctx.L.cgpu_parse_batch
        self._args = [ctx.handle, None, flags, None, _stream_handle(stream)]
        self._cb = batch.cbatch()
        self._po = N.ParseOut()
        self._po.meta = out.meta.data_ptr()
        self._po.csum = out.csum.data_ptr() if out.csum is not None else None
        self._po.flow_hash = out.flow_hash.data_ptr()
        self._po.fields = out.fields.data_ptr() if out.fields is not None else None
        self._args[1] = ctypes.byref(self._cb)
        self._args[3] = ctypes.byref(self._po)

    def __call__(self):
        rc = self._fn(*self._args)
        if rc:
            N.check(rc, "cgpu_parse_batch")


class Nat64Launcher:
    """A `Nat64Gateway.nat_6to4` (or `nat_4to6`) call with prebuilt ctypes
    arguments."""

    def __init__(self, gw, batch, out, stream=None, direction="6to4"):
        out_arena, out_off, out_len, disp, status = out
        self._keep = (gw, batch, out)
        self._cb = batch.cbatch()
        self._name = {"6to4": "cgpu_nat64_6to4", "4to6": "cgpu_nat64_4to6"}[direction]
        self._fn = getattr(gw.ctx.L, self._name)
        self._args = [gw.ctx.handle, gw._h, ctypes.byref(self._cb), _ptr(out_arena),
                      out_arena.numel(), _ptr(out_off), _ptr(out_len), _ptr(disp), _ptr(status),
                      _stream_handle(stream)]

    def __call__(self):
        rc = self._fn(*self._args)
        if rc:
            N.check(rc, self._name)
