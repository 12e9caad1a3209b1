"""ctypes handle on the CPU oracle (oracle/liboracle.so) — test-side only.

The oracle is the parity checker: tests, __graft_entry__.smoke() and
bench.py's cpu_baseline leg are the only users (oracle/oracle.h).
"""
import ctypes
import pathlib
import subprocess

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
ORACLE_DIR = ROOT / "oracle"


def load(name="liboracle.so"):
    path = ORACLE_DIR / name
    if not path.exists():
        subprocess.run(["make", "-C", str(ORACLE_DIR), name], check=True,
                       stdout=subprocess.DEVNULL)
    L = ctypes.CDLL(str(path))
    vp, u8, u16, u32, u64, sz, i32 = (ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint16,
                                      ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t,
                                      ctypes.c_int)
    L.or_compute.restype = u16
    L.or_compute.argtypes = [u16, vp, sz]
    L.or_compute_inc.restype = u16
    L.or_compute_inc.argtypes = [u16, vp, vp, sz]
    L.or_pseudo_v4.restype = u16
    L.or_pseudo_v4.argtypes = [u32, u32, u16, u8]
    L.or_pseudo_v6.restype = u16
    L.or_pseudo_v6.argtypes = [vp, vp, u16, u8]
    L.or_siphash.restype = u64
    L.or_siphash.argtypes = [i32, i32, u64, u64, vp, sz]
    L.or_flow_bytes.restype = sz
    L.or_flow_bytes.argtypes = [i32, vp, vp, u16, u16, u8, vp]
    L.or_flow_hash.restype = u64
    L.or_flow_hash.argtypes = [i32, vp, vp, u16, u16, u8]
    L.or_parse_batch.restype = None
    L.or_parse_batch.argtypes = [vp, vp, vp, u32, u32, vp, vp, vp, vp]
    L.or_parse_batch_ext.restype = None
    L.or_parse_batch_ext.argtypes = [vp, vp, vp, u32, u32, vp, vp, vp, vp, vp]
    L.or_multi_parse_udp.restype = u32
    L.or_multi_parse_udp.argtypes = [vp, vp, vp, u32]
    L.or_set_mbuf_data_room.restype = None
    L.or_set_mbuf_data_room.argtypes = [u32]
    L.or_portmap_new.restype = vp
    L.or_portmap_new.argtypes = [u16]
    L.or_portmap_free.restype = None
    L.or_portmap_free.argtypes = [vp]
    L.or_portmap_next_port.restype = u16
    L.or_portmap_next_port.argtypes = [vp]
    L.or_portmap_size.restype = u32
    L.or_portmap_size.argtypes = [vp]
    L.or_nat64_6to4.restype = None
    L.or_nat64_6to4.argtypes = [vp, vp, vp, vp, u32, vp, vp, vp, vp, vp]
    L.or_group_by.restype = None
    L.or_group_by.argtypes = [vp, u32, u32, u32, vp, vp]
    L.or_nat64_4to6.restype = None
    L.or_nat64_4to6.argtypes = [vp, vp, vp, vp, u32, vp, vp, vp, vp, vp]
    L.or_set_ip.restype = None
    L.or_set_ip.argtypes = [vp, vp, vp, vp, u32, vp, u32, vp, u32, vp]
    L.or_reconcile.restype = None
    L.or_reconcile.argtypes = [vp, u64, vp, vp, vp, u32, u32, u32, vp]
    return L


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = load()
    return _lib


def _p(a):
    return a.ctypes.data if a is not None else None


def parse_batch_ext(arena, off, length, flags):
    """Oracle parse with extension records -> (meta, csum, hash, fields [n,96], ext [n,48])."""
    n = len(off)
    arena = np.ascontiguousarray(arena, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    length = np.ascontiguousarray(length, np.uint16)
    meta = np.zeros(n, np.uint32)
    csum = np.zeros(n, np.uint32)
    h = np.zeros(n, np.uint64)
    fl = np.zeros((n, 96), np.uint8)
    ext = np.zeros((n, 48), np.uint8)
    lib().or_parse_batch_ext(_p(arena), _p(off), _p(length), n, flags, _p(meta), _p(csum), _p(h),
                             _p(fl), _p(ext))
    return meta, csum, h, fl, ext


def parse_batch(arena, off, length, flags, fields=True):
    """Oracle parse -> (meta u32, csum u32, hash u64, fields bytes [n,96])."""
    n = len(off)
    arena = np.ascontiguousarray(arena, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    length = np.ascontiguousarray(length, np.uint16)
    meta = np.zeros(n, np.uint32)
    csum = np.zeros(n, np.uint32)
    h = np.zeros(n, np.uint64)
    fl = np.zeros((n, 96), np.uint8) if fields else None
    lib().or_parse_batch(_p(arena), _p(off), _p(length), n, flags, _p(meta), _p(csum), _p(h),
                         _p(fl))
    return meta, csum, h, fl


IP_ADDR = np.dtype([("octets", "u1", (16,)), ("family", "<u4")])  # cgpu_ip_addr, 20 B


def ip_addrs(addrs):
    """[(family 4|6, bytes)] -> cgpu_ip_addr array."""
    a = np.zeros(len(addrs), IP_ADDR)
    for i, (fam, b) in enumerate(addrs):
        a[i]["family"] = fam
        a[i]["octets"][: len(b)] = np.frombuffer(bytes(b), np.uint8)
    return a


def set_ip(arena, off, length, meta, src=None, dst=None):
    """Oracle Udp/Tcp::set_src_ip / set_dst_ip over a batch (arena copied) ->
    (new arena, status u8[n]).  src/dst: cgpu_ip_addr arrays of length 1
    (broadcast) or n."""
    n = len(off)
    out = np.array(arena, np.uint8, copy=True)
    off = np.ascontiguousarray(off, np.uint32)
    length = np.ascontiguousarray(length, np.uint16)
    meta = np.ascontiguousarray(meta, np.uint32)
    st = np.zeros(n, np.uint8)
    ss = 0 if src is None or len(src) == 1 else 1
    ds = 0 if dst is None or len(dst) == 1 else 1
    lib().or_set_ip(_p(out), _p(off), _p(length), _p(meta), n, _p(src), ss, _p(dst), ds, _p(st))
    return out, st


def reconcile(arena, off, length, meta, flags, depth, arena_len=None):
    """Oracle Packet::reconcile_all at `depth` (3 = L3, 4 = L4) over a parsed
    batch (arena copied) -> (new arena, status u8[n]).  `arena_len`: the
    arena's length as the device sees it (default: all of `arena`); a frame
    past it is skipped."""
    n = len(off)
    out = np.array(arena, np.uint8, copy=True)
    off = np.ascontiguousarray(off, np.uint32)
    length = np.ascontiguousarray(length, np.uint16)
    meta = np.ascontiguousarray(meta, np.uint32)
    st = np.zeros(n, np.uint8)
    lib().or_reconcile(_p(out), len(out) if arena_len is None else arena_len, _p(off), _p(length), _p(meta), n, flags, depth, _p(st))
    return out, st


def group_by(key, n_groups, kind=0):
    """Oracle group_by -> (idx u32[n], group_off u32[n_groups + 1])."""
    key = np.ascontiguousarray(key)
    n = len(key)
    idx = np.zeros(n, np.uint32)
    off = np.zeros(n_groups + 1, np.uint32)
    lib().or_group_by(_p(key), kind, n, n_groups, _p(idx), _p(off))
    return idx, off


class data_room:
    """Context manager: the oracle's simulated mbufs get `room` bytes of data
    room (a custom mempool) instead of DPDK's default 2048."""

    def __init__(self, room):
        self.room = room

    def __enter__(self):
        lib().or_set_mbuf_data_room(self.room)

    def __exit__(self, *exc):
        lib().or_set_mbuf_data_room(2048)


class PortMap:
    def __init__(self, first_port=1025):
        self.h = lib().or_portmap_new(first_port)

    def next_port(self):
        return lib().or_portmap_next_port(self.h)

    def size(self):
        return lib().or_portmap_size(self.h)

    def nat_6to4(self, arena, off, length, out_off=None, out_size=None):
        return self._nat(lib().or_nat64_6to4, arena, off, length, out_off, out_size)

    def nat_4to6(self, arena, off, length, out_off, out_size):
        return self._nat(lib().or_nat64_4to6, arena, off, length, out_off, out_size)

    def _nat(self, fn, arena, off, length, out_off, out_size):
        n = len(off)
        arena = np.ascontiguousarray(arena, np.uint8)
        off = np.ascontiguousarray(off, np.uint32)
        length = np.ascontiguousarray(length, np.uint16)
        out_off = off if out_off is None else np.ascontiguousarray(out_off, np.uint32)
        out = np.zeros(out_size or len(arena), np.uint8)
        out_len = np.zeros(n, np.uint16)
        disp = np.zeros(n, np.uint8)
        st = np.zeros(n, np.uint8)
        fn(self.h, _p(arena), _p(off), _p(length), n, _p(out), _p(out_off), _p(out_len), _p(disp),
           _p(st))
        return out, out_len, disp, st

    def __del__(self):
        try:
            lib().or_portmap_free(self.h)
        except Exception:
            pass
