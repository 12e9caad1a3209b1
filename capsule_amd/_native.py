"""ctypes binding of the C ABI in include/capsule_gpu.h (libcapsule_gpu.so).

This is the Python-side equivalent of the bindgen crate a Rust maintainer
would add next to the reference's ffi/ bindings: the same
structs, constants and entry points, nothing more.  The library is the HIP
build in capsule_amd/libcapsule_gpu.so; importing this module fails loudly if
it is missing (there is no CPU fallback anywhere in capsule_amd).
"""
import ctypes
import os
import pathlib

_HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = pathlib.Path(os.environ.get("CAPSULE_GPU_LIB", _HERE / "libcapsule_gpu.so"))
# The test build (capi.hip with CGPU_TEST_HOOKS): environment hooks that the
# GPU tests use to force rare paths.  Only tests load it (lib(test=True));
# the product library reads no environment.
TEST_LIB_PATH = _HERE / "libcapsule_gpu_test.so"

# ---- constants (include/capsule_gpu.h) ------------------------------------
ABI_VERSION = 6

OK, EINVAL, ENOMEM, ENODEV, EIO, ENOSPC, EBUSY = 0, -22, -12, -19, -5, -28, -16

PKT_STATUS = [
    "OK", "ETH_BAD_OFFSET", "ETH_OUT_OF_BUFFER", "NOT_IPV4", "NOT_IPV6", "NOT_IP",
    "L3_BAD_OFFSET", "L3_OUT_OF_BUFFER", "NOT_UDP", "NOT_TCP", "NOT_L4", "L4_BAD_OFFSET",
    "L4_OUT_OF_BUFFER", "NOT_RESIZED", "TABLE_FULL", "NOT_ICMPV4", "NOT_ICMPV6",
    "EXT_BAD_OFFSET", "EXT_OUT_OF_BUFFER", "SRH_INCONSISTENT",
]
PKT = {name: i for i, name in enumerate(PKT_STATUS)}

META_IP_CSUM_OK = 1 << 20
META_L4_CSUM_OK = 1 << 21
META_DOT1Q = 1 << 22
META_QINQ = 1 << 23
L3_NONE, L3_IPV4, L3_IPV6 = 0, 1, 2
L4_NONE, L4_UDP, L4_TCP, L4_ICMP = 0, 1, 2, 3

F_ACCEPT_V4 = 1 << 0
F_ACCEPT_V6 = 1 << 1
F_ACCEPT_UDP = 1 << 2
F_ACCEPT_TCP = 1 << 3
F_ACCEPT_ALL = 0xF
F_CSUM_IP = 1 << 4
F_CSUM_L4 = 1 << 5
F_FLOW_HASH = 1 << 6
F_ACCEPT_ICMP = 1 << 7  # not part of F_ACCEPT_ALL
F_V6_EXT = 1 << 8       # IPv6 SegmentRouting / Fragment headers before L4
EXT_NONE, EXT_SRH, EXT_FRAGMENT = 0, 1, 2

ACT, DROP, ABORT = 0, 1, 2

# rte_mbuf ingress (include/capsule_gpu.h; DPDK 19.11 field offsets)
MBUF_BUF_ADDR_OFF, MBUF_DATA_OFF_OFF, MBUF_DATA_LEN_OFF, MBUF_SIZE = 0, 16, 40, 128
INGRESS_STAGE, INGRESS_ZERO_COPY = 0, 1
MBUF_PKT_LEN_OFF, MBUF_BUF_LEN_OFF = 36, 54
NAT64_6TO4, NAT64_4TO6 = 0, 1

KEY_U8, KEY_META_CLASS = 0, 1

# cgpu_set_ip (Udp/Tcp::set_src_ip / set_dst_ip)
SETIP_OK, SETIP_SKIPPED, SETIP_SRC_MISMATCH, SETIP_DST_MISMATCH = 0, 1, 2, 3
IP_ADDR_FIELDS = [("octets", "u1", (16,)), ("family", "<u4")]  # cgpu_ip_addr
IP_ADDR_SIZE = 20

# cgpu_reconcile (Packet::reconcile_all)
LAYER_L2, LAYER_L3, LAYER_L4 = 2, 3, 4
RECON_OK, RECON_SKIPPED = 0, 1


def meta_status(m):
    return m & 0xFF


def meta_eth_len(m):
    return (m >> 8) & 0xFF


def meta_l3(m):
    return (m >> 16) & 0x3


def meta_l4(m):
    return (m >> 18) & 0x3


# ---- structs ----------------------------------------------------------------
class Batch(ctypes.Structure):
    _fields_ = [
        ("arena", ctypes.c_void_p),
        ("arena_len", ctypes.c_uint64),
        ("off", ctypes.c_void_p),
        ("len", ctypes.c_void_p),
        ("n", ctypes.c_uint32),
    ]


class ParseOut(ctypes.Structure):
    _fields_ = [
        ("meta", ctypes.c_void_p),
        ("csum", ctypes.c_void_p),
        ("flow_hash", ctypes.c_void_p),
        ("fields", ctypes.c_void_p),
        ("ext", ctypes.c_void_p),
    ]


# numpy dtype of cgpu_hdr_record (96 bytes), field offsets as in the header.
HDR_RECORD_FIELDS = [
    ("dst_mac", "u1", (6,)), ("src_mac", "u1", (6,)), ("ether_type", "<u2"), ("eth_len", "u1"),
    ("vlan", "u1"), ("version", "u1"), ("ihl", "u1"), ("dscp", "u1"), ("ecn", "u1"),
    ("ip_length", "<u2"), ("identification", "<u2"), ("ip_flags", "u1"), ("ttl", "u1"),
    ("fragment_offset", "<u2"), ("protocol", "u1"), ("pad0", "u1"), ("ip_checksum", "<u2"),
    ("flow_label", "<u4"), ("pad1", "<u4"), ("src_ip", "u1", (16,)), ("dst_ip", "u1", (16,)),
    ("src_port", "<u2"), ("dst_port", "<u2"), ("udp_length_or_window", "<u2"),
    ("l4_checksum", "<u2"), ("seq_no", "<u4"), ("ack_no", "<u4"), ("data_offset", "u1"),
    ("tcp_flags", "u1"), ("ns", "u1"), ("pad2", "u1"), ("urgent_pointer", "<u2"),
    ("pad3", "<u2"),
]
HDR_RECORD_SIZE = 96

EXT_RECORD_FIELDS = [  # cgpu_ext_record, 48 bytes
    ("kind", "u1"), ("next_header", "u1"), ("header_len", "<u2"), ("hdr_ext_len", "u1"),
    ("routing_type", "u1"), ("segments_left", "u1"), ("last_entry", "u1"), ("srh_flags", "u1"),
    ("more_fragments", "u1"), ("tag", "<u2"), ("fragment_offset", "<u2"), ("pad0", "<u2"),
    ("identification", "<u4"), ("pad1", "<u4"), ("segment0", "u1", (16,)), ("pad2", "u1", (8,)),
]
EXT_RECORD_SIZE = 48

# Every symbol include/capsule_gpu.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "cgpu_ctx_create", "cgpu_ctx_destroy", "cgpu_parse_batch", "cgpu_parse_host",
    "cgpu_portmap_create", "cgpu_portmap_destroy", "cgpu_portmap_next_port",
    "cgpu_portmap_size", "cgpu_nat64_6to4", "cgpu_nat64_4to6", "cgpu_group_by", "cgpu_last_error", "cgpu_strerror",
    "cgpu_pkt_status_str", "cgpu_abi_version", "cgpu_host_register", "cgpu_host_unregister",
    "cgpu_parse_mbufs", "cgpu_set_ip", "cgpu_nat64_mbufs", "cgpu_parse_frames",
    "cgpu_nat64_frames", "cgpu_portmap_reset", "cgpu_reconcile", "cgpu_reconcile_frames",
    "cgpu_ctx_check", "cgpu_parse_frames_submit", "cgpu_parse_frames_wait",
]

_libs = {}


def lib(test=False):
    """Load libcapsule_gpu.so (test=True: the test build) once; raise if it
    is absent (no fallback)."""
    if test in _libs:
        return _libs[test]
    path = TEST_LIB_PATH if test else LIB_PATH
    if not path.exists():
        raise RuntimeError(
            f"capsule_amd: HIP library {path} not built; run "
            "`python -c 'import __graft_entry__ as g; g.build()'` (make -C capsule_amd/csrc)")
    L = ctypes.CDLL(str(path))
    vp, u32, u16, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_int
    P = ctypes.POINTER
    L.cgpu_abi_version.restype = i32
    L.cgpu_last_error.restype = i32
    L.cgpu_strerror.restype = ctypes.c_char_p
    L.cgpu_strerror.argtypes = [i32]
    L.cgpu_pkt_status_str.restype = ctypes.c_char_p
    L.cgpu_pkt_status_str.argtypes = [i32]
    L.cgpu_ctx_create.restype = i32
    L.cgpu_ctx_create.argtypes = [i32, P(vp)]
    L.cgpu_ctx_destroy.restype = None
    L.cgpu_ctx_destroy.argtypes = [vp]
    L.cgpu_ctx_check.restype = i32
    L.cgpu_ctx_check.argtypes = [vp, vp]
    L.cgpu_parse_frames_submit.restype = i32
    L.cgpu_parse_frames_submit.argtypes = [vp, vp, vp, u32, u32, vp, vp, vp, P(u32)]
    L.cgpu_parse_frames_wait.restype = i32
    L.cgpu_parse_frames_wait.argtypes = [vp, u32]
    L.cgpu_parse_batch.restype = i32
    L.cgpu_parse_batch.argtypes = [vp, P(Batch), u32, P(ParseOut), vp]
    L.cgpu_parse_host.restype = i32
    L.cgpu_parse_host.argtypes = [vp, P(vp), vp, u32, u32, vp, vp, vp, vp]
    L.cgpu_portmap_create.restype = i32
    L.cgpu_portmap_create.argtypes = [vp, u32, u16, P(vp)]
    L.cgpu_portmap_destroy.restype = None
    L.cgpu_portmap_destroy.argtypes = [vp]
    L.cgpu_portmap_next_port.restype = i32
    L.cgpu_portmap_next_port.argtypes = [vp, P(u16)]
    L.cgpu_portmap_size.restype = i32
    L.cgpu_portmap_size.argtypes = [vp, P(u32)]
    L.cgpu_portmap_reset.restype = i32
    L.cgpu_portmap_reset.argtypes = [vp, u16, vp]
    L.cgpu_nat64_6to4.restype = i32
    L.cgpu_nat64_6to4.argtypes = [vp, vp, P(Batch), vp, ctypes.c_uint64, vp, vp, vp, vp, vp]
    L.cgpu_nat64_4to6.restype = i32
    L.cgpu_nat64_4to6.argtypes = [vp, vp, P(Batch), vp, ctypes.c_uint64, vp, vp, vp, vp, vp]
    L.cgpu_host_register.restype = i32
    L.cgpu_host_register.argtypes = [vp, vp, ctypes.c_size_t]
    L.cgpu_host_unregister.restype = i32
    L.cgpu_host_unregister.argtypes = [vp, vp]
    L.cgpu_parse_mbufs.restype = i32
    L.cgpu_parse_mbufs.argtypes = [vp, vp, u32, u32, u32, vp, vp, vp, vp]
    L.cgpu_nat64_frames.restype = i32
    L.cgpu_nat64_frames.argtypes = [vp, vp, u32, vp, vp, vp, u32, vp, vp, vp]
    L.cgpu_parse_frames.restype = i32
    L.cgpu_parse_frames.argtypes = [vp, vp, vp, u32, u32, u32, vp, vp, vp, vp]
    L.cgpu_group_by.restype = i32
    L.cgpu_group_by.argtypes = [vp, vp, u32, u32, u32, vp, vp, vp]
    L.cgpu_nat64_mbufs.restype = i32
    L.cgpu_nat64_mbufs.argtypes = [vp, vp, u32, vp, u32, vp, vp]
    L.cgpu_set_ip.restype = i32
    L.cgpu_set_ip.argtypes = [vp, vp, ctypes.c_uint64, vp, vp, vp, u32, vp, u32, vp, u32, vp, vp]
    L.cgpu_reconcile.restype = i32
    L.cgpu_reconcile.argtypes = [vp, vp, ctypes.c_uint64, vp, vp, vp, u32, u32, u32, vp, vp]
    L.cgpu_reconcile_frames.restype = i32
    L.cgpu_reconcile_frames.argtypes = [vp, vp, vp, vp, u32, u32, u32, vp]
    if L.cgpu_abi_version() != ABI_VERSION:
        raise RuntimeError(f"capsule_amd: {path.name} ABI version mismatch")
    _libs[test] = L
    return L


class CgpuError(RuntimeError):
    """A call-level failure (negative errno-style code), like DpdkError."""

    def __init__(self, code, what):
        self.code = code
        msg = lib().cgpu_strerror(code).decode()
        super().__init__(f"{what}: {msg} ({code})")


def check(rc, what):
    if rc != 0:
        raise CgpuError(rc, what)
