"""The C-ABI library loads and exports every symbol include/capsule_gpu.h
declares (no GPU work: only the pure-host entry points are called)."""
import ctypes
import pathlib
import re
import subprocess

from capsule_amd import _native as N

ROOT = pathlib.Path(__file__).resolve().parents[1]


def declared_functions():
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names |= set(re.findall(r"\b(cgpu_\w+)\s*\(", text))
    return names


def test_header_declares_what_binding_binds():
    assert declared_functions() == set(N.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = N.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", str(N.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\b(cgpu_\w+)\b", out))
    assert declared_functions() <= exported


def test_library_is_gfx950_hip_code():
    """The shared object carries a gfx950 HIP fat binary (no other target)."""
    data = N.LIB_PATH.read_bytes()
    assert b".hip_fatbin" in data
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in data
    assert b"--gfx942" not in data and b"--gfx90a" not in data


def test_host_only_entry_points():
    L = N.lib()
    assert L.cgpu_abi_version() == N.ABI_VERSION
    assert L.cgpu_strerror(N.EINVAL) == b"invalid argument"
    assert L.cgpu_strerror(N.OK) == b"success"
    # the reference's own error strings (ip/v4.rs:430, v6/mod.rs:277, udp.rs:290, tcp.rs:561)
    assert L.cgpu_pkt_status_str(N.PKT["NOT_IPV4"]) == b"not an IPv4 packet."
    assert L.cgpu_pkt_status_str(N.PKT["NOT_IPV6"]) == b"not an IPv6 packet."
    assert L.cgpu_pkt_status_str(N.PKT["NOT_UDP"]) == b"not a UDP packet."
    assert L.cgpu_pkt_status_str(N.PKT["NOT_TCP"]) == b"not a TCP packet."
    for s, name in enumerate(N.PKT_STATUS):
        assert L.cgpu_pkt_status_str(s) != b"unknown status", name


def test_null_arguments_fail_with_einval_and_set_last_error():
    L = N.lib()
    assert L.cgpu_parse_batch(None, None, 0, None, None) == N.EINVAL
    assert L.cgpu_last_error() == N.EINVAL
    out = ctypes.c_void_p()
    assert L.cgpu_portmap_create(None, 20, 1025, ctypes.byref(out)) == N.EINVAL
    assert L.cgpu_nat64_6to4(None, None, None, None, 0, None, None, None, None, None) == N.EINVAL


def test_record_layout_matches_header():
    import numpy as np

    dt = np.dtype(N.HDR_RECORD_FIELDS)
    assert dt.itemsize == N.HDR_RECORD_SIZE == 96
    for field, off in (("ether_type", 12), ("ip_length", 20), ("protocol", 28),
                       ("ip_checksum", 30), ("flow_label", 32), ("src_ip", 40), ("dst_ip", 56),
                       ("src_port", 72), ("l4_checksum", 78), ("seq_no", 80), ("data_offset", 88),
                       ("urgent_pointer", 92)):
        assert dt.fields[field][1] == off, field


def test_host_modules_import_without_gpu():
    import capsule_amd
    from capsule_amd import packets, shards  # noqa: F401

    assert capsule_amd.packets is packets


def test_plain_c_consumer_compiles_and_links(tmp_path):
    """include/capsule_gpu.h as a C11 translation unit (the bindgen input):
    record layouts and rte_mbuf offsets pinned by _Static_assert, every entry
    point linked from libcapsule_gpu.so, host-only calls run."""
    exe = tmp_path / "abi_check"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-pedantic",
                    f"-I{ROOT / 'include'}", str(ROOT / "tests" / "c" / "abi_check.c"),
                    f"-L{N.LIB_PATH.parent}", "-lcapsule_gpu",
                    f"-Wl,-rpath,{N.LIB_PATH.parent}", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stderr)
    assert r.stdout.startswith(f"abi ok: {len(N.EXPORTS)} entry points, not a UDP packet.")


def test_host_register_takes_whole_pages_only():
    """cgpu_host_register refuses a base or a size that is not a multiple
    of the page size (hipHostRegister pins whole pages, so a partial page
    would pin bytes of other allocations) before it touches the context or
    the device.  No GPU here: the context argument is a zeroed stand-in that
    the argument checks never read."""
    import mmap

    from capsule_amd import synth

    L = N.lib()
    fake_ctx = ctypes.create_string_buffer(1 << 16)
    page = mmap.PAGESIZE
    buf = synth.host_buffer(4 * page)
    assert buf.nbytes == 4 * page and buf.ctypes.data % page == 0
    base = buf.ctypes.data
    for b, n in ((base + 64, 2 * page), (base, 2 * page + 1), (base + page // 2, page),
                 (base, 100), (base, 0), (0, page)):
        assert L.cgpu_host_register(fake_ctx, ctypes.c_void_p(b), n) == N.EINVAL, (b - base, n)
        assert L.cgpu_last_error() == N.EINVAL
    assert L.cgpu_host_unregister(None, ctypes.c_void_p(base)) == N.EINVAL
    assert L.cgpu_ctx_check(None, None) == N.EINVAL


def test_test_build_is_separate():
    """The environment hooks live only in the test build: the product
    library has no getenv reference and none of the hook names."""
    prod = N.LIB_PATH.read_bytes()
    for name in (b"CGPU_TEST_SCHED_WAVES", b"CGPU_TEST_SCHED_SPINS", b"CGPU_TEST_NAT64_TAG_MASK"):
        assert name not in prod, name
    out = subprocess.run(["nm", "-D", "--undefined-only", str(N.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    assert not re.search(r"\bgetenv\b", out)
    test = N.TEST_LIB_PATH.read_bytes()
    assert b"CGPU_TEST_SCHED_SPINS" in test
    T = N.lib(test=True)
    assert T.cgpu_abi_version() == N.ABI_VERSION
