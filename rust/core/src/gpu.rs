//! `core/src/gpu.rs` — capsule's side of the MI355X packet path.
//!
//! Drop-in module for the reference crate (add `mod gpu;` to core/src/lib.rs
//! and `capsule-gpu-ffi = { path = "../gpu-ffi" }` to core/Cargo.toml; see
//! rust/README.md).  It wraps include/capsule_gpu.h the way core/src/ffi.rs
//! wraps DPDK: a nonzero return code becomes an `Err` carrying the library's
//! message (`ToResult`, reference core/src/ffi.rs:86-141; the thread-local
//! code is `cgpu_last_error()`, the `_rte_errno()` analogue of
//! ffi/src/shim.c:24-26).  Not compiled in this repository (no Rust
//! toolchain); the same entry points are exercised from Python and C there.
//!
//! Ownership follows Mbuf (mbuf.rs:467-479): the library borrows packet
//! bytes for one call and never frees or keeps an mbuf.
use crate::Mbuf;
use crate::ffi;
use capsule_gpu_ffi as g;
use std::ffi::{c_void, CStr};
use std::net::IpAddr;
use std::ptr;

/// A call-level failure of the GPU library.
#[derive(Debug, thiserror::Error)]
#[error("capsule-gpu: {0} ({1})")]
pub struct GpuError(String, i32);

fn check(rc: i32) -> anyhow::Result<()> {
    if rc == 0 {
        return Ok(());
    }
    let msg = unsafe { CStr::from_ptr(g::cgpu_strerror(rc)) };
    Err(GpuError(msg.to_string_lossy().into_owned(), rc).into())
}

/// The reference's error text for a per-packet status byte ("not an IPv4
/// packet.", ...; ip/v4.rs:430, udp.rs:290, mbuf.rs:85-98).
pub fn status_str(status: u32) -> &'static str {
    unsafe { CStr::from_ptr(g::cgpu_pkt_status_str(status as i32)) }
        .to_str()
        .unwrap_or("unknown packet status.")
}

/// One per core thread / RX queue (runtime/core_map.rs:236-293: shared
/// nothing).  Send but not Sync, like Mbuf (mbuf.rs:484).
pub struct GpuContext(*mut g::cgpu_ctx);
unsafe impl Send for GpuContext {}

impl GpuContext {
    pub fn new(hip_device: i32) -> anyhow::Result<Self> {
        let mut p = ptr::null_mut();
        check(unsafe { g::cgpu_ctx_create(hip_device, &mut p) })?;
        Ok(GpuContext(p))
    }

    /// Page-lock and map a mempool's memzone (mempool.rs:64-106) for the
    /// zero-copy entry points; once per memzone.
    pub fn register_mempool(&mut self, base: *mut u8, len: usize) -> anyhow::Result<()> {
        check(unsafe { g::cgpu_host_register(self.0, base as *mut c_void, len) })
    }

    /// Parse a burst exactly as `PacketRx::receive` returns it (batch/mod.rs:
    /// 110-119): the rte_mbuf pointers go across as they are and the device
    /// reads the registered mempool.  The mbufs come back whether or not the
    /// call succeeded.
    pub fn parse_burst(&mut self, mbufs: Vec<Mbuf>, flags: u32, out: &mut ParsedBurst)
                       -> (Vec<Mbuf>, anyhow::Result<()>) {
        let ptrs: Vec<*mut ffi::rte_mbuf> = mbufs.into_iter().map(Mbuf::into_ptr).collect();
        out.resize(ptrs.len());
        let rc = check(unsafe {
            g::cgpu_parse_mbufs(self.0, ptrs.as_ptr() as *const *mut c_void, ptrs.len() as u32,
                                flags, g::CGPU_INGRESS_ZERO_COPY, out.meta.as_mut_ptr(),
                                out.csum.as_mut_ptr(), out.hash.as_mut_ptr(), ptr::null_mut())
        });
        let mbufs = ptrs.into_iter().map(|p| unsafe { Mbuf::from_ptr(p) }).collect();
        (mbufs, rc)
    }

    /// The same burst as (data_address, data_len) pairs: the core reads the
    /// mbuf headers it has just written, the device reads only the frames.
    pub fn parse_burst_frames(&mut self, mbufs: &[Mbuf], flags: u32, out: &mut ParsedBurst)
                              -> anyhow::Result<()> {
        let addrs: Vec<*const u8> =
            mbufs.iter().map(|m| unsafe { m.data_address(0) } as *const u8).collect();
        let lens: Vec<u16> = mbufs.iter().map(|m| m.data_len() as u16).collect();
        out.resize(mbufs.len());
        check(unsafe {
            g::cgpu_parse_frames(self.0, addrs.as_ptr(), lens.as_ptr(), mbufs.len() as u32, flags,
                                 g::CGPU_INGRESS_ZERO_COPY, out.meta.as_mut_ptr(),
                                 out.csum.as_mut_ptr(), out.hash.as_mut_ptr(), ptr::null_mut())
        })
    }
}

impl Drop for GpuContext {
    fn drop(&mut self) {
        unsafe { g::cgpu_ctx_destroy(self.0) }
    }
}

/// One packet's results: the meta word (status byte, layer kinds, CSUM_OK
/// bits), the checksum values and the flow hash.
#[derive(Clone, Copy, Debug, Default)]
pub struct Parsed {
    pub meta: u32,
    pub csum: u32,
    pub hash: u64,
}

impl Parsed {
    pub fn status(&self) -> u32 {
        self.meta & 0xff
    }
    pub fn is_ok(&self) -> bool {
        self.status() == g::cgpu_pkt_status::CGPU_PKT_OK
    }
    /// Ethernet::header_len (ethernet.rs:253-261): 14, 18 or 22.
    pub fn eth_len(&self) -> usize {
        ((self.meta >> 8) & 0xff) as usize
    }
}

/// A burst's results, SoA as the ABI writes them.
#[derive(Default)]
pub struct ParsedBurst {
    pub meta: Vec<u32>,
    pub csum: Vec<u32>,
    pub hash: Vec<u64>,
}

impl ParsedBurst {
    pub fn resize(&mut self, n: usize) {
        self.meta.resize(n, 0);
        self.csum.resize(n, 0);
        self.hash.resize(n, 0);
    }
    pub fn get(&self, i: usize) -> Parsed {
        Parsed { meta: self.meta[i], csum: self.csum[i], hash: self.hash[i] }
    }
}

/// A device-resident burst (the cgpu_batch a device pipeline keeps in HBM):
/// arena / off / len / meta are device pointers owned by the caller, plus a
/// device scratch word area for per-call records.  Calls are asynchronous
/// on `stream` (a hipStream_t; null = the legacy default stream).
pub struct DeviceBurst {
    pub arena: *mut u8,
    pub arena_len: u64,
    pub off: *const u32,
    pub len: *const u16,
    pub meta: *mut u32,
    pub n: u32,
    pub scratch: *mut u8,
    pub stream: *mut c_void,
}

extern "C" {
    // libamdhip64 (linked by gpu-ffi/build.rs): hipMemcpy(dst, src, bytes, kind)
    fn hipMemcpy(dst: *mut c_void, src: *const c_void, bytes: usize, kind: i32) -> i32;
}

impl DeviceBurst {
    fn batch(&self) -> g::cgpu_batch {
        g::cgpu_batch { arena: self.arena, arena_len: self.arena_len, off: self.off, len: self.len,
                        n: self.n }
    }

    /// The parse chain + checksums + flow hash into `meta` (and the optional
    /// device arrays), as cgpu_parse_batch documents.
    pub fn parse(&self, ctx: &mut GpuContext, flags: u32, csum: *mut u32, hash: *mut u64)
                 -> anyhow::Result<()> {
        let out = g::cgpu_parse_out { meta: self.meta, csum, flow_hash: hash,
                                      fields: ptr::null_mut(), ext: ptr::null_mut() };
        let b = self.batch();
        check(unsafe { g::cgpu_parse_batch(ctx.0, &b, flags, &out, self.stream) })
    }

    /// `udp.set_src_ip(ip)?` (udp.rs:174-201) for every UDP/TCP packet of the
    /// burst; per-packet errors ("cannot mix IPv4 and IPv6 addresses.") come
    /// back in `status` (device u8 [n]).
    pub fn set_src_ip(&self, ctx: &mut GpuContext, ip: IpAddr, status: *mut u8)
                      -> anyhow::Result<()> {
        let mut a = g::cgpu_ip_addr::default();
        match ip {
            IpAddr::V4(v4) => {
                a.family = 4;
                a.octets[..4].copy_from_slice(&v4.octets());
            }
            IpAddr::V6(v6) => {
                a.family = 6;
                a.octets.copy_from_slice(&v6.octets());
            }
        }
        // the address record must be device-visible: copy it into the scratch
        let sz = std::mem::size_of::<g::cgpu_ip_addr>();
        if unsafe { hipMemcpy(self.scratch as *mut c_void, &a as *const _ as *const c_void, sz, 1) } != 0 {
            return Err(GpuError("hipMemcpy".into(), 0).into());
        }
        check(unsafe {
            g::cgpu_set_ip(ctx.0, self.arena, self.arena_len, self.off, self.len, self.meta, self.n,
                           self.scratch as *const g::cgpu_ip_addr, 0, ptr::null(), 0, status,
                           self.stream)
        })
    }

    /// `packet.reconcile_all()` (packets/mod.rs:297-300) for every packet of
    /// the burst, held at `depth` (g::CGPU_LAYER_L4 / _L3 / _L2) with the
    /// layers its parse recorded: UDP length + checksum, TCP / ICMP checksum,
    /// IPv4 total_length + header checksum, IPv6 payload_length, in place.
    /// `flags`: the accept set of the parse.
    pub fn reconcile_all(&self, ctx: &mut GpuContext, flags: u32, depth: u32, status: *mut u8)
                         -> anyhow::Result<()> {
        check(unsafe {
            g::cgpu_reconcile(ctx.0, self.arena, self.arena_len, self.off, self.len, self.meta,
                              self.n, flags, depth, status, self.stream)
        })
    }

    /// `batch.group_by(|p| class, ...)` (group_by.rs:143-172) by the parse's
    /// layer kinds: arm 0 v4/UDP, 1 v4/TCP, 2 v6/UDP, 3 v6/TCP, 4 the rest.
    pub fn group_by_class(&self, ctx: &mut GpuContext, idx: *mut u32, group_off: *mut u32)
                          -> anyhow::Result<()> {
        check(unsafe {
            g::cgpu_group_by(ctx.0, self.meta as *const c_void, g::CGPU_KEY_META_CLASS, self.n, 5,
                             idx, group_off, self.stream)
        })
    }
}

/// examples/nat64's PORT_MAP / ADDR_MAP / NEXT_PORT (main.rs:37-53) on the
/// device, for `install_6to4` / `install_4to6` (main.rs:152-165) over
/// rte_mbuf bursts.
pub struct GpuNat64 {
    pm: *mut g::cgpu_portmap,
}
unsafe impl Send for GpuNat64 {}

/// Act / Drop / Abort per packet (batch/mod.rs:54-107) as the device decided.
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub enum GpuDisposition {
    Act,
    Drop,
    Abort(u32),
}

impl GpuNat64 {
    /// `capacity_log2`: table slots (keep the load below one half);
    /// `first_port`: NEXT_PORT's start (1025 in the reference, main.rs:42).
    pub fn new(ctx: &mut GpuContext, capacity_log2: u32, first_port: u16) -> anyhow::Result<Self> {
        let mut pm = ptr::null_mut();
        check(unsafe { g::cgpu_portmap_create(ctx.0, capacity_log2, first_port, &mut pm) })?;
        Ok(GpuNat64 { pm })
    }

    pub fn next_port(&self) -> anyhow::Result<u16> {
        let mut p = 0u16;
        check(unsafe { g::cgpu_portmap_next_port(self.pm, &mut p) })?;
        Ok(p)
    }

    /// Rewrite a burst in place in its mbufs (6to4: g::CGPU_NAT64_6TO4,
    /// 4to6: g::CGPU_NAT64_4TO6): the mbufs come back with data_len / pkt_len
    /// adjusted for Act packets and a disposition each, in burst order.
    pub fn nat_burst(&mut self, ctx: &mut GpuContext, direction: u32, mbufs: Vec<Mbuf>)
                     -> (Vec<(Mbuf, GpuDisposition)>, anyhow::Result<()>) {
        let ptrs: Vec<*mut ffi::rte_mbuf> = mbufs.into_iter().map(Mbuf::into_ptr).collect();
        let n = ptrs.len();
        let mut disp = vec![0u8; n];
        let mut status = vec![0u8; n];
        let rc = check(unsafe {
            g::cgpu_nat64_mbufs(ctx.0, self.pm, direction, ptrs.as_ptr() as *const *mut c_void,
                                n as u32, disp.as_mut_ptr(), status.as_mut_ptr())
        });
        let out = ptrs
            .into_iter()
            .enumerate()
            .map(|(i, p)| {
                let d = match (&rc, disp[i] as u32) {
                    (Err(_), _) => GpuDisposition::Abort(0),
                    (Ok(()), g::cgpu_disposition::CGPU_ACT) => GpuDisposition::Act,
                    (Ok(()), g::cgpu_disposition::CGPU_DROP) => GpuDisposition::Drop,
                    (Ok(()), _) => GpuDisposition::Abort(status[i] as u32),
                };
                (unsafe { Mbuf::from_ptr(p) }, d)
            })
            .collect();
        (out, rc)
    }
}

impl Drop for GpuNat64 {
    fn drop(&mut self) {
        unsafe { g::cgpu_portmap_destroy(self.pm) }
    }
}
