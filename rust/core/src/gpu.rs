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
use crate::packets::ip::v4::Ipv4;
use crate::packets::ip::v6::Ipv6;
use crate::packets::{Ethernet, Packet, Tcp, Udp};
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
    /// zero-copy entry points; once per memzone.  The memzone is whole pages
    /// (the library refuses anything else) and stays mapped while the
    /// context lives: the library borrows it (mbuf.rs:467-479).
    pub fn register_mempool(&mut self, base: *mut u8, len: usize) -> anyhow::Result<()> {
        check(unsafe { g::cgpu_host_register(self.0, base as *mut c_void, len) })
    }

    /// The context's device error word (cgpu_ctx_check): waits for `stream`
    /// (null: the default stream) and fails if a kernel of this context
    /// could not complete its part of a call since the last check.  The
    /// synchronous calls above check it themselves.
    pub fn check(&mut self, stream: *mut c_void) -> anyhow::Result<()> {
        check(unsafe { g::cgpu_ctx_check(self.0, stream) })
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

    /// `reconcile_all` (packets/mod.rs:297-300) in place over typed packets
    /// whose frames lie in a registered mempool (cgpu_reconcile_frames): each
    /// packet's layers come from its type, so nothing is parsed again.
    /// Returns one flag per packet: reconciled (true) or skipped.
    pub fn reconcile_typed<T: GpuTyped>(&mut self, pkts: &[T]) -> anyhow::Result<Vec<bool>> {
        let frames: Vec<*mut u8> = pkts.iter().map(|p| unsafe { p.mbuf().data_address(0) }).collect();
        let lens: Vec<u16> = pkts.iter().map(|p| p.mbuf().data_len() as u16).collect();
        let meta: Vec<u32> = pkts.iter().map(|p| p.gpu_meta()).collect();
        let mut st = vec![0u8; pkts.len()];
        check(unsafe {
            g::cgpu_reconcile_frames(self.0, frames.as_ptr(), lens.as_ptr(), meta.as_ptr(),
                                     pkts.len() as u32, T::ACCEPT, T::DEPTH, st.as_mut_ptr())
        })?;
        Ok(st.iter().map(|&s| s == g::cgpu_recon_status::CGPU_RECON_OK as u8).collect())
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

impl GpuContext {
    /// `cgpu_parse_frames_submit`: start the parse of a burst's frames and
    /// return its ticket at once.  The results land in `out`, whose vectors
    /// must not be touched (moved out, resized or dropped) until
    /// `wait_frames(ticket)` has returned.  At most two bursts in flight.
    pub fn submit_frames(&mut self, mbufs: &[Mbuf], flags: u32, out: &mut ParsedBurst)
                         -> anyhow::Result<u32> {
        let addrs: Vec<*const u8> =
            mbufs.iter().map(|m| unsafe { m.data_address(0) } as *const u8).collect();
        let lens: Vec<u16> = mbufs.iter().map(|m| m.data_len() as u16).collect();
        out.resize(mbufs.len());
        let mut ticket = 0u32;
        check(unsafe {
            g::cgpu_parse_frames_submit(self.0, addrs.as_ptr(), lens.as_ptr(), mbufs.len() as u32,
                                        flags, out.meta.as_mut_ptr(), out.csum.as_mut_ptr(),
                                        out.hash.as_mut_ptr(), &mut ticket)
        })?;
        Ok(ticket)
    }

    /// `cgpu_parse_frames_wait`: the burst of `ticket` is parsed.
    pub fn wait_frames(&mut self, ticket: u32) -> anyhow::Result<()> {
        check(unsafe { g::cgpu_parse_frames_wait(self.0, ticket) })
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
    /// g::CGPU_L3_*: the IP layer the parse found (0 none).
    pub fn l3(&self) -> u32 {
        (self.meta >> 16) & 3
    }
    /// g::CGPU_L4_*: the L4 layer the parse found (0 none).
    pub fn l4(&self) -> u32 {
        (self.meta >> 18) & 3
    }
    /// The flow hash of `Udp::flow` / `Tcp::flow` (udp.rs:151-159,
    /// tcp.rs:409-417) under DESIGN.md §4's convention.
    pub fn flow_hash(&self) -> u64 {
        self.hash
    }
    /// The IPv4 header and L4 checksums as stored equal the recomputed ones.
    pub fn ip_csum_ok(&self) -> bool {
        self.meta & g::CGPU_META_IP_CSUM_OK != 0
    }
    pub fn l4_csum_ok(&self) -> bool {
        self.meta & g::CGPU_META_L4_CSUM_OK != 0
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
    /// The burst goes across as (data_address, data_len, tailroom) triples
    /// read from the headers `rte_eth_rx_burst` has just written
    /// (cgpu_nat64_frames: the device touches only the frames, in one
    /// launch sequence and one synchronisation), and the
    /// lengths are set here as `Mbuf::shrink` / `extend` would leave them
    /// (mbuf.rs:225-275: data_off unchanged, data_len and pkt_len -20 / +20).
    pub fn nat_burst(&mut self, ctx: &mut GpuContext, direction: u32, mbufs: Vec<Mbuf>)
                     -> (Vec<(Mbuf, GpuDisposition)>, anyhow::Result<()>) {
        let ptrs: Vec<*mut ffi::rte_mbuf> = mbufs.into_iter().map(Mbuf::into_ptr).collect();
        let n = ptrs.len();
        let mut addrs: Vec<*const u8> = Vec::with_capacity(n);
        let mut lens: Vec<u16> = Vec::with_capacity(n);
        let mut tail: Vec<u16> = Vec::with_capacity(n);
        for &p in &ptrs {
            // the fields Mbuf::data_address / data_len / tailroom read (mbuf.rs:196-213)
            let m = unsafe { &*p };
            addrs.push(unsafe { (m.buf_addr as *const u8).offset(m.data_off as isize) });
            lens.push(m.data_len);
            tail.push(m.buf_len - m.data_off - m.data_len);
        }
        let mut out_len = vec![0u16; n];
        let mut disp = vec![0u8; n];
        let mut status = vec![0u8; n];
        let rc = check(unsafe {
            g::cgpu_nat64_frames(ctx.0, self.pm, direction, addrs.as_ptr(), lens.as_ptr(), tail.as_ptr(),
                                 n as u32, out_len.as_mut_ptr(), disp.as_mut_ptr(), status.as_mut_ptr())
        });
        let out = ptrs
            .into_iter()
            .enumerate()
            .map(|(i, p)| {
                let d = match (&rc, disp[i] as u32) {
                    (Err(_), _) => GpuDisposition::Abort(0),
                    (Ok(()), g::cgpu_disposition::CGPU_ACT) => {
                        let m = unsafe { &mut *p };
                        let grown = out_len[i] as u32 > m.data_len as u32;
                        m.pkt_len = if grown { m.pkt_len + 20 } else { m.pkt_len - 20 };
                        m.data_len = out_len[i];
                        GpuDisposition::Act
                    }
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

/// The layer a per-packet status names (2 Ethernet, 3 IP, 4 L4): a typed
/// chain of depth d fails only on statuses of layers <= d, as
/// `p.parse::<Ethernet>()?.parse::<Ipv4>()?` never looks at L4.
fn status_layer(status: u32) -> u32 {
    use g::cgpu_pkt_status::*;
    match status {
        CGPU_PKT_ETH_BAD_OFFSET | CGPU_PKT_ETH_OUT_OF_BUFFER => 2,
        CGPU_PKT_NOT_IPV4 | CGPU_PKT_NOT_IPV6 | CGPU_PKT_NOT_IP | CGPU_PKT_L3_BAD_OFFSET
        | CGPU_PKT_L3_OUT_OF_BUFFER => 3,
        _ => 4,
    }
}

/// The reference's typed packets, built from the device parse instead of
/// `parse::<Ethernet>()?.parse::<Ipv4>()?.parse::<Udp4>()?`.  Each layer is
/// made by the `pub(crate)` constructor `from_device(envelope, offset)` that
/// rust/README.md adds to the layer's own file: the struct the reference's
/// `try_parse` returns (ethernet.rs:279-300, ip/v4.rs:427-442, ip/v6/mod.rs:
/// 274-289, udp.rs:287-302, tcp.rs:558-573), with the header pointer at the
/// envelope's payload offset, without `read_data`'s bounds check and the
/// `ensure!`s: the device's status byte says they passed.
pub trait GpuTyped: Packet + Sized {
    /// The accept set of the parse (g::CGPU_F_ACCEPT_*): the typed chain.
    const ACCEPT: u32;
    /// g::CGPU_LAYER_*: the layer the chain ends at.
    const DEPTH: u32;

    /// The typed packet, or the reference's error of the first layer of the
    /// chain that failed (its message as `try_parse` words it).
    fn from_gpu(mbuf: Mbuf, parsed: &Parsed) -> anyhow::Result<Self> {
        let st = parsed.status();
        if st != g::cgpu_pkt_status::CGPU_PKT_OK && status_layer(st) <= Self::DEPTH {
            return Err(anyhow::anyhow!("{}", status_str(st)));
        }
        // the layers the type names, as the parse found them (a packet of
        // another kind fails like try_parse's ensure! does)
        Self::check_kind(parsed)?;
        Ok(unsafe { Self::build(mbuf) })
    }

    /// The kind check of the typed chain against the parse's layers.
    fn check_kind(parsed: &Parsed) -> anyhow::Result<()>;

    /// The typed packet over `mbuf`, every layer's header at its envelope's
    /// payload offset.
    ///
    /// # Safety
    ///
    /// The device parse of these bytes found exactly these layers, in bounds.
    unsafe fn build(mbuf: Mbuf) -> Self;

    /// The meta word that describes this packet's layers to the reconcile
    /// kernel (status OK, Ethernet header length and VLAN bits, L3, L4).
    fn gpu_meta(&self) -> u32;
}

fn eth_meta(eth: &Ethernet) -> u32 {
    let hl = eth.header_len() as u32;
    let vlan = match hl {
        18 => g::CGPU_META_DOT1Q,
        22 => g::CGPU_META_QINQ,
        _ => 0,
    };
    (hl << 8) | vlan
}

fn kind_err(want: u32, got: u32, msg: &str) -> anyhow::Result<()> {
    if want == got {
        Ok(())
    } else {
        Err(anyhow::anyhow!("{}", msg))
    }
}

impl GpuTyped for Ethernet {
    const ACCEPT: u32 = 0;
    const DEPTH: u32 = g::CGPU_LAYER_L2;
    fn check_kind(_: &Parsed) -> anyhow::Result<()> {
        Ok(())
    }
    unsafe fn build(mbuf: Mbuf) -> Self {
        Ethernet::from_device(mbuf, 0)
    }
    fn gpu_meta(&self) -> u32 {
        eth_meta(self)
    }
}

impl GpuTyped for Ipv4 {
    const ACCEPT: u32 = g::CGPU_F_ACCEPT_V4;
    const DEPTH: u32 = g::CGPU_LAYER_L3;
    fn check_kind(p: &Parsed) -> anyhow::Result<()> {
        kind_err(g::CGPU_L3_IPV4, p.l3(), "not an IPv4 packet.")
    }
    unsafe fn build(mbuf: Mbuf) -> Self {
        let eth = <Ethernet as GpuTyped>::build(mbuf);
        let at = eth.payload_offset();
        Ipv4::from_device(eth, at)
    }
    fn gpu_meta(&self) -> u32 {
        eth_meta(self.envelope()) | (g::CGPU_L3_IPV4 << 16)
    }
}

impl GpuTyped for Ipv6 {
    const ACCEPT: u32 = g::CGPU_F_ACCEPT_V6;
    const DEPTH: u32 = g::CGPU_LAYER_L3;
    fn check_kind(p: &Parsed) -> anyhow::Result<()> {
        kind_err(g::CGPU_L3_IPV6, p.l3(), "not an IPv6 packet.")
    }
    unsafe fn build(mbuf: Mbuf) -> Self {
        let eth = <Ethernet as GpuTyped>::build(mbuf);
        let at = eth.payload_offset();
        Ipv6::from_device(eth, at)
    }
    fn gpu_meta(&self) -> u32 {
        eth_meta(self.envelope()) | (g::CGPU_L3_IPV6 << 16)
    }
}

/// Udp4 / Udp6 / Tcp4 / Tcp6 (udp.rs:358-361, tcp.rs:625-628).
macro_rules! gpu_l4 {
    ($ty:ident, $ip:ident, $l4:expr, $acc:expr, $msg:expr) => {
        impl GpuTyped for $ty<$ip> {
            const ACCEPT: u32 = <$ip as GpuTyped>::ACCEPT | $acc;
            const DEPTH: u32 = g::CGPU_LAYER_L4;
            fn check_kind(p: &Parsed) -> anyhow::Result<()> {
                <$ip as GpuTyped>::check_kind(p)?;
                kind_err($l4, p.l4(), $msg)
            }
            unsafe fn build(mbuf: Mbuf) -> Self {
                let ip = <$ip as GpuTyped>::build(mbuf);
                let at = ip.payload_offset();
                $ty::from_device(ip, at)
            }
            fn gpu_meta(&self) -> u32 {
                self.envelope().gpu_meta() | ($l4 << 18)
            }
        }
    };
}
gpu_l4!(Udp, Ipv4, g::CGPU_L4_UDP, g::CGPU_F_ACCEPT_UDP, "not a UDP packet.");
gpu_l4!(Udp, Ipv6, g::CGPU_L4_UDP, g::CGPU_F_ACCEPT_UDP, "not a UDP packet.");
gpu_l4!(Tcp, Ipv4, g::CGPU_L4_TCP, g::CGPU_F_ACCEPT_TCP, "not a TCP packet.");
gpu_l4!(Tcp, Ipv6, g::CGPU_L4_TCP, g::CGPU_F_ACCEPT_TCP, "not a TCP packet.");
