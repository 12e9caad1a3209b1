//! `core/src/batch/gpu_parse.rs` — burst-level GPU combinators for capsule's
//! Batch pipeline (drop-in: `mod gpu_parse; pub use self::gpu_parse::*;` in
//! core/src/batch/mod.rs; see rust/README.md).
//!
//! The reference pulls one packet per `Batch::next` (batch/mod.rs:122-135);
//! the GPU path works on whole bursts, so these combinators drain their
//! upstream in `replenish`, make one library call for its Act packets, and
//! then yield the results in upstream order.  One upstream burst is at most
//! RX_BURST_MAX = 32 mbufs (`PortQueue::receive`, dpdk/port.rs:149-171,
//! through `Poll::replenish`, batch/poll.rs:47-53), and a device round trip
//! per 32 packets costs more than the CPU parse it replaces (DESIGN.md §8:
//! about 20 us per synchronous call), so `replenish` keeps pulling upstream
//! bursts until it holds `target` Act packets (GPU_BURST_TARGET by default)
//! or a pull brings nothing (the RX queue is drained: a burst never waits
//! for packets that have not arrived).  Emit / Drop /
//! Abort pass through unchanged, as `FilterMap::next` passes them through
//! `Disposition::map` (filter_map.rs:73-81, mod.rs:73-86).  A failed parse
//! aborts the packet with the reference's error string, like a failing `?`
//! inside a `filter_map` closure.  Not compiled in this repository (no Rust
//! toolchain).
use super::{Batch, Disposition};
use crate::gpu::{status_str, GpuContext, GpuDisposition, GpuNat64, GpuTyped, Parsed, ParsedBurst};
use crate::Mbuf;
use anyhow::anyhow;
use std::collections::VecDeque;

/// `batch.map(|p| p.parse::<Ethernet>()?.parse::<Ipv4>()?.parse::<Udp4>())`
/// as one device call per burst: yields the reference's own typed packet
/// (`Udp4`, `Tcp6`, `Ipv4`, `Ethernet`, ...) built from the device parse, so
/// the closures downstream (`filter_map(|udp: Udp4| ...)`, `udp.src_port()`,
/// `udp.flow()`, `udp.reconcile_all()`) run unchanged and nothing is parsed
/// again on the CPU.  The device results the reference would compute on the
/// CPU afterwards (the flow hash, the checksum verification) reach an
/// optional `inspect_parsed` closure next to each packet.
pub struct GpuParse<B: Batch<Item = Mbuf>, T: GpuTyped> {
    batch: B,
    ctx: GpuContext,
    flags: u32,
    target: usize,
    double_buffer: bool,
    pending: Option<InFlight>,
    spare: ParsedBurst,
    ready: VecDeque<Disposition<T>>,
    on_parsed: Option<Box<dyn FnMut(&T, &Parsed)>>,
}

/// A gathered burst on its way through the device: its upstream slots (None
/// marks an Act packet), the Act mbufs, the results' buffers and the ticket
/// of its `cgpu_parse_frames_submit` (or the submit's error).
struct InFlight {
    slots: Vec<Option<Disposition<Mbuf>>>,
    act: Vec<Mbuf>,
    out: ParsedBurst,
    ticket: anyhow::Result<Option<u32>>,
}

/// Act packets a GPU combinator gathers from its upstream before one device
/// call (the synchronous call's fixed cost against the rate
/// of one core's CPU parse).
pub const GPU_BURST_TARGET: usize = 2048;

impl<B: Batch<Item = Mbuf>, T: GpuTyped> GpuParse<B, T> {
    /// The typed chain's accept set, with the checksums verified and the flow
    /// hash computed (g::CGPU_F_CSUM_IP | CSUM_L4 | FLOW_HASH).
    pub fn new(batch: B, ctx: GpuContext) -> Self {
        use capsule_gpu_ffi as g;
        let flags = T::ACCEPT | g::CGPU_F_CSUM_IP | g::CGPU_F_CSUM_L4 | g::CGPU_F_FLOW_HASH;
        Self::with_flags(batch, ctx, flags)
    }

    /// Explicit flags (T::ACCEPT is always added): e.g. no checksums.
    pub fn with_flags(batch: B, ctx: GpuContext, flags: u32) -> Self {
        GpuParse { batch, ctx, flags: flags | T::ACCEPT, target: GPU_BURST_TARGET,
                   double_buffer: true, pending: None, spare: ParsedBurst::default(),
                   ready: VecDeque::new(), on_parsed: None }
    }

    /// One burst in flight at a time: each replenish yields the burst it
    /// gathered (no overlap; the packets leave one poll earlier).  By
    /// default the device parses the burst just gathered while the packets
    /// of the previous one are yielded (2x the rate at 512 to
    /// 4,096 packets).
    pub fn single_buffered(mut self) -> Self {
        self.double_buffer = false;
        self
    }

    /// Act packets gathered per device call (1: one call per upstream burst).
    pub fn with_target(mut self, target: usize) -> Self {
        self.target = target.max(1);
        self
    }

    /// Called with each Act packet and its device results as it is yielded.
    pub fn inspect_parsed<F: FnMut(&T, &Parsed) + 'static>(mut self, f: F) -> Self {
        self.on_parsed = Some(Box::new(f));
        self
    }
}

/// Drains upstream bursts until `target` Act packets are in hand or a
/// replenish brings nothing: Act items in one vector (in order), the other
/// dispositions kept in their places (None marks an Act slot).  Every
/// upstream burst is drained to its end before the next replenish, so no
/// packet is lost (`Poll::replenish` replaces its queue, poll.rs:47-53).
fn drain_bursts<B: Batch>(batch: &mut B, target: usize)
                          -> (Vec<Option<Disposition<B::Item>>>, Vec<B::Item>) {
    let mut slots = Vec::new();
    let mut act = Vec::new();
    loop {
        batch.replenish();
        let before = slots.len();
        while let Some(d) = batch.next() {
            match d {
                Disposition::Act(p) => {
                    slots.push(None);
                    act.push(p);
                }
                other => slots.push(Some(other)),
            }
        }
        if act.len() >= target || slots.len() == before {
            break;
        }
    }
    (slots, act)
}

impl<B: Batch<Item = Mbuf>, T: GpuTyped> GpuParse<B, T> {
    /// Waits for a burst and yields it in upstream order.
    fn finish(&mut self, f: InFlight) {
        let InFlight { slots, act, out, ticket } = f;
        let rc = ticket.and_then(|t| match t {
            Some(t) => self.ctx.wait_frames(t),
            None => Ok(()),
        });
        let mut act = act.into_iter().enumerate();
        for s in slots {
            let d = match s {
                // Emit / Drop / Abort as they came (Act never reaches this arm)
                Some(d) => d.map(|_| unreachable!()),
                None => {
                    let (i, mbuf) = act.next().expect("one mbuf per Act slot");
                    match &rc {
                        // a failed call aborts the burst's packets; they are
                        // freed when dropped, like any aborted packet
                        Err(e) => Disposition::Abort(anyhow!("GPU parse failed: {}", e)),
                        Ok(()) => {
                            let parsed = out.get(i);
                            match T::from_gpu(mbuf, &parsed) {
                                Ok(pkt) => {
                                    if let Some(f) = self.on_parsed.as_mut() {
                                        f(&pkt, &parsed);
                                    }
                                    Disposition::Act(pkt)
                                }
                                Err(e) => Disposition::Abort(e),
                            }
                        }
                    }
                }
            };
            self.ready.push_back(d);
        }
        self.spare = out;
    }
}

impl<B: Batch<Item = Mbuf>, T: GpuTyped> Batch for GpuParse<B, T> {
    type Item = T;

    fn replenish(&mut self) {
        let (slots, act) = drain_bursts(&mut self.batch, self.target);
        let gathered = if slots.is_empty() { None } else {
            // (data_address, data_len) pairs: the device reads the frames
            // alone, in one launch (cgpu_parse_frames_submit's direct path)
            let mut out = std::mem::take(&mut self.spare);
            let ticket = if act.is_empty() { Ok(None) } else {
                self.ctx.submit_frames(&act, self.flags, &mut out).map(Some)
            };
            Some(InFlight { slots, act, out, ticket })
        };
        // the previous burst leaves while this one is parsed; with nothing
        // new gathered (the queue is drained) the pending burst leaves now
        if let Some(prev) = self.pending.take() {
            self.finish(prev);
        }
        if let Some(f) = gathered {
            if self.double_buffer {
                self.pending = Some(f);
            } else {
                self.finish(f);
            }
        }
    }

    fn next(&mut self) -> Option<Disposition<Self::Item>> {
        self.ready.pop_front()
    }
}

/// `batch.map(|mut p| { p.reconcile_all(); Ok(p) })` (packets/mod.rs:297-300)
/// over a burst of typed packets in one device call (cgpu_reconcile_frames):
/// the burst's frames are reconciled in place in the registered mempool,
/// from the packets' own layer (their type) outward, and come back Act in
/// upstream order.  Typically after closures that rewrote ports or
/// addresses: `GpuParse::<_, Udp4>::new(..).map(|mut u| { u.set_dst_port(53);
/// Ok(u) }).gpu_reconcile(ctx)`.
pub struct GpuReconcile<B: Batch<Item = T>, T: GpuTyped> {
    batch: B,
    ctx: GpuContext,
    target: usize,
    ready: VecDeque<Disposition<T>>,
}

impl<B: Batch<Item = T>, T: GpuTyped> GpuReconcile<B, T> {
    pub fn new(batch: B, ctx: GpuContext) -> Self {
        GpuReconcile { batch, ctx, target: GPU_BURST_TARGET, ready: VecDeque::new() }
    }

    /// Act packets gathered per device call.
    pub fn with_target(mut self, target: usize) -> Self {
        self.target = target.max(1);
        self
    }
}

impl<B: Batch<Item = T>, T: GpuTyped> Batch for GpuReconcile<B, T> {
    type Item = T;

    fn replenish(&mut self) {
        let (slots, act) = drain_bursts(&mut self.batch, self.target);
        let rc = if act.is_empty() { Ok(Vec::new()) } else { self.ctx.reconcile_typed(&act) };
        let mut act = act.into_iter().enumerate();
        for s in slots {
            let d = match s {
                Some(d) => d,
                None => {
                    let (i, pkt) = act.next().expect("one packet per Act slot");
                    match &rc {
                        Err(e) => Disposition::Abort(anyhow!("GPU reconcile failed: {}", e)),
                        // every typed packet reconciles (reconcile_all is
                        // infallible); skipped would mean a frame that
                        // shrank below its own headers
                        Ok(done) if done[i] => Disposition::Act(pkt),
                        Ok(_) => Disposition::Abort(anyhow!("reconcile skipped: the frame no longer holds its headers.")),
                    }
                }
            };
            self.ready.push_back(d);
        }
    }

    fn next(&mut self) -> Option<Disposition<Self::Item>> {
        self.ready.pop_front()
    }
}

/// The combinators as methods, like the reference's `Batch` provided methods
/// (batch/mod.rs:137-387).
pub trait GpuBatchExt: Batch + Sized {
    fn gpu_parse<T: GpuTyped>(self, ctx: GpuContext) -> GpuParse<Self, T>
    where
        Self: Batch<Item = Mbuf>,
    {
        GpuParse::new(self, ctx)
    }

    fn gpu_reconcile(self, ctx: GpuContext) -> GpuReconcile<Self, Self::Item>
    where
        Self::Item: GpuTyped,
    {
        GpuReconcile::new(self, ctx)
    }
}

impl<B: Batch> GpuBatchExt for B {}


/// `install_6to4` / `install_4to6` (examples/nat64/main.rs:152-165) as one
/// combinator: the burst's Act mbufs are rewritten in place by the device
/// (data_len / pkt_len -20 / +20) and come back Act, Drop or Abort with the
/// reference's error, in upstream order.
pub struct GpuNat64Map<B: Batch<Item = Mbuf>> {
    batch: B,
    ctx: GpuContext,
    nat: GpuNat64,
    direction: u32,
    target: usize,
    ready: VecDeque<Disposition<Mbuf>>,
}

impl<B: Batch<Item = Mbuf>> GpuNat64Map<B> {
    pub fn new(batch: B, ctx: GpuContext, nat: GpuNat64, direction: u32) -> Self {
        GpuNat64Map { batch, ctx, nat, direction, target: GPU_BURST_TARGET, ready: VecDeque::new() }
    }

    /// Act packets gathered per device call.
    pub fn with_target(mut self, target: usize) -> Self {
        self.target = target.max(1);
        self
    }
}

impl<B: Batch<Item = Mbuf>> Batch for GpuNat64Map<B> {
    type Item = Mbuf;

    fn replenish(&mut self) {
        let (slots, act) = drain_bursts(&mut self.batch, self.target);
        let (done, rc) = if act.is_empty() { (Vec::new(), Ok(())) } else {
            self.nat.nat_burst(&mut self.ctx, self.direction, act)
        };
        let mut done = done.into_iter();
        for s in slots {
            let d = match s {
                Some(d) => d,
                None => {
                    let (mbuf, gd) = done.next().expect("one mbuf per Act slot");
                    match (&rc, gd) {
                        (Err(e), _) => Disposition::Abort(anyhow!("GPU nat64 failed: {}", e)),
                        (Ok(()), GpuDisposition::Act) => Disposition::Act(mbuf),
                        (Ok(()), GpuDisposition::Drop) => Disposition::Drop(mbuf),
                        (Ok(()), GpuDisposition::Abort(st)) => Disposition::Abort(anyhow!("{}", status_str(st))),
                    }
                }
            };
            self.ready.push_back(d);
        }
    }

    fn next(&mut self) -> Option<Disposition<Self::Item>> {
        self.ready.pop_front()
    }
}
