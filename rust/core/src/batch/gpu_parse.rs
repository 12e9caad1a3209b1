//! `core/src/batch/gpu_parse.rs` — burst-level GPU combinators for capsule's
//! Batch pipeline (drop-in: `mod gpu_parse; pub use self::gpu_parse::*;` in
//! core/src/batch/mod.rs; see rust/README.md).
//!
//! The reference pulls one packet per `Batch::next` (batch/mod.rs:122-135);
//! the GPU path works on whole bursts, so these combinators drain their
//! upstream burst in `replenish`, make one library call for its Act
//! packets, and then yield the results in upstream order.  Emit / Drop /
//! Abort pass through unchanged, as `FilterMap::next` passes them through
//! `Disposition::map` (filter_map.rs:73-81, mod.rs:73-86).  A failed parse
//! aborts the packet with the reference's error string, like a failing `?`
//! inside a `filter_map` closure.  Not compiled in this repository (no Rust
//! toolchain).
use super::{Batch, Disposition};
use crate::gpu::{status_str, GpuContext, GpuDisposition, GpuNat64, Parsed, ParsedBurst};
use crate::packets::{Internal, Packet};
use crate::Mbuf;
use anyhow::{anyhow, Result};
use std::collections::VecDeque;

/// An mbuf with its device parse results (meta, checksums, flow hash).
pub struct GpuParsed {
    mbuf: Mbuf,
    pub parsed: Parsed, // #[derive(Clone, Copy)]: meta / csum / hash of this packet
}

impl Packet for GpuParsed {
    type Envelope = Mbuf;
    fn envelope(&self) -> &Mbuf { &self.mbuf }
    fn envelope_mut(&mut self) -> &mut Mbuf { &mut self.mbuf }
    fn offset(&self) -> usize { 0 }
    fn header_len(&self) -> usize { 0 }
    unsafe fn clone(&self, internal: Internal) -> Self {
        GpuParsed { mbuf: Packet::clone(&self.mbuf, internal), parsed: self.parsed }
    }
    fn try_parse(_: Mbuf, _: Internal) -> Result<Self> {
        Err(anyhow!("GpuParsed is produced by GpuParse only."))
    }
    fn try_push(_: Mbuf, _: Internal) -> Result<Self> {
        Err(anyhow!("GpuParsed is produced by GpuParse only."))
    }
    fn deparse(self) -> Mbuf { self.mbuf }
}

pub struct GpuParse<B: Batch<Item = Mbuf>> {
    batch: B,
    ctx: GpuContext,
    flags: u32,
    out: ParsedBurst,
    ready: VecDeque<Disposition<GpuParsed>>,
}

impl<B: Batch<Item = Mbuf>> GpuParse<B> {
    pub fn new(batch: B, ctx: GpuContext, flags: u32) -> Self {
        GpuParse { batch, ctx, flags, out: ParsedBurst::default(), ready: VecDeque::new() }
    }
}

impl<B: Batch<Item = Mbuf>> Batch for GpuParse<B> {
    type Item = GpuParsed;

    fn replenish(&mut self) {
        self.batch.replenish();
        // the upstream burst: Act packets go to the device in one call, the
        // other dispositions keep their place (None marks an Act slot)
        let mut slots: Vec<Option<Disposition<Mbuf>>> = Vec::new();
        let mut act: Vec<Mbuf> = Vec::new();
        while let Some(d) = self.batch.next() {
            match d {
                Disposition::Act(m) => {
                    slots.push(None);
                    act.push(m);
                }
                other => slots.push(Some(other)),
            }
        }
        let (act, rc) = if act.is_empty() { (act, Ok(())) } else {
            self.ctx.parse_burst(act, self.flags, &mut self.out)
        };
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
                            let parsed = self.out.get(i);
                            if parsed.meta & 0xff == 0 {
                                Disposition::Act(GpuParsed { mbuf, parsed })
                            } else {
                                Disposition::Abort(anyhow!("{}", status_str(parsed.meta & 0xff)))
                            }
                        }
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


/// `install_6to4` / `install_4to6` (examples/nat64/main.rs:152-165) as one
/// combinator: the burst's Act mbufs are rewritten in place by the device
/// (data_len / pkt_len -20 / +20) and come back Act, Drop or Abort with the
/// reference's error, in upstream order.
pub struct GpuNat64Map<B: Batch<Item = Mbuf>> {
    batch: B,
    ctx: GpuContext,
    nat: GpuNat64,
    direction: u32,
    ready: VecDeque<Disposition<Mbuf>>,
}

impl<B: Batch<Item = Mbuf>> GpuNat64Map<B> {
    pub fn new(batch: B, ctx: GpuContext, nat: GpuNat64, direction: u32) -> Self {
        GpuNat64Map { batch, ctx, nat, direction, ready: VecDeque::new() }
    }
}

impl<B: Batch<Item = Mbuf>> Batch for GpuNat64Map<B> {
    type Item = Mbuf;

    fn replenish(&mut self) {
        self.batch.replenish();
        let mut slots: Vec<Option<Disposition<Mbuf>>> = Vec::new();
        let mut act: Vec<Mbuf> = Vec::new();
        while let Some(d) = self.batch.next() {
            match d {
                Disposition::Act(m) => {
                    slots.push(None);
                    act.push(m);
                }
                other => slots.push(Some(other)),
            }
        }
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
