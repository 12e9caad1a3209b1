// ingress.hip — zero-copy ingress of an rte_mbuf burst: the device reads the
// mbufs and their frames straight from page-locked host memory (a mempool
// registered with cgpu_host_register) over PCIe and lays the burst out in
// HBM as a cgpu_batch (64-byte slots), ready for the parse kernel.
//
// Reference: the rte_mbuf fields read are buf_addr, data_off and data_len at
// the DPDK 19.11 offsets of the bindgen layout test
// (ffi/src/bindings_rustdoc.rs:6869-6898); the frame is
// buf_addr + data_off .. + data_len, first segment only, as Mbuf::data_len /
// data_address / read_data (core/src/dpdk/mbuf.rs:196-205, 313-327).
//
// Quads of lanes read the mbuf headers (one 64-B request per mbuf) -- or the
// caller hands over (data_address, data_len) pairs and no header is read --
// the wave
// allocates its slots with one atomic, and then 16-lane groups copy four
// frames at a time, 16 B per lane, all of a wave's first-256-B loads in
// flight before any store.  Every host address is translated through the
// registered regions and range-checked first: a pointer outside them, or a
// frame that runs past its own buffer, is counted (the call fails) and never
// dereferenced; for nat64 egress the check covers every byte the rewritten
// frame may occupy.  No slot is written past the arena's capacity.
#include "capsule_gpu.h"
#include "device_common.hpp"
#include "kernels.hpp"

namespace cgpu {

namespace {

constexpr uint32_t kBlock = 256;

// host [addr, addr + size) -> device address, if inside a registered region
__device__ __forceinline__ bool translate(const GatherArgs &g, uint64_t addr, uint64_t size,
                                          uint64_t &dev) {
  for (uint32_t r = 0; r < g.nreg; ++r) {
    const HostRegion &h = g.reg[r];
    if (addr >= h.host_base && addr - h.host_base <= h.bytes && size <= h.bytes - (addr - h.host_base)) {
      dev = h.dev_base + (addr - h.host_base);
      return true;
    }
  }
  return false;
}

__device__ __forceinline__ u32x4 load_host16(uint64_t dev, uint32_t avail) {
  const uint8_t *p = reinterpret_cast<const uint8_t *>(dev);
  if ((dev & 15u) == 0u && avail >= 16u) return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
  u32x4 v = {0u, 0u, 0u, 0u};
  if ((dev & 3u) == 0u && avail >= 16u) {
    const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
    return u32x4{q[0], q[1], q[2], q[3]};
  }
  for (uint32_t b = 0; b < 16u && b < avail; ++b) v[b >> 2] |= (uint32_t)p[b] << (8u * (b & 3u));
  return v;
}

// The frame of mbuf i: buf_addr + data_off, data_len, checked and translated.
__device__ __forceinline__ void mbuf_frame(const GatherArgs &g, uint32_t i, uint32_t lane, bool valid,
                                           uint64_t &src, uint32_t &L) {
  // --- the mbuf header: buf_addr @0, data_off @16, data_len @40 --------------
  // Read cooperatively: in round r the quad of lanes 4m..4m+3 loads bytes
  // 0..47 of mbuf 16r + m as three 16-B pieces of one 64-B segment (one PCIe
  // read request instead of three small ones per mbuf); the owner lane then
  // picks its fields up with ds_bpermute.
  uint64_t dm = 0;
  const bool mok = valid && translate(g, g.mbufs[i], CGPU_MBUF_SIZE, dm);
  if (valid && !mok) atomicAdd(g.bad, 1u);
  const uint32_t q = lane & 3u;
  u32x4 H[4];
#pragma unroll
  for (uint32_t r = 0; r < 4u; ++r) {
    const uint32_t m = 16u * r + (lane >> 2);
    const uint64_t dmm = __shfl(dm, (int)m);
    const bool okm = __shfl((int)mok, (int)m) != 0;
    H[r] = u32x4{0u, 0u, 0u, 0u};
    // the whole 64-B segment: buf_addr @0, data_off @16, pkt_len @36,
    // data_len @40, buf_len @54
    if (okm) H[r] = *reinterpret_cast<const u32x4 *>(dmm + 16u * q);
  }
  const uint32_t r_own = lane >> 4, src_lane = 4u * (lane & 15u);
  uint32_t ba_lo = 0, ba_hi = 0, doff = 0, dlen = 0, plen = 0, blen = 0;
#pragma unroll
  for (uint32_t r = 0; r < 4u; ++r) {
    const uint32_t lo = __shfl(H[r][0], (int)src_lane), hi = __shfl(H[r][1], (int)src_lane);
    const uint32_t d16 = __shfl(H[r][0], (int)(src_lane + 1u));  // bytes 16..19
    const uint32_t d40 = __shfl(H[r][2], (int)(src_lane + 2u));  // bytes 40..43
    const uint32_t d36 = __shfl(H[r][1], (int)(src_lane + 2u));  // bytes 36..39
    const uint32_t d52 = __shfl(H[r][1], (int)(src_lane + 3u));  // bytes 52..55
    if (r == r_own) {
      ba_lo = lo;
      ba_hi = hi;
      doff = d16 & 0xffffu;
      dlen = d40 & 0xffffu;
      plen = d36;
      blen = d52 >> 16;
    }
  }
  src = 0;
  L = 0;
  bool ok = false;
  if (mok) {
    // the frame lies in its own buffer (data_off + data_len <= buf_len, the
    // invariant of every mbuf Mbuf::extend / shrink maintain) and in a
    // registered region
    const uint64_t buf_addr = ((uint64_t)ba_hi << 32) | ba_lo;
    // with the bytes a 4to6 rewrite may grow into (extend's tailroom check)
    const uint32_t tail = (blen - doff - dlen) & 0xffffu;
    const uint32_t span = dlen + (g.slot_extra != 0u && tail > g.slot_extra ? g.slot_extra : 0u);
    ok = doff + dlen <= blen && (dlen == 0u || translate(g, buf_addr + doff, span, src));
    L = ok ? dlen : 0u;
    if (!ok) atomicAdd(g.bad, 1u);
  }
  if (valid && g.mb_dev) {
    g.mb_dev[i] = ok ? dm : 0ull;
    g.fr_dev[i] = src;
    g.pkt_len[i] = plen;
    g.tailroom[i] = (blen - doff - dlen) & 0xffffu;  // u16 arithmetic, as Mbuf::tailroom
  }
}

__global__ __launch_bounds__(kBlock) void mbuf_gather(GatherArgs g) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  const bool valid = i < g.n;
  uint64_t src = 0;
  uint32_t L = 0;
  if (g.frames) {
    // (data_address, data_len) pairs from the RX core: the frame alone, one
    // request per 64 B of frame, no mbuf header line
    const uint32_t fl = valid ? g.flen[i] : 0u;
    // the bytes the egress may write too: a 4to6 frame grows by slot_extra
    // when its tailroom allows (the scatter's extend check)
    const uint32_t ft = valid && g.ftail ? g.ftail[i] : 0u;
    const uint32_t span = fl + (g.slot_extra != 0u && ft > g.slot_extra ? g.slot_extra : 0u);
    const bool ok = valid && (fl == 0u || translate(g, g.frames[i], span, src));
    if (valid && !ok) atomicAdd(g.bad, 1u);
    L = ok ? fl : 0u;
    if (valid && g.mb_dev) {  // egress records: the frame only, no header to update
      g.mb_dev[i] = 0ull;
      g.fr_dev[i] = ok ? src : 0ull;
      g.pkt_len[i] = 0u;
      g.tailroom[i] = g.ftail ? g.ftail[i] : 0u;
    }
  } else {
    mbuf_frame(g, i, lane, valid, src, L);
  }
  if (!g.arena) return;  // validate only (wave-uniform)
  // --- slots: one atomic per wave, prefix within the wave ---------------------
  const uint32_t slot = (L + g.slot_extra + 63u) & ~63u;
  uint32_t incl = slot;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += y;
  }
  const uint32_t total = __shfl(incl, 63);
  uint64_t base = 0;
  if (lane == 0u && total) base = atomicAdd(g.cursor, (unsigned long long)total);
  base = __shfl(base, 0);
  // A slot past the arena is not written (the frame reads as empty); the
  // cursor still counts it, and the host redoes the chunk with an arena of
  // the size the cursor reports (frames of a jumbo mempool).
  const uint64_t o64 = base + incl - slot;
  if (o64 + slot > g.arena_cap) L = 0u;
  const uint32_t o = (uint32_t)o64;
  if (valid) {
    g.off[i] = o;
    g.len[i] = (uint16_t)L;
  }
  // --- copy: 16-lane groups, 4 frames per round, 16 rounds per wave ------------
  const uint32_t grp = lane >> 4, gl = lane & 15u;
  u32x4 v[16];
#pragma unroll
  for (uint32_t r = 0; r < 16u; ++r) {
    const uint32_t f = 4u * r + grp;
    const uint64_t fs = __shfl(src, (int)f);
    const uint32_t fl = __shfl(L, (int)f);
    v[r] = u32x4{0u, 0u, 0u, 0u};
    if (16u * gl < fl) v[r] = load_host16(fs + 16u * gl, fl - 16u * gl);
  }
#pragma unroll
  for (uint32_t r = 0; r < 16u; ++r) {
    const uint32_t f = 4u * r + grp;
    const uint32_t fl = __shfl(L, (int)f), fo = __shfl(o, (int)f);
    if (16u * gl < fl) *reinterpret_cast<u32x4 *>(g.arena + fo + 16u * gl) = v[r];
  }
  // frames longer than 256 B: the rest, round by round
  for (uint32_t r = 0; r < 16u; ++r) {
    const uint32_t f = 4u * r + grp;
    const uint64_t fs = __shfl(src, (int)f);
    const uint32_t fl = __shfl(L, (int)f), fo = __shfl(o, (int)f);
    if (!__ballot(fl > 256u)) continue;
    for (uint32_t pos = 256u + 16u * gl; pos < fl; pos += 256u)
      *reinterpret_cast<u32x4 *>(g.arena + fo + pos) = load_host16(fs + pos, fl - pos);
  }
}

// Egress for nat64 over mbufs: every ACT frame back into its own mbuf, at
// buf_addr + data_off (Mbuf::shrink / extend move bytes, never data_off,
// mbuf.rs:225-270), and data_len / pkt_len adjusted by the same delta.  4to6
// first applies extend's tailroom check (`20 < tailroom`, mbuf.rs:228) with
// the mbuf's real buf_len: a frame without the room is ABORT / NOT_RESIZED
// and its mbuf is left as it was.  A 16-lane group per frame, 16 B per lane
// and 256 B per group and instruction, as posted PCIe writes to the
// registered mempool: every frame's bytes are in flight after one read of
// its metadata and one of its output, so a burst of a few thousand frames
// costs a couple of round trips, not one per frame of a wave.
__global__ __launch_bounds__(kBlock) void mbuf_scatter(ScatterArgs a) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t i = t >> 4, gl = t & 15u;
  if (i >= a.n) return;
  if (a.disposition[i] != CGPU_ACT || a.fr_dev[i] == 0ull) return;
  if (a.delta > 0 && !((uint32_t)a.delta < a.tailroom[i])) {
    if (gl == 0u) {
      a.disposition[i] = CGPU_ABORT;
      a.status[i] = CGPU_PKT_NOT_RESIZED;
    }
    return;
  }
  const uint32_t nl = a.out_len[i], fo = a.out_off[i];
  const uint64_t fd = a.fr_dev[i];
  if (gl == 0u && a.mb_dev != nullptr && a.mb_dev[i] != 0ull) {  // rte_mbufs (not frame pairs)
    uint8_t *h = reinterpret_cast<uint8_t *>(a.mb_dev[i]);
    *reinterpret_cast<uint16_t *>(h + CGPU_MBUF_DATA_LEN_OFF) = (uint16_t)nl;
    *reinterpret_cast<uint32_t *>(h + CGPU_MBUF_PKT_LEN_OFF) = a.pkt_len[i] + (uint32_t)a.delta;
  }
  for (uint32_t pos = 16u * gl; pos < nl; pos += 256u) {
    const u32x4 v = *reinterpret_cast<const u32x4 *>(a.out_arena + fo + pos);
    uint8_t *p = reinterpret_cast<uint8_t *>(fd + pos);
    const uint32_t r16 = nl - pos;
    if (((fd + pos) & 15u) == 0u && r16 >= 16u) {
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
    } else {
      for (uint32_t b = 0; b < 16u && b < r16; ++b) p[b] = (uint8_t)(v[b >> 2] >> (8u * (b & 3u)));
    }
  }
}

}  // namespace

hipError_t launch_mbuf_scatter(const ScatterArgs &a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(mbuf_scatter, dim3((uint32_t)(((uint64_t)a.n * 16u + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     s, a);
  return hipGetLastError();
}

hipError_t launch_mbuf_gather(const GatherArgs &g, hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  hipLaunchKernelGGL(mbuf_gather, dim3((g.n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, g);
  return hipGetLastError();
}

}  // namespace cgpu
