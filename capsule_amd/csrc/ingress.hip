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
// One lane per mbuf reads its header (one PCIe round trip), the wave
// allocates its slots with one atomic, and then 16-lane groups copy four
// frames at a time, 16 B per lane, all of a wave's first-256-B loads in
// flight before any store.  Every host address is translated through the
// registered regions and range-checked first: a pointer outside them is
// counted (the call fails) and never dereferenced.
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

__global__ __launch_bounds__(kBlock) void mbuf_gather(GatherArgs g) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  const bool valid = i < g.n;
  // --- the mbuf header: buf_addr, data_off, data_len --------------------------
  uint64_t src = 0;
  uint32_t L = 0;
  bool ok = false;
  if (valid) {
    uint64_t dm;
    if (translate(g, g.mbufs[i], CGPU_MBUF_SIZE, dm)) {
      const uint64_t buf_addr = *reinterpret_cast<const uint64_t *>(dm + CGPU_MBUF_BUF_ADDR_OFF);
      const uint32_t data_off = *reinterpret_cast<const uint16_t *>(dm + CGPU_MBUF_DATA_OFF_OFF);
      const uint32_t data_len = *reinterpret_cast<const uint16_t *>(dm + CGPU_MBUF_DATA_LEN_OFF);
      ok = data_len == 0u || translate(g, buf_addr + data_off, data_len, src);
      L = ok ? data_len : 0u;
    }
    if (!ok) atomicAdd(g.bad, 1u);
  }
  // --- slots: one atomic per wave, prefix within the wave ---------------------
  const uint32_t slot = (L + 63u) & ~63u;
  uint32_t incl = slot;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += y;
  }
  const uint32_t total = __shfl(incl, 63);
  uint32_t base = 0;
  if (lane == 0u && total) base = atomicAdd(g.cursor, total);
  base = __shfl(base, 0);
  const uint32_t o = base + incl - slot;
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

}  // namespace

hipError_t launch_mbuf_gather(const GatherArgs &g, hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  hipLaunchKernelGGL(mbuf_gather, dim3((g.n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, g);
  return hipGetLastError();
}

}  // namespace cgpu
