// setip.hip — batched Udp/Tcp::set_src_ip / set_dst_ip (core/src/packets/
// udp.rs:174-201, tcp.rs:432-459): the address store plus the RFC 1624
// incremental L4 checksum update of checksum::compute_with_ipaddr
// (checksum.rs:202-220) and compute_inc (checksum.rs:182-195).
//
// One lane per packet.  The parse meta word already holds the layer offsets
// (eth header length, L3 and L4 kinds), so a lane touches only the address
// words and the checksum field of its own frame: 10 B read + 6 B written
// (IPv4) or 34 B + 18 B (IPv6) per address, next to the 4-B meta and the
// 6-B descriptor.  Frames sit at arbitrary byte offsets, so the fields are
// accessed bytewise; the accesses of neighbouring lanes fall in distinct
// frames, and L2 merges the partial lines.
#include "capsule_gpu.h"
#include "kernels.hpp"

namespace cgpu {

namespace {

constexpr uint32_t kBlock = 256;

__device__ __forceinline__ uint32_t ld16(const uint8_t *p) {
  return (uint32_t(p[0]) << 8) | p[1];
}

// checksum.rs:182-195: fold(~HC + sum(~m + m')), complemented.  `old` and
// `nw` are `words` big-endian u16 address words (2 for IPv4, 8 for IPv6).
__device__ __forceinline__ uint32_t update(uint32_t ck, uint8_t *addr, const uint8_t *nw,
                                           uint32_t words) {
  uint32_t acc = ~ck & 0xffffu;
  for (uint32_t w = 0; w < words; ++w) {
    acc += (~ld16(addr + 2 * w) & 0xffffu) + ld16(nw + 2 * w);
  }
  while (acc >> 16) acc = (acc >> 16) + (acc & 0xffffu);
  for (uint32_t b = 0; b < 2 * words; ++b) addr[b] = nw[b];  // envelope_mut().set_src/dst
  return ~acc & 0xffffu;
}

__global__ __launch_bounds__(kBlock) void set_ip_kernel(SetIpArgs a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.n) return;
  const uint32_t m = a.meta[i];
  const uint32_t l3 = (m >> 16) & 3u, l4 = (m >> 18) & 3u, ext = (m >> 24) & 3u;
  const uint32_t eth = (m >> 8) & 0xffu;
  const uint32_t off = a.off[i], len = a.len[i];
  const bool udp = l4 == CGPU_L4_UDP, v6 = l3 == CGPU_L3_IPV6;
  const uint32_t l4_off = eth + (v6 ? 40u : 20u);
  // Only frames the parse accepted as Udp/Tcp (and still in the arena).
  const bool ok = (m & 0xffu) == CGPU_PKT_OK && (udp || l4 == CGPU_L4_TCP) && ext == 0u &&
                  l3 != CGPU_L3_NONE && l4_off + (udp ? 8u : 20u) <= len &&
                  (uint64_t)off + len <= a.arena_len;
  if (!ok) {
    if (a.status) a.status[i] = CGPU_SETIP_SKIPPED;
    return;
  }
  uint8_t *f = a.arena + off;
  uint8_t *ckp = f + l4_off + (udp ? 6u : 16u);
  const uint32_t fam = v6 ? 6u : 4u, words = v6 ? 8u : 2u;
  uint32_t ck = ld16(ckp);
  uint32_t st = CGPU_SETIP_OK;
  if (a.src) {
    const cgpu_ip_addr &s = a.src[(size_t)i * a.src_stride];
    if (s.family != fam) {
      st = CGPU_SETIP_SRC_MISMATCH;
    } else {
      ck = update(ck, f + eth + (v6 ? 8u : 12u), s.octets, words);
      if (udp && ck == 0u) ck = 0xffffu;  // Udp::set_checksum (udp.rs:132-141)
    }
  }
  if (a.dst && st == CGPU_SETIP_OK) {
    const cgpu_ip_addr &d = a.dst[(size_t)i * a.dst_stride];
    if (d.family != fam) {
      st = CGPU_SETIP_DST_MISMATCH;
    } else {
      ck = update(ck, f + eth + (v6 ? 24u : 16u), d.octets, words);
      if (udp && ck == 0u) ck = 0xffffu;
    }
  }
  ckp[0] = uint8_t(ck >> 8);
  ckp[1] = uint8_t(ck);
  if (a.status) a.status[i] = uint8_t(st);
}

}  // namespace

hipError_t launch_set_ip(const SetIpArgs &a, hipStream_t s) {
  const dim3 grid((a.n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(set_ip_kernel, grid, dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace cgpu
