// group_by.hip — device-side `group_by` (core/src/batch/group_by.rs:143-172):
// a stable partition of a batch's packet indices into the arms of a
// selector, with the catch-all arm of the `compose!` macro
// (group_by.rs:186-200) for keys that name no arm.
//
// The reference feeds packets one at a time through the arm the selector
// picks, in arrival order, so each arm sees its packets in batch order.  The
// device equivalent is a stable counting sort over small keys:
//   pass 1 (count)   one wave per 1024-packet tile; per distinct key of a
//                    64-packet row: ballot, popcount, the count kept in the
//                    VGPR lane named by the key (lane k holds arm k)
//   pass 2 (scan)    one workgroup: exclusive scan of the arm-major
//                    [arm][tile] counts = each tile's first output slot per arm
//   pass 3 (scatter) the count pass again; a packet's slot is its tile's base
//                    for its arm + the arm's running count + mbcnt of the ballot
// Traffic per packet: key (1 B, or a 4-B meta word) read twice, 4-B index
// written once.  No LDS, no atomics.
#include "capsule_gpu.h"
#include "kernels.hpp"

namespace cgpu {

namespace {

constexpr uint32_t kIter = 16;          // 64-packet rows per tile
constexpr uint32_t kTile = 64 * kIter;  // packets per tile (one wave)
constexpr uint32_t kBlock = 256;
constexpr uint32_t kScanBlock = 1024;

__device__ __forceinline__ uint32_t arm_of(const GroupByArgs &a, uint32_t i) {
  uint32_t k;
  if (a.kind == CGPU_KEY_META_CLASS) {
    const uint32_t m = static_cast<const uint32_t *>(a.key)[i];
    const uint32_t l3 = (m >> 16) & 3u, l4 = (m >> 18) & 3u;
    // arms 0-3: the UDP/TCP classes; 4: failed parses and every other L4
    // layer (ICMP), so no ICMP frame reaches a Udp or Tcp arm
    const bool udp_tcp = l4 == CGPU_L4_UDP || l4 == CGPU_L4_TCP;
    k = ((m & 0xffu) || !udp_tcp)
            ? 4u
            : (((l3 == CGPU_L3_IPV6) ? 2u : 0u) | ((l4 == CGPU_L4_TCP) ? 1u : 0u));
  } else {
    k = static_cast<const uint8_t *>(a.key)[i];
  }
  return k < a.groups - 1u ? k : a.groups - 1u;  // no arm -> catch-all
}

template <bool SCATTER>
__global__ __launch_bounds__(kBlock) void group_by_pass(GroupByArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t tile = blockIdx.x * (kBlock / 64u) + (threadIdx.x >> 6);
  if (tile >= a.tiles) return;  // wave-uniform
  const uint32_t base = tile * kTile;
  uint32_t key[kIter];
#pragma unroll
  for (uint32_t j = 0; j < kIter; ++j) {
    const uint32_t i = base + j * 64u + lane;
    key[j] = i < a.n ? arm_of(a, i) : 0xffu;
  }
  uint32_t cnt = 0;
  if (SCATTER && lane < a.groups) cnt = a.counts[lane * a.tiles + tile];
#pragma unroll
  for (uint32_t j = 0; j < kIter; ++j) {
    const uint32_t i = base + j * 64u + lane;
    uint64_t todo = __ballot(i < a.n);
    while (todo) {
      const uint32_t k = __builtin_amdgcn_readfirstlane(
          __builtin_amdgcn_readlane(key[j], static_cast<int>(__builtin_ctzll(todo))));
      const bool mine = key[j] == k;
      const uint64_t m = __ballot(mine);
      todo &= ~m;
      if (SCATTER) {
        const uint32_t at = __builtin_amdgcn_readlane(cnt, static_cast<int>(k));
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
            static_cast<uint32_t>(m >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
        if (mine) a.idx[at + rank] = i;
      }
      if (lane == k) cnt += static_cast<uint32_t>(__popcll(m));
    }
  }
  if (!SCATTER && lane < a.groups) a.counts[lane * a.tiles + tile] = cnt;
}

// Exclusive scan of counts[groups * tiles] in place (one workgroup); the arm
// offsets are the scanned values at each arm's first tile.
__global__ __launch_bounds__(kScanBlock) void group_by_scan(GroupByArgs a) {
  __shared__ uint32_t wsum[kScanBlock / 64];
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
  const uint32_t total = a.groups * a.tiles;
  const uint32_t per = (total + kScanBlock - 1) / kScanBlock;
  const uint32_t lo = t * per < total ? t * per : total;
  const uint32_t hi = lo + per < total ? lo + per : total;
  uint32_t s = 0;
  for (uint32_t e = lo; e < hi; ++e) s += a.counts[e];
  // inclusive wave scan, then across waves
  uint32_t x = s;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t v = 0; v < w; ++v) before += wsum[v];
  uint32_t run = before + x - s;  // exclusive prefix of this thread's range
  for (uint32_t e = lo; e < hi; ++e) {
    const uint32_t c = a.counts[e];
    a.counts[e] = run;
    run += c;
  }
  __syncthreads();
  if (t < a.groups) a.group_off[t] = a.counts[t * a.tiles];
  if (t == 0) a.group_off[a.groups] = a.n;
}

}  // namespace

uint32_t group_by_tiles(uint32_t n) { return (n + kTile - 1) / kTile; }

hipError_t launch_group_by(const GroupByArgs &a, hipStream_t s) {
  const dim3 grid((a.tiles + kBlock / 64 - 1) / (kBlock / 64));
  hipLaunchKernelGGL(group_by_pass<false>, grid, dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(group_by_scan, dim3(1), dim3(kScanBlock), 0, s, a);
  hipLaunchKernelGGL(group_by_pass<true>, grid, dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace cgpu
