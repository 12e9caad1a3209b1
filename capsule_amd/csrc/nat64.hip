// nat64.hip — examples/nat64 IPv6 -> IPv4 rewrite ("6to4") on gfx950.
//
// Reference: examples/nat64/main.rs:121-150 (nat_6to4), :41-53
// (assigned_port), :79-83 (map6to4), :35 (V4_ADDR); Packet::remove
// (core/src/packets/mod.rs:242) -> Mbuf::shrink (mbuf.rs:256-275);
// Ethernet::push::<Ipv4> -> Ipv4::try_push (ip/v4.rs:455-469, default header
// :594-609) -> Mbuf::extend (mbuf.rs:225-245); setters (ip/v4.rs:189-203,
// 293-357); Tcp::reconcile_all -> Tcp::compute_checksum (tcp.rs:462-477) then
// Ipv4::reconcile (ip/v4.rs:486-489).
//
// The reference assigns gateway ports from a global AtomicU16 (first 1025)
// in first-seen order of (v6 src, tcp src port).  A batch reproduces that
// order exactly:
//   K1 probe   : one lane per frame.  Classify (Act / Drop / Abort), look the
//                key up in an open-addressing table (plain loads for keys
//                committed by earlier batches; atomicCAS claims an empty slot,
//                atomicMin records the first packet index of a new key), and
//                write the frame's new IPv4 header (it does not depend on the
//                port) to a 24-byte record.
//   K2 count   : per-workgroup count of "first packet of a new key".
//   K3 scan    : exclusive scan of the counts (one workgroup) + NEXT_PORT.
//   K4 assign  : ballot/popcount prefix -> ordinal -> port = base + ordinal.
//   K5 rewrite : four lanes per frame, four 16-B output chunks per lane,
//                loaded from the input shifted by 20 bytes (16 loads of a
//                256-B frame in flight per group), TCP span summed with
//                v_sad_u16 and reduced across the group; the lane holding
//                the TCP checksum field stores it last; keys are committed.
// Kernel boundaries are the only cross-workgroup hand-offs besides the
// device-scope atomics on the slots' ref / min words.
#include "capsule_gpu.h"
#include "device_common.hpp"
#include "kernels.hpp"

namespace cgpu {

namespace {

constexpr uint32_t kBlock = 256;
#ifndef CGPU_NAT64_GROUP
#define CGPU_NAT64_GROUP 4
#endif
#ifndef CGPU_NAT64_CHUNKS
#define CGPU_NAT64_CHUNKS 4
#endif
constexpr uint32_t kGroup = CGPU_NAT64_GROUP;    // lanes per frame in K5
constexpr uint32_t kChunks = CGPU_NAT64_CHUNKS;  // 16-B output chunks per lane per pass (>= 4)
constexpr uint32_t kNoSlot = 0xffffffffu;
constexpr uint32_t kFirstBit = 0x80000000u;  // pkt_slot: first packet of a new key
constexpr uint32_t kLocalBit = 0x40000000u;  // pkt_slot: key first seen in this batch
constexpr uint32_t kSlotMask = 0x3fffffffu;
constexpr uint32_t kV4Addr = 0x017100cbu;    // 203.0.113.1 as LE dword of wire bytes
constexpr uint32_t kDataRoom = 2048u;        // RTE_MBUF_DEFAULT_DATAROOM
constexpr uint32_t kNoRead = 0xffffff00u;    // > any arena length the ABI accepts

__device__ __forceinline__ uint32_t sel3(uint32_t k, uint32_t a, uint32_t b, uint32_t c) {
  return k == 0u ? a : (k == 1u ? b : c);
}

__device__ __forceinline__ uint32_t sad16(uint32_t x, uint32_t acc) {
  return __builtin_amdgcn_sad_u16(x, 0u, acc);
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int b) {
  return (x << b) | (x >> (32 - b));
}

__device__ __forceinline__ uint32_t key_hash(const uint32_t (&key)[5]) {
  uint32_t h = 0x9e3779b9u;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    h ^= key[j] * 0xcc9e2d51u;
    h = rotl32(h, 13) * 5u + 0xe6546b64u;
  }
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

// Byte mask of dword [lo, lo+4) restricted to [s, e).
__device__ __forceinline__ uint32_t range_mask(uint32_t lo, uint32_t s, uint32_t e) {
  uint32_t m = 0xffffffffu;
  if (s > lo) m = s >= lo + 4u ? 0u : (0xffffffffu << (8u * (s - lo)));
  if (e < lo + 4u) m &= e <= lo ? 0u : (0xffffffffu >> (8u * (lo + 4u - e)));
  return m;
}

// Classification of one input frame by the reference nat_6to4 control flow.
struct V6 {
  uint32_t k, eth_len;
  uint32_t disp, st;
  uint32_t L[11];  // L3-relative dwords: v6 header 0..9, TCP source port in L[10] lo
};

// Frame-relative dwords 0..19 (80 B) -> V6.  Fast path: dword-aligned frames
// well inside the arena (wave-uniform), otherwise the tail-safe loader.
__device__ __forceinline__ void classify(rsrc_t rs, uint32_t arena_len, uint32_t off,
                                         uint32_t len, V6 &v) {
  constexpr int NW = 20;
  uint32_t P[NW];
  const bool slow = (off & 3u) != 0u || (uint64_t)off + 80u > (uint64_t)arena_len;
  if (__ballot(slow)) {
    const uint32_t sh = off & 3u, base = off - sh;
    const uint32_t need = sh + (len < 80u ? len : 80u);
    uint32_t D[NW + 1];
#pragma unroll
    for (int j = 0; j < NW + 1; ++j)
      D[j] = (uint32_t)(4 * j) < need ? load4_tail(rs, base + 4u * j, arena_len) : 0u;
#pragma unroll
    for (int j = 0; j < NW; ++j) P[j] = __builtin_amdgcn_alignbyte(D[j + 1], D[j], sh);
  } else {
#pragma unroll
    for (int c = 0; c < NW / 4; ++c) {
      const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off + 16u * c), 0, 0);
      P[4 * c] = q[0];
      P[4 * c + 1] = q[1];
      P[4 * c + 2] = q[2];
      P[4 * c + 3] = q[3];
    }
  }
  const uint32_t marker = be16_lo(P[3]);
  v.k = marker == 0x8100u ? 1u : (marker == 0x88a8u ? 2u : 0u);
  v.eth_len = 14u + 4u * v.k;
  const uint32_t et = be16_lo(sel3(v.k, P[3], P[4], P[5]));
  uint32_t A[13];
#pragma unroll
  for (int j = 0; j < 13; ++j) A[j] = __builtin_amdgcn_alignbyte(P[4 + j], P[3 + j], 2);
#pragma unroll
  for (int j = 0; j < 11; ++j) v.L[j] = sel3(v.k, A[j], A[j + 1], A[j + 2]);
  v.disp = CGPU_ABORT;
  // packet.parse::<Ethernet>()? (ethernet.rs:279-300)
  if (len == 0u) { v.st = CGPU_PKT_ETH_BAD_OFFSET; return; }
  if (len < v.eth_len) { v.st = CGPU_PKT_ETH_OUT_OF_BUFFER; return; }
  // ethernet.parse::<Ipv6>()? (ip/v6/mod.rs:274-289)
  if (et != 0x86ddu) { v.st = CGPU_PKT_NOT_IPV6; return; }
  if (v.eth_len >= len) { v.st = CGPU_PKT_L3_BAD_OFFSET; return; }
  if (v.eth_len + 40u > len) { v.st = CGPU_PKT_L3_OUT_OF_BUFFER; return; }
  // if v6.next_header() == Tcp (main.rs:124) else Either::Drop
  if (((v.L[1] >> 16) & 0xffu) != 6u) { v.st = CGPU_PKT_OK; v.disp = CGPU_DROP; return; }
  // v6.remove()? : shrink(eth_len, 40) cannot fail after a successful parse.
  // push::<Ipv4>()? : extend(eth_len, 20) needs 20 < tailroom (mbuf.rs:228).
  const uint32_t shrunk = len - 40u;
  if (!(20u < (shrunk < kDataRoom ? kDataRoom - shrunk : 0u))) {
    v.st = CGPU_PKT_NOT_RESIZED;
    return;
  }
  // v4.parse::<Tcp4>()? on the rewritten frame (tcp.rs:558-573)
  const uint32_t new_len = len - 20u, tcp_off = v.eth_len + 20u;
  if (tcp_off >= new_len) { v.st = CGPU_PKT_L4_BAD_OFFSET; return; }
  if (tcp_off + 20u > new_len) { v.st = CGPU_PKT_L4_OUT_OF_BUFFER; return; }
  v.st = CGPU_PKT_OK;
  v.disp = CGPU_ACT;
}

// key = (v6 src, tcp src port) = assigned_port(src, port) (main.rs:129,142-143)
__device__ __forceinline__ void make_key(const V6 &v, uint32_t (&key)[5]) {
  key[0] = v.L[2];
  key[1] = v.L[3];
  key[2] = v.L[4];
  key[3] = v.L[5];
  key[4] = be16_lo(v.L[10]);
}

__device__ __forceinline__ bool key_eq(const uint32_t (&a)[5], const uint32_t (&b)[5]) {
  return a[0] == b[0] && a[1] == b[1] && a[2] == b[2] && a[3] == b[3] && a[4] == b[4];
}

// ---- K1: classify + probe + header record -----------------------------------
__global__ __launch_bounds__(kBlock) void nat64_probe(Nat64Args a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const bool valid = i < a.n;
  const rsrc_t rs = make_rsrc(a.arena, a.arena_len);
  const uint32_t off = valid ? a.off[i] : 0u, len = valid ? (uint32_t)a.len[i] : 0u;
  V6 v;
  classify(rs, a.arena_len, off, len, v);
  if (!valid) return;
  uint32_t slot = kNoSlot, port = 0xffffffffu;  // port known now for committed keys
  if (v.disp == CGPU_ACT) {
    uint32_t key[5];
    make_key(v, key);
    uint32_t h = key_hash(key) & a.pm.cap_mask;
    for (uint32_t probe = 0; probe <= a.pm.cap_mask; ++probe) {
      // Keys committed by earlier batches are matched from one 32-B slot
      // load; an empty slot is claimed with a CAS.  refs only ever go
      // 0 -> (i + 1) -> kPersist, so a stale 0 just leads to the CAS.
      const u32x4 *sp = reinterpret_cast<const u32x4 *>(&a.pm.slots[h]);
      const u32x4 s0 = sp[0], s1 = sp[1];
      uint32_t ref = s0[0];
      bool claimed = false;
      if (ref == 0u) {
        ref = atomicCAS(&a.pm.slots[h].w[0], 0u, i + 1u);
        claimed = ref == 0u;
      }
      bool match;
      if (claimed) {
        match = true;  // this packet represents the key: publish the key words
#pragma unroll
        for (int j = 0; j < 4; ++j) a.pm.slots[h].w[1 + j] = key[j];
        a.pm.slots[h].w[5] = key[4];
      } else if (ref & kPersist) {
        const uint32_t other[5] = {s0[1], s0[2], s0[3], s1[0], s1[1]};
        match = key_eq(key, other);
        if (match) port = s1[2];
      } else {
        // a key first seen in this batch: compare with the representative
        // frame's own bytes (immutable input), never with the table words
        // its claimer may still be writing.
        const uint32_t rep = ref - 1u;
        V6 rv;
        classify(rs, a.arena_len, a.off[rep], a.len[rep], rv);
        uint32_t other[5];
        make_key(rv, other);
        match = key_eq(key, other);
      }
      if (match) {
        if (!(ref & kPersist)) {
          atomicMin(&a.pm.slots[h].w[7], i);
          slot = h | kLocalBit;
        } else {
          slot = h;
        }
        break;
      }
      h = (h + 1u) & a.pm.cap_mask;
    }
    if (slot == kNoSlot) {
      v.disp = CGPU_ABORT;
      v.st = CGPU_PKT_TABLE_FULL;
    } else {
      // The pushed IPv4 header (v4.rs:594-609) with the setters of main.rs:
      // 133-138 and Ipv4::reconcile (v4.rs:486-489) already applied.
      const uint32_t w = be32(v.L[0]);
      const uint32_t dscp = (w & 0x0fc00000u) >> 22, ecn = (w & 0x00300000u) >> 20;
      const uint32_t ttl = ((v.L[1] >> 24) - 1u) & 0xffu;  // hop_limit - 1 (u8, wrapping)
      const uint32_t dscp_ecn = (((dscp << 2) & 0xfcu) | (ecn & 0x3u)) & 0xffu;
      const uint32_t new_len = len - 20u;
      uint32_t H[5];
      H[0] = 0x45u | (dscp_ecn << 8) | (swap16((new_len - v.eth_len) & 0xffffu) << 16);
      H[1] = 0u;               // identification 0, flags/fragment 0
      H[2] = ttl | (6u << 8);  // protocol = next_header (6)
      H[3] = kV4Addr;          // V4_ADDR (main.rs:35)
      H[4] = v.L[9];           // map6to4(dst): low 32 bits (main.rs:79-83)
      const uint32_t ip_c =
          (~swap16(fold64((uint64_t)H[0] + H[1] + H[2] + H[3] + H[4]))) & 0xffffu;
      H[2] |= swap16(ip_c) << 16;
      const u32x4 hv = {H[0], H[1], H[2], H[3]};
      a.rec_h[i] = hv;
      a.rec_b[i] = make_uint2(H[4], v.k | (port << 16) | (port == 0xffffffffu ? 0u : 4u));
    }
  }
  a.pkt_slot[i] = slot;
  a.disposition[i] = (uint8_t)v.disp;
  a.status[i] = (uint8_t)v.st;
}

// Only packets whose key was first seen in this batch touch the table here.
__device__ __forceinline__ bool is_first_new(const Nat64Args &a, uint32_t i) {
  const uint32_t ps = a.pkt_slot[i];
  if (ps == kNoSlot || !(ps & kLocalBit)) return false;
  return a.pm.slots[ps & kSlotMask].w[7] == i;
}

// ---- K2: per-block count of first packets of new keys ----------------------
__global__ __launch_bounds__(kBlock) void nat64_count(Nat64Args a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const bool f = i < a.n && is_first_new(a, i);
  const int c = __syncthreads_count(f);
  if (threadIdx.x == 0) a.block_sums[blockIdx.x] = (uint32_t)c;
}

// ---- K3: exclusive scan of block counts + NEXT_PORT update (1 workgroup) ---
constexpr uint32_t kScanBlock = 1024;
__global__ __launch_bounds__(kScanBlock) void nat64_scan(Nat64Args a, uint32_t nb) {
  __shared__ uint32_t wsum[kScanBlock / 64];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  for (uint32_t base = 0; base < nb; base += kScanBlock) {
    const uint32_t idx = base + threadIdx.x;
    const uint32_t v = idx < nb ? a.block_sums[idx] : 0u;
    uint32_t x = v;  // inclusive wave scan
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63u) wsum[wave] = x;
    __syncthreads();
    uint32_t wpre = 0;
    for (uint32_t w = 0; w < wave; ++w) wpre += wsum[w];
    const uint32_t c0 = carry;
    if (idx < nb) a.block_sums[idx] = c0 + wpre + x - v;
    __syncthreads();
    if (threadIdx.x == kScanBlock - 1) carry = c0 + wpre + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const uint32_t total = carry;
    const uint32_t base_port = a.pm.state[0];
    a.pm.state[2] = base_port;
    a.pm.state[3] = total;
    a.pm.state[0] = (base_port + total) & 0xffffu;  // AtomicU16 wrap
    a.pm.state[1] += total;
  }
}

// ---- K4: ordinal -> port for the first packet of each new key --------------
__global__ __launch_bounds__(kBlock) void nat64_assign(Nat64Args a) {
  __shared__ uint32_t wcount[kBlock / 64];
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const bool f = i < a.n && is_first_new(a, i);
  const uint64_t mask = __ballot(f);
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t below = (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
  if (lane == 0) wcount[wave] = (uint32_t)__popcll(mask);
  __syncthreads();
  uint32_t pre = a.block_sums[blockIdx.x];
  for (uint32_t w = 0; w < wave; ++w) pre += wcount[w];
  if (f) {
    const uint32_t ps = a.pkt_slot[i], slot = ps & kSlotMask;
    const uint32_t ordinal = pre + below;
    const uint32_t port = (a.pm.state[2] + ordinal) & 0xffffu;
    a.pm.slots[slot].w[6] = port;
    a.pkt_slot[i] = ps | kFirstBit;
    // ADDR_MAP.insert_new(port, key) (main.rs:50): the first mapping of a
    // port wins, also after NEXT_PORT wraps; ordinals are global
    const uint64_t tag = ((uint64_t)(a.pm.state[1] - a.pm.state[3] + ordinal) << 32) | slot;
    atomicMin((unsigned long long *)&a.pm.rev[port], (unsigned long long)tag);
  }
}

// 16 input bytes at any frame-relative byte position (tail-safe).
__device__ __forceinline__ u32x4 load_in(rsrc_t rs, uint32_t arena_len, uint32_t abs_off,
                                         bool aligned_wave) {
  if (aligned_wave) return load16(rs, abs_off, arena_len);
  const uint32_t sh = abs_off & 3u, base = abs_off - sh;
  uint32_t D[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) D[j] = load4_tail(rs, base + 4u * j, arena_len);
  u32x4 v;
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = __builtin_amdgcn_alignbyte(D[j + 1], D[j], sh);
  return v;
}

// Store output bytes [16c, 16c+16) of a frame of `len` bytes at out_base;
// bytes at or past `len` are never written (packed slots do not clobber).
__device__ __forceinline__ void store_out(rsrc_t ors, uint8_t *out_arena, uint32_t out_base,
                                          uint32_t c, u32x4 v, uint32_t len, bool aligned) {
  const uint32_t o = out_base + 16u * c;
  if (aligned && 16u * c + 16u <= len) {
    __builtin_amdgcn_raw_buffer_store_b128(v, ors, (int)o, 0, 0);
    return;
  }
#pragma unroll
  for (uint32_t t = 0; t < 4u; ++t) {
    const uint32_t b = 16u * c + 4u * t;
    if (aligned && b + 4u <= len) {
      __builtin_amdgcn_raw_buffer_store_b32(v[t], ors, (int)(o + 4u * t), 0, 0);
    } else {
      for (uint32_t q = 0; q < 4u; ++q)
        if (b + q < len) out_arena[o + 4u * t + q] = (uint8_t)(v[t] >> (8u * q));
    }
  }
}

// Output dwords 0..15 (chunks 0..3) of the rewritten frame for VLAN depth K
// (compile-time, so every select folds away), from the input dwords A (same
// position) and o (input shifted by 20 bytes).  Returns the u16-word sum of
// the TCP span bytes [34 + 4K, new_len) inside these chunks.
template <int K>
__device__ __forceinline__ uint32_t build_header(u32x4 (&o)[kChunks], const u32x4 (&A)[4],
                                                 const uint32_t (&H)[5], uint32_t port_be,
                                                 uint32_t new_len) {
  uint32_t acc = 0;
#pragma unroll
  for (int n = 0; n < 4; ++n) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int r = 4 * n + t - K;
      uint32_t d = o[n][t];
      if (r < 3) d = A[n][t];                                                 // Ethernet
      else if (r == 3) d = __builtin_amdgcn_alignbyte(H[0], 0x00080000u, 2);  // ether_type
      else if (r == 4) d = __builtin_amdgcn_alignbyte(H[1], H[0], 2);
      else if (r == 5) d = __builtin_amdgcn_alignbyte(H[2], H[1], 2);
      else if (r == 6) d = __builtin_amdgcn_alignbyte(H[3], H[2], 2);
      else if (r == 7) d = __builtin_amdgcn_alignbyte(H[4], H[3], 2);
      else if (r == 8) d = (H[4] >> 16) | (port_be << 16);  // dst tail | TCP src port
      else if (r == 12) d &= 0x0000ffffu;                     // TCP checksum zeroed
      o[n][t] = d;
      if (r >= 8) {  // TCP span: from the high half of dword 8 + K
        uint32_t m = r == 8 ? 0xffff0000u : 0xffffffffu;
        m &= range_mask(16u * n + 4u * t, 0u, new_len);
        acc = sad16(d & m, acc);
      }
    }
  }
  return acc;
}

// One pass of K5 for one lane: output chunks c0 .. c0 + kChunks - 1.
template <bool FAST>
__device__ __forceinline__ void rewrite_pass(const Nat64Args &a, rsrc_t rs, rsrc_t ors, uint32_t q,
                                             uint32_t g, uint32_t in_off, uint32_t o_off,
                                             uint32_t new_len, uint32_t k, const uint32_t (&H)[5],
                                             uint32_t port_be, uint32_t &acc, u32x4 &held,
                                             bool in_al_wave) {
  const uint32_t c0 = (q * kGroup + g) * kChunks;
  u32x4 o[kChunks];
  // output byte b >= 34+4k is input byte b + 20 (v6 header 40 B -> v4 20 B)
#pragma unroll
  for (uint32_t n = 0; n < kChunks; ++n) {
    const uint32_t c = c0 + n;
    const bool need = 16u * c < new_len;
    if (FAST) {
      o[n] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(need ? in_off + 16u * c + 20u : kNoRead), 0, 0);
    } else {
      o[n] = u32x4{0u, 0u, 0u, 0u};
      if (need) o[n] = load_in(rs, a.arena_len, in_off + 16u * c + 20u, in_al_wave);
    }
  }
  if (c0 == 0u) {  // header region, output bytes 0..63 (lane 0 of pass 0)
    u32x4 A[4];
#pragma unroll
    for (uint32_t n = 0; n < 4u; ++n)
      A[n] = FAST ? __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(in_off + 16u * n), 0, 0)
                  : load_in(rs, a.arena_len, in_off + 16u * n, in_al_wave);
    // one compile-time variant per VLAN depth present in the wave
    if (__ballot(k == 0u) && k == 0u) acc = build_header<0>(o, A, H, port_be, new_len);
    if (__ballot(k == 1u) && k == 1u) acc = build_header<1>(o, A, H, port_be, new_len);
    if (__ballot(k == 2u) && k == 2u) acc = build_header<2>(o, A, H, port_be, new_len);
    held = o[3];
  } else {
    // whole chunks (unneeded ones are zero), then the bytes past new_len of
    // the last chunk subtracted
#pragma unroll
    for (uint32_t n = 0; n < kChunks; ++n) acc = sad16(o[n][3], sad16(o[n][2], sad16(o[n][1], sad16(o[n][0], acc))));
    const uint32_t pc = (new_len - 1u) >> 4;  // chunk holding the last byte
    if ((new_len & 15u) != 0u && pc >= c0 && pc < c0 + kChunks) {
      u32x4 last = o[0];
#pragma unroll
      for (uint32_t n = 1; n < kChunks; ++n)
        if (pc == c0 + n) last = o[n];
#pragma unroll
      for (uint32_t t = 0; t < 4u; ++t) {
        const uint32_t x = last[t] & ~range_mask(16u * pc + 4u * t, 0u, new_len);
        acc -= (x & 0xffffu) + (x >> 16);
      }
    }
  }
  if (FAST) {
    // full chunks: one dwordx4 store each; the partial last chunk: dword and
    // byte stores (all predicated by offset, never past new_len)
#pragma unroll
    for (uint32_t n = 0; n < kChunks; ++n) {
      const uint32_t c = c0 + n;
      const bool full = 16u * c + 16u <= new_len && c != 3u;
      __builtin_amdgcn_raw_buffer_store_b128(o[n], ors, (int)(full ? o_off + 16u * c : kNoRead), 0, 0);
    }
    const uint32_t pc = (new_len - 1u) >> 4;
    if ((new_len & 15u) != 0u && pc >= c0 && pc < c0 + kChunks && pc != 3u) {
      u32x4 last = o[0];
#pragma unroll
      for (uint32_t n = 1; n < kChunks; ++n)
        if (pc == c0 + n) last = o[n];
#pragma unroll
      for (uint32_t t = 0; t < 4u; ++t) {
        const uint32_t b = 16u * pc + 4u * t;
        __builtin_amdgcn_raw_buffer_store_b32(last[t], ors, (int)(b + 4u <= new_len ? o_off + b : kNoRead), 0, 0);
#pragma unroll
        for (uint32_t x = 0; x < 3u; ++x)
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(last[t] >> (8u * x)), ors,
                                               (int)(b + 4u > new_len && b + x < new_len ? o_off + b + x : kNoRead), 0, 0);
      }
    }
  } else {
#pragma unroll
    for (uint32_t n = 0; n < kChunks; ++n) {
      const uint32_t c = c0 + n;
      if (16u * c < new_len && c != 3u)
        store_out(ors, a.out_arena, o_off, c, o[n], new_len, (o_off & 3u) == 0u);
    }
  }
}

// ---- K5: rewrite (kGroup lanes per frame, kChunks x 16 B per lane) + commit --
// Lane g of a frame's group builds output chunks c = (q*kGroup + g)*kChunks + n
// (16 B each) from coalesced loads of the input shifted by 20 bytes; lane 0
// of pass 0 owns chunks 0..3, i.e. the Ethernet/IPv4 header and the TCP
// header up to its checksum field (output bytes 50+4k, chunk 3), and stores
// chunk 3 after the group has reduced the TCP span sum.
__global__ __launch_bounds__(kBlock) void nat64_rewrite(Nat64Args a) {
  const uint32_t g = threadIdx.x & (kGroup - 1u);
  const uint32_t p = blockIdx.x * (kBlock / kGroup) + threadIdx.x / kGroup;
  const bool valid = p < a.n;
  const uint32_t ps = valid ? a.pkt_slot[p] : kNoSlot;
  const uint32_t in_off = valid ? a.off[p] : 0u;
  const uint32_t o_off = valid ? a.out_off[p] : 0u;
  // the new length comes from the descriptor, so the frame's loads depend on
  // one round trip only (the record and the port arrive alongside them)
  const uint32_t new_len = valid ? (uint32_t)a.len[p] - 20u : 0u;
  const bool in_al_wave = !__ballot((in_off & 3u) != 0u);
  if (ps == kNoSlot) {  // uniform within the group
    if (valid && g == 0) a.out_len[p] = 0;
    return;
  }
  const u32x4 hv = a.rec_h[p];
  const uint2 bv = a.rec_b[p];
  const uint32_t H[5] = {hv[0], hv[1], hv[2], hv[3], bv.x};
  const uint32_t k = bv.y & 3u;
  // port: from the record for committed keys, else assigned by K4
  const uint32_t port_be =
      swap16((bv.y & 4u) ? (bv.y >> 16) : a.pm.slots[ps & kSlotMask].w[6]);
  const uint32_t span_lo = 34u + 4u * k;  // TCP header in the output frame
  const rsrc_t rs = make_rsrc(a.arena, a.arena_len);
  const rsrc_t ors = make_rsrc(a.out_arena, a.out_arena_len);
  uint32_t acc = 0;
  u32x4 held = {0u, 0u, 0u, 0u};
  // Fast path (wave-uniform): every frame of the wave is dword-aligned on both
  // sides and well inside both arenas.  Loads and full-chunk stores are then
  // branch-free: a chunk a lane does not need gets an offset past num_records,
  // which the buffer range check turns into a zero load / dropped store.
  const bool fast = !__ballot(!((in_off & 3u) == 0u && (o_off & 3u) == 0u &&
                                (uint64_t)in_off + new_len + 64u <= (uint64_t)a.arena_len &&
                                (uint64_t)o_off + new_len + 16u <= (uint64_t)a.out_arena_len));
  if (fast) {
    for (uint32_t q = 0; 16u * kChunks * kGroup * q < new_len; ++q)
      rewrite_pass<true>(a, rs, ors, q, g, in_off, o_off, new_len, k, H, port_be, acc, held, true);
  } else {
    for (uint32_t q = 0; 16u * kChunks * kGroup * q < new_len; ++q)
      rewrite_pass<false>(a, rs, ors, q, g, in_off, o_off, new_len, k, H, port_be, acc, held,
                          in_al_wave);
  }
  // group reduction of the span sum
#pragma unroll
  for (uint32_t d = kGroup / 2; d > 0; d >>= 1) acc += __shfl_xor(acc, d, kGroup);
  if (g == 0u) {
    // TCP checksum with the v4 pseudo-header (checksum.rs:93-103): src
    // 203.0.113.1, dst, protocol 6, span length
    const uint32_t span = (new_len - span_lo) & 0xffffu;
    const uint32_t dst = be32(H[4]);
    const uint32_t ph = fold32(0xcb00u + 0x7101u + (dst >> 16) + (dst & 0xffffu) + 6u + span);
    const uint32_t tcp_c = (~fold32(ph + swap16(fold32(acc)))) & 0xffffu;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if ((uint32_t)t == k) held[t] |= swap16(tcp_c) << 16;
    store_out(ors, a.out_arena, o_off, 3u, held, new_len, (o_off & 3u) == 0u);
    a.out_len[p] = (uint16_t)new_len;
    if (ps & kFirstBit) {  // commit the new key (PORT_MAP.insert_new, main.rs:49)
      const uint32_t slot = ps & kSlotMask;
      a.pm.slots[slot].w[7] = 0xffffffffu;
      a.pm.slots[slot].w[0] = kPersist;
    }
  }
}

// ============================ 4to6 direction =================================
// examples/nat64/main.rs:86-118 (nat_4to6), :56-58 (assigned_addr), :62-74
// (map4to6); Ipv4::remove -> shrink 20, Ethernet::push::<Ipv6> (ip/v6/mod.rs:
// 302-316, default header :453-464) -> extend 40; Tcp::reconcile_all with the
// v6 pseudo-header, then Ipv6::reconcile (payload_length, :331-334).
//   K1' probe  : one lane per frame: classify, look the TCP destination port up
//                in the reverse map ADDR_MAP (rev[port] -> slot -> v6 key),
//                write the frame's complete IPv6 header + original port.
//   K2' rewrite: four lanes per frame as in K5, output = input shifted by +20
//                bytes behind the new 40-byte header; the TCP checksum field
//                (output bytes 70+4k) lives in chunk 4, held by lane 1.

// ---- K1': classify + ADDR_MAP lookup + IPv6 header record -------------------
__global__ __launch_bounds__(kBlock) void nat64_4to6_probe(Nat64Args a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const bool valid = i < a.n;
  const rsrc_t rs = make_rsrc(a.arena, a.arena_len);
  const uint32_t off = valid ? a.off[i] : 0u, len = valid ? (uint32_t)a.len[i] : 0u;
  // frame-relative dwords 0..11 (48 B): Ethernet + IPv4 + TCP ports, QinQ included
  constexpr int NW = 12;
  uint32_t P[NW];
  const bool slow = (off & 3u) != 0u || (uint64_t)off + 48u > (uint64_t)a.arena_len;
  if (__ballot(slow)) {
    const uint32_t sh = off & 3u, base = off - sh;
    const uint32_t need = sh + (len < 48u ? len : 48u);
    uint32_t D[NW + 1];
#pragma unroll
    for (int j = 0; j < NW + 1; ++j)
      D[j] = (uint32_t)(4 * j) < need ? load4_tail(rs, base + 4u * j, a.arena_len) : 0u;
#pragma unroll
    for (int j = 0; j < NW; ++j) P[j] = __builtin_amdgcn_alignbyte(D[j + 1], D[j], sh);
  } else {
#pragma unroll
    for (int c = 0; c < NW / 4; ++c) {
      const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off + 16u * c), 0, 0);
      P[4 * c] = q[0];
      P[4 * c + 1] = q[1];
      P[4 * c + 2] = q[2];
      P[4 * c + 3] = q[3];
    }
  }
  if (!valid) return;
  const uint32_t marker = be16_lo(P[3]);
  const uint32_t k = marker == 0x8100u ? 1u : (marker == 0x88a8u ? 2u : 0u);
  const uint32_t eth_len = 14u + 4u * k;
  const uint32_t et = be16_lo(sel3(k, P[3], P[4], P[5]));
  uint32_t A[8];  // L3-relative dwords 0..6 (IPv4 header, TCP ports)
#pragma unroll
  for (int j = 0; j < 8; ++j) A[j] = __builtin_amdgcn_alignbyte(P[4 + j], P[3 + j], 2);
  uint32_t L[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) L[j] = sel3(k, A[j], j + 1 < 8 ? A[j + 1] : 0u, j + 2 < 8 ? A[j + 2] : 0u);
  uint32_t disp = CGPU_ABORT, st;
  uint32_t slot = kNoSlot;
  if (len == 0u) st = CGPU_PKT_ETH_BAD_OFFSET;                 // parse::<Ethernet>()?
  else if (len < eth_len) st = CGPU_PKT_ETH_OUT_OF_BUFFER;
  else if (et != 0x0800u) st = CGPU_PKT_NOT_IPV4;              // parse::<Ipv4>()?
  else if (eth_len >= len) st = CGPU_PKT_L3_BAD_OFFSET;
  else if (eth_len + 20u > len) st = CGPU_PKT_L3_OUT_OF_BUFFER;
  else {
    st = CGPU_PKT_OK;
    disp = CGPU_DROP;
    const uint32_t flags_frag = be16_hi(L[1]);  // flags/fragment offset: L3 bytes 6-7
    const uint32_t proto = (L[2] >> 8) & 0xffu;
    if (proto == 6u && (flags_frag & 0x1fffu) == 0u && !(flags_frag & 0x2000u)) {
      const uint32_t tcp_off = eth_len + 20u;
      if (tcp_off >= len) { st = CGPU_PKT_L4_BAD_OFFSET; disp = CGPU_ABORT; }   // peek::<Tcp4>()?
      else if (tcp_off + 20u > len) { st = CGPU_PKT_L4_OUT_OF_BUFFER; disp = CGPU_ABORT; }
      else {
        const uint32_t gw_port = be16_hi(L[5]);  // TCP destination port (L3 bytes 22-23)
        const uint64_t r = a.pm.rev[gw_port];
        if (r != ~0ull) {  // assigned_addr(port) = Some((dst, port))
          if (len >= kDataRoom - 20u) {  // push::<Ipv6>(): extend 40 needs 40 < tailroom
            st = CGPU_PKT_NOT_RESIZED;
            disp = CGPU_ABORT;
          } else {
            slot = (uint32_t)r;
            disp = CGPU_ACT;
            const u32x4 *sp = reinterpret_cast<const u32x4 *>(&a.pm.slots[slot]);
            const u32x4 s0 = sp[0], s1 = sp[1];
            const uint32_t de = (L[0] >> 8) & 0xffu;             // dscp_ecn (v4.rs:186-203)
            const uint32_t dscp = de >> 2, ecn = de & 3u;
            const uint32_t hop = ((L[2] & 0xffu) - 1u) & 0xffu;   // ttl - 1 (u8, wrapping)
            const uint32_t new_len = len + 20u;
            // Ipv6Header::default + set_dscp/ecn/next_header/hop_limit/src/dst
            const uint32_t w = (6u << 28) | ((dscp << 22) & 0x0fc00000u) | ((ecn << 20) & 0x00300000u);
            uint32_t V[10];
            V[0] = be32(w);
            V[1] = swap16((new_len - eth_len - 40u) & 0xffffu) | (6u << 16) | (hop << 24);
            V[2] = 0x9bff6400u;  // 64:ff9b::/96 (map4to6, main.rs:62-74)
            V[3] = 0u;
            V[4] = 0u;
            V[5] = L[3];         // v4 source address
            V[6] = s0[1];        // ADDR_MAP key: the original v6 source
            V[7] = s0[2];
            V[8] = s0[3];
            V[9] = s1[0];
            const uint32_t orig_port = s1[1];
            // v6 pseudo-header addresses as a folded LE residue
            uint32_t ph = 0;
#pragma unroll
            for (int j = 2; j < 10; ++j) ph = __builtin_amdgcn_sad_u16(V[j], 0u, ph);
            u32x4 *rec = a.rec_h + 3u * i;
            rec[0] = u32x4{V[0], V[1], V[2], V[3]};
            rec[1] = u32x4{V[4], V[5], V[6], V[7]};
            rec[2] = u32x4{V[8], V[9], k | (orig_port << 16), fold32(ph)};
          }
        }
      }
    }
  }
  a.pkt_slot[i] = slot;
  a.disposition[i] = (uint8_t)disp;
  a.status[i] = (uint8_t)st;
}

// Output dwords 0..15 (chunks 0..3) for VLAN depth K: Ethernet, ether_type
// 0x86dd, the 40-byte IPv6 header V, then TCP from the input shifted by +20
// (o), with the destination port (dword 14+K) patched.  Returns the u16-word
// sum of the TCP span bytes [54 + 4K, new_len) in these chunks.
template <int K>
__device__ __forceinline__ uint32_t build_header6(u32x4 (&o)[kChunks], const u32x4 (&A)[4],
                                                  const uint32_t (&V)[10], uint32_t port_be,
                                                  uint32_t new_len) {
  uint32_t acc = 0;
#pragma unroll
  for (int n = 0; n < 4; ++n) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int r = 4 * n + t - K;
      uint32_t d = o[n][t];
      if (r < 3) d = A[n][t];
      else if (r == 3) d = __builtin_amdgcn_alignbyte(V[0], 0xdd860000u, 2);  // ether_type 0x86dd
      else if (r >= 4 && r <= 12) d = __builtin_amdgcn_alignbyte(V[r - 3], V[r - 4], 2);
      else if (r == 13) d = (d & 0xffff0000u) | (V[9] >> 16);  // dst tail | TCP src port
      else if (r == 14) d = (d & 0xffff0000u) | port_be;       // TCP dst port | seq
      o[n][t] = d;
      if (r >= 13) {
        uint32_t m = r == 13 ? 0xffff0000u : 0xffffffffu;
        m &= range_mask(16u * n + 4u * t, 0u, new_len);
        acc = sad16(d & m, acc);
      }
    }
  }
  return acc;
}

// ---- K2': rewrite (kGroup lanes per frame, kChunks x 16 B per lane) ---------
__global__ __launch_bounds__(kBlock) void nat64_4to6_rewrite(Nat64Args a) {
  const uint32_t g = threadIdx.x & (kGroup - 1u);
  const uint32_t p = blockIdx.x * (kBlock / kGroup) + threadIdx.x / kGroup;
  const bool valid = p < a.n;
  const uint32_t ps = valid ? a.pkt_slot[p] : kNoSlot;
  const uint32_t in_off = valid ? a.off[p] : 0u;
  const uint32_t o_off = valid ? a.out_off[p] : 0u;
  const uint32_t new_len = valid ? (uint32_t)a.len[p] + 20u : 0u;
  const bool in_al_wave = !__ballot((in_off & 3u) != 0u);
  if (ps == kNoSlot) {  // uniform within the group
    if (valid && g == 0) a.out_len[p] = 0;
    return;
  }
  const u32x4 *rec = a.rec_h + 3u * p;
  const u32x4 r0 = rec[0], r1 = rec[1], r2 = rec[2];
  const uint32_t V[10] = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3], r2[0], r2[1]};
  const uint32_t k = r2[2] & 3u, port_be = swap16(r2[2] >> 16), ph_le = r2[3];
  const uint32_t span_lo = 54u + 4u * k;  // TCP header in the output frame
  const rsrc_t rs = make_rsrc(a.arena, a.arena_len);
  const rsrc_t ors = make_rsrc(a.out_arena, a.out_arena_len);
  const bool out_al = (o_off & 3u) == 0u;
  uint32_t acc = 0;
  u32x4 held = {0u, 0u, 0u, 0u};
  for (uint32_t q = 0; 16u * kChunks * kGroup * q < new_len; ++q) {
    const uint32_t c0 = (q * kGroup + g) * kChunks;
    u32x4 o[kChunks];
#pragma unroll
    for (uint32_t n = 0; n < kChunks; ++n) {  // output byte b >= 54+4k is input byte b - 20
      const uint32_t c = c0 + n;
      o[n] = u32x4{0u, 0u, 0u, 0u};
      if (16u * c < new_len && c >= 2u) o[n] = load_in(rs, a.arena_len, in_off + 16u * c - 20u, in_al_wave);
    }
    if (c0 == 0u) {
      u32x4 A[4];
#pragma unroll
      for (uint32_t n = 0; n < 4u; ++n)
        A[n] = n < 2u ? load_in(rs, a.arena_len, in_off + 16u * n, in_al_wave) : u32x4{0u, 0u, 0u, 0u};
      if (__ballot(k == 0u) && k == 0u) acc = build_header6<0>(o, A, V, port_be, new_len);
      if (__ballot(k == 1u) && k == 1u) acc = build_header6<1>(o, A, V, port_be, new_len);
      if (__ballot(k == 2u) && k == 2u) acc = build_header6<2>(o, A, V, port_be, new_len);
    } else {
      if (c0 == 4u) {
        // chunk 4 = output dwords 16..19: the TCP destination port for k = 2
        // (dword 14 + k) and the checksum field (high half of dword 17 + k)
#pragma unroll
        for (uint32_t t = 0; t < 4u; ++t) {
          const uint32_t j = 16u + t;
          if (j == 14u + k) o[0][t] = (o[0][t] & 0xffff0000u) | port_be;
          if (j == 17u + k) o[0][t] &= 0x0000ffffu;
        }
      }
#pragma unroll
      for (uint32_t n = 0; n < kChunks; ++n)
        if (16u * (c0 + n) < new_len) acc = sad16(o[n][3], sad16(o[n][2], sad16(o[n][1], sad16(o[n][0], acc))));
      const uint32_t pc = (new_len - 1u) >> 4;
      if ((new_len & 15u) != 0u && pc >= c0 && pc < c0 + kChunks) {
        u32x4 last = o[0];
#pragma unroll
        for (uint32_t n = 1; n < kChunks; ++n)
          if (pc == c0 + n) last = o[n];
#pragma unroll
        for (uint32_t t = 0; t < 4u; ++t) {
          const uint32_t x = last[t] & ~range_mask(16u * pc + 4u * t, 0u, new_len);
          acc -= (x & 0xffffu) + (x >> 16);
        }
      }
      if (c0 == 4u) held = o[0];
    }
#pragma unroll
    for (uint32_t n = 0; n < kChunks; ++n) {
      const uint32_t c = c0 + n;
      if (16u * c < new_len && c != 4u) store_out(ors, a.out_arena, o_off, c, o[n], new_len, out_al);
    }
  }
#pragma unroll
  for (uint32_t d = kGroup / 2; d > 0; d >>= 1) acc += __shfl_xor(acc, d, kGroup);
  if (g == 1u) {
    // TCP checksum with the v6 pseudo-header (checksum.rs:123-128)
    const uint32_t span = (new_len - span_lo) & 0xffffu;
    const uint32_t tcp_c = (~fold32(swap16(fold32(acc + ph_le)) + span + 6u)) & 0xffffu;
#pragma unroll
    for (uint32_t t = 0; t < 4u; ++t)
      if (16u + t == 17u + k) held[t] |= swap16(tcp_c) << 16;
    store_out(ors, a.out_arena, o_off, 4u, held, new_len, out_al);
  }
  if (g == 0u) a.out_len[p] = (uint16_t)new_len;
}

__global__ void portmap_init(PortMapDev pm, uint32_t first_port) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= pm.cap_mask) {
#pragma unroll
    for (int j = 0; j < 7; ++j) pm.slots[i].w[j] = 0u;
    pm.slots[i].w[7] = 0xffffffffu;
  }
  if (i < 65536u) pm.rev[i] = ~0ull;
  if (i == 0) {
    pm.state[0] = first_port;
    pm.state[1] = 0u;
    pm.state[2] = 0u;
    pm.state[3] = 0u;
  }
}

}  // namespace

uint32_t nat64_num_blocks(uint32_t n) { return (n + kBlock - 1) / kBlock; }

hipError_t launch_portmap_init(const PortMapDev &pm, uint32_t first_port, hipStream_t s) {
  const uint32_t cap = pm.cap_mask + 1u > 65536u ? pm.cap_mask + 1u : 65536u;
  hipLaunchKernelGGL(portmap_init, dim3((cap + 255) / 256), dim3(256), 0, s, pm, first_port);
  return hipGetLastError();
}

hipError_t launch_nat64_6to4(const Nat64Args &a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  const uint32_t nb = nat64_num_blocks(a.n);
  const uint32_t nb5 = (a.n + kBlock / kGroup - 1) / (kBlock / kGroup);
  hipLaunchKernelGGL(nat64_probe, dim3(nb), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(nat64_count, dim3(nb), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(nat64_scan, dim3(1), dim3(kScanBlock), 0, s, a, nb);
  hipLaunchKernelGGL(nat64_assign, dim3(nb), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(nat64_rewrite, dim3(nb5), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_nat64_4to6(const Nat64Args &a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  const uint32_t nb = nat64_num_blocks(a.n);
  const uint32_t nb5 = (a.n + kBlock / kGroup - 1) / (kBlock / kGroup);
  hipLaunchKernelGGL(nat64_4to6_probe, dim3(nb), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(nat64_4to6_rewrite, dim3(nb5), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace cgpu
