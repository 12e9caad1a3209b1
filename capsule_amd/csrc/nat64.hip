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
// in first-seen order of (v6 src, tcp src port).  The batch reproduces that
// order exactly:
//   K1 probe   : parse, classify (Act / Drop / Abort), insert-or-find the key
//                in an open-addressing table; atomicMin the packet index
//                into the slot so each new key knows its first packet.
//   K2 count   : per-block count of "first packet of a new key".
//   K3 scan    : exclusive scan of the block counts (one workgroup) and the
//                NEXT_PORT update, all on the device.
//   K4 assign  : in-block ballot scan -> ordinal -> port = base + ordinal.
//   K5 rewrite : build the IPv4 frame, TCP + IPv4 checksums, write it, and
//                commit new keys to the persistent table.
// Kernel boundaries are the only cross-workgroup hand-offs besides the
// device-scope atomics on slot_ref / slot_min.
#include "capsule_gpu.h"
#include "device_common.hpp"
#include "kernels.hpp"

namespace cgpu {

namespace {

constexpr uint32_t kBlock = 256;
constexpr uint32_t kNoSlot = 0xffffffffu;
constexpr uint32_t kFirstBit = 0x80000000u;  // pkt_slot: first packet of a new key
constexpr uint32_t kV4Addr = 0x017100cbu;    // 203.0.113.1 as LE dword of wire bytes
constexpr uint32_t kDataRoom = 2048u;        // RTE_MBUF_DEFAULT_DATAROOM

__device__ __forceinline__ uint32_t sel3(uint32_t k, uint32_t a, uint32_t b, uint32_t c) {
  return k == 0u ? a : (k == 1u ? b : c);
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

// Classification of one input frame by the reference nat_6to4 control flow.
struct V6 {
  uint32_t k, eth_len, len;
  uint32_t disp, st;
  uint32_t L[18];  // L3-relative dwords (v6 header at 0..9, TCP at 10..14)
};

template <int NW>
__device__ __forceinline__ void classify(rsrc_t rs, uint32_t arena_len, uint32_t off,
                                         uint32_t len, V6 &v, uint32_t (&P)[NW]) {
  load_window<NW>(rs, arena_len, off, len < 4u * NW ? len : 4u * NW, P);
  const uint32_t marker = be16_lo(P[3]);
  v.k = marker == 0x8100u ? 1u : (marker == 0x88a8u ? 2u : 0u);
  v.eth_len = 14u + 4u * v.k;
  v.len = len;
  const uint32_t et = be16_lo(sel3(v.k, P[3], P[4], P[5]));
  constexpr int NA = NW - 4;
  uint32_t A[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) A[j] = __builtin_amdgcn_alignbyte(P[4 + j], P[3 + j], 2);
#pragma unroll
  for (int j = 0; j < 18; ++j) {
    if (j + 2 < NA) v.L[j] = sel3(v.k, A[j], A[j + 1], A[j + 2]);
    else v.L[j] = 0u;
  }
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

// ---- K1: classify + probe --------------------------------------------------
__global__ __launch_bounds__(kBlock) void nat64_probe(Nat64Args a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.n) return;
  const rsrc_t rs = make_rsrc(a.arena, a.arena_len);
  V6 v;
  uint32_t P[20];
  classify<20>(rs, a.arena_len, a.off[i], a.len[i], v, P);
  uint32_t slot = kNoSlot;
  if (v.disp == CGPU_ACT) {
    uint32_t key[5];
    make_key(v, key);
    uint32_t h = key_hash(key) & a.pm.cap_mask;
    for (uint32_t probe = 0; probe <= a.pm.cap_mask; ++probe) {
      const uint32_t ref = atomicCAS(&a.pm.slot_ref[h], 0u, i + 1u);
      bool match;
      if (ref == 0u) {
        match = true;  // claimed an empty slot: this packet represents the key
      } else if (ref & kPersist) {
        uint32_t other[5];
#pragma unroll
        for (int j = 0; j < 4; ++j) other[j] = a.pm.key_src[4u * h + j];
        other[4] = a.pm.key_port[h];
        match = key_eq(key, other);
      } else {
        // batch-local entry: compare against the representative's own bytes
        const uint32_t rep = ref - 1u;
        V6 rv;
        uint32_t RP[20];
        classify<20>(rs, a.arena_len, a.off[rep], a.len[rep], rv, RP);
        uint32_t other[5];
        make_key(rv, other);
        match = key_eq(key, other);
      }
      if (match) {
        if (!(ref & kPersist)) atomicMin(&a.pm.slot_min[h], i);
        slot = h;
        break;
      }
      h = (h + 1u) & a.pm.cap_mask;
    }
    if (slot == kNoSlot) {
      v.disp = CGPU_ABORT;
      v.st = CGPU_PKT_TABLE_FULL;
    }
  }
  a.pkt_slot[i] = slot;
  a.disposition[i] = (uint8_t)v.disp;
  a.status[i] = (uint8_t)v.st;
}

__device__ __forceinline__ bool is_first_new(const Nat64Args &a, uint32_t i) {
  const uint32_t slot = a.pkt_slot[i];
  if (slot == kNoSlot) return false;
  return !(a.pm.slot_ref[slot] & kPersist) && a.pm.slot_min[slot] == i;
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
    // inclusive wave scan
    uint32_t x = v;
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
    const uint32_t slot = a.pkt_slot[i];
    a.pm.slot_port[slot] = (a.pm.state[2] + pre + below) & 0xffffu;
    a.pkt_slot[i] = slot | kFirstBit;
  }
}

// Output packet-relative dword j of the rewritten frame, for a fixed VLAN
// depth KK (so every register index is static).  H = new IPv4 header dwords,
// P = input window, pt = tcp src port dword patch.
template <int KK>
__device__ __forceinline__ uint32_t out_dw_k(int j, const uint32_t (&P)[24],
                                             const uint32_t (&H)[5], uint32_t port_be) {
  if (j < 3 + KK) return P[j];
  if (j == 3 + KK) return __builtin_amdgcn_alignbyte(H[0], 0x00080000u, 2);  // ether_type 0x0800
  if (j < 8 + KK) return __builtin_amdgcn_alignbyte(H[j - 3 - KK], H[j - 4 - KK], 2);
  if (j == 8 + KK) return (H[4] >> 16) | (port_be << 16);  // dst tail | new tcp src port
  if (j == 12 + KK) return P[j + 5] & 0x0000ffffu;          // tcp checksum zeroed
  return P[j + 5];                                          // shifted TCP header/payload
}

__device__ __forceinline__ uint32_t out_dw(uint32_t k, int j, const uint32_t (&P)[24],
                                           const uint32_t (&H)[5], uint32_t port_be) {
  return sel3(k, out_dw_k<0>(j, P, H, port_be), out_dw_k<1>(j, P, H, port_be),
              out_dw_k<2>(j, P, H, port_be));
}

// Chunk c (output bytes [16c, 16c+16)) of a frame of `len` bytes at a
// 4-byte-aligned output offset.  Bytes at or past `len` are never written, so
// tightly packed output slots do not clobber each other.
__device__ __forceinline__ void store16(rsrc_t ors, uint32_t out_base, uint32_t c, u32x4 v,
                                        uint32_t len) {
  const uint32_t o = out_base + 16u * c;
  if (16u * c + 16u <= len) {
    __builtin_amdgcn_raw_buffer_store_b128(v, ors, (int)o, 0, 0);
    return;
  }
#pragma unroll
  for (uint32_t t = 0; t < 4u; ++t) {
    const uint32_t b = 16u * c + 4u * t;
    if (b + 4u <= len) {
      __builtin_amdgcn_raw_buffer_store_b32(v[t], ors, (int)(o + 4u * t), 0, 0);
    } else {
      for (uint32_t k = 0; k < 3u; ++k)
        if (b + k < len)
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v[t] >> (8u * k)), ors,
                                               (int)(o + 4u * t + k), 0, 0);
    }
  }
}

__device__ __forceinline__ void store16_bytes(uint8_t *p, uint32_t lim, u32x4 v) {
  for (uint32_t b = 0; b < 16u && b < lim; ++b) p[b] = (uint8_t)(v[b >> 2] >> (8u * (b & 3u)));
}

// ---- K5: rewrite + commit ----------------------------------------------------
__global__ __launch_bounds__(kBlock) void nat64_rewrite(Nat64Args a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.n) return;
  const uint32_t ps = a.pkt_slot[i];
  if (ps == kNoSlot) {
    a.out_len[i] = 0;
    return;
  }
  const uint32_t slot = ps & ~kFirstBit;
  const rsrc_t rs = make_rsrc(a.arena, a.arena_len);
  const uint32_t off = a.off[i];
  const uint32_t len = a.len[i];
  V6 v;
  uint32_t P[24];
  classify<24>(rs, a.arena_len, off, len, v, P);
  const uint32_t k = v.k, eth_len = v.eth_len;
  const uint32_t new_len = len - 20u;
  const uint32_t port = a.pm.slot_port[slot];

  // v6 fields (ip/v6/mod.rs:123-134, 172-200) and the pushed IPv4 header.
  const uint32_t w = be32(v.L[0]);
  const uint32_t dscp = (w & 0x0fc00000u) >> 22, ecn = (w & 0x00300000u) >> 20;
  const uint32_t ttl = ((v.L[1] >> 24) - 1u) & 0xffu;  // hop_limit - 1 (u8, wrapping)
  const uint32_t dscp_ecn = (((dscp << 2) & 0xfcu) | (ecn & 0x3u)) & 0xffu;
  const uint32_t total_len = new_len - eth_len;
  uint32_t H[5];
  H[0] = 0x45u | (dscp_ecn << 8) | (swap16(total_len & 0xffffu) << 16);
  H[1] = 0u;                   // identification 0, flags/frag 0 (v4.rs:594-609)
  H[2] = ttl | (6u << 8);      // protocol = next_header (6); checksum below
  H[3] = kV4Addr;              // V4_ADDR (main.rs:35)
  H[4] = v.L[9];               // map6to4(dst): low 32 bits (main.rs:79-83)
  const uint32_t ip_c =
      (~swap16(fold64((uint64_t)H[0] + H[1] + H[2] + H[3] + H[4]))) & 0xffffu;
  H[2] |= swap16(ip_c) << 16;
  const uint32_t port_be = swap16(port);

  const bool aligned = (a.out_off[i] & 3u) == 0u;
  const uint32_t out_base = a.out_off[i];
  const rsrc_t ors = make_rsrc(a.out_arena, a.out_arena_len);
  uint8_t *obytes = a.out_arena + out_base;

  // TCP span in output packet-relative bytes: [eth_len + 20, new_len).
  const uint32_t span_dw = 8u + k;  // dword holding the span start (hi half)
  uint64_t acc = 0;
  u32x4 chunk3;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    u32x4 o;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = 4 * c + t;
      const uint32_t d = out_dw(k, j, P, H, port_be);
      o[t] = d;
      uint32_t m = (uint32_t)j < span_dw ? 0u : end_mask(j, new_len);
      if ((uint32_t)j == span_dw) m &= 0xffff0000u;
      acc += (uint64_t)(d & m);
    }
    if (c < 3) {
      if (aligned) store16(ors, out_base, c, o, new_len);
      else store16_bytes(obytes + 16 * c, new_len - 16u * c, o);
    } else {
      chunk3 = o;
    }
  }
  // Stream the rest: out dword j = input packet-relative dword j + 5.
  const uint32_t sh = off & 3u, in_base = off - sh;
  for (uint32_t c = 4; 16u * c < new_len; ++c) {
    // input packet-relative dwords 4c+5 .. 4c+8 need absolute dwords 4c+5 .. 4c+9
    const u32x4 q1 = load16(rs, in_base + 16u * (c + 1u), a.arena_len);
    const u32x4 q2 = load16(rs, in_base + 16u * (c + 2u), a.arena_len);
    u32x4 o;
    o[0] = __builtin_amdgcn_alignbyte(q1[2], q1[1], sh);
    o[1] = __builtin_amdgcn_alignbyte(q1[3], q1[2], sh);
    o[2] = __builtin_amdgcn_alignbyte(q2[0], q1[3], sh);
    o[3] = __builtin_amdgcn_alignbyte(q2[1], q2[0], sh);
#pragma unroll
    for (int t = 0; t < 4; ++t) acc += (uint64_t)(o[t] & end_mask((int)(4u * c) + t, new_len));
    if (aligned) store16(ors, out_base, c, o, new_len);
    else store16_bytes(obytes + 16u * c, new_len - 16u * c, o);
  }
  // TCP checksum with the v4 pseudo-header (checksum.rs:93-103).
  const uint32_t span = (new_len - eth_len - 20u) & 0xffffu;
  const uint32_t dst = be32(H[4]);
  const uint32_t ph =
      fold32(0xcb00u + 0x7101u + (dst >> 16) + (dst & 0xffffu) + 6u + span);  // 203.0.113.1
  const uint32_t tcp_c = (~fold32(ph + swap16(fold64(acc)))) & 0xffffu;
  // the checksum sits in the high half of output dword 12 + k (chunk 3)
  const uint32_t cs_t = (12u + k) & 3u;
#pragma unroll
  for (int t = 0; t < 4; ++t)
    if ((uint32_t)t == cs_t) chunk3[t] |= swap16(tcp_c) << 16;
  if (aligned) store16(ors, out_base, 3, chunk3, new_len);
  else store16_bytes(obytes + 48, new_len - 48u, chunk3);

  a.out_len[i] = (uint16_t)new_len;
  if (ps & kFirstBit) {  // commit the new key (PORT_MAP.insert_new, main.rs:49)
    uint32_t key[5];
    make_key(v, key);
#pragma unroll
    for (int j = 0; j < 4; ++j) a.pm.key_src[4u * slot + j] = key[j];
    a.pm.key_port[slot] = key[4];
    a.pm.slot_min[slot] = 0xffffffffu;
    a.pm.slot_ref[slot] = kPersist;
  }
}

__global__ void portmap_init(PortMapDev pm, uint32_t first_port) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= pm.cap_mask) {
    pm.slot_ref[i] = 0u;
    pm.slot_min[i] = 0xffffffffu;
    pm.slot_port[i] = 0u;
    pm.key_port[i] = 0u;
  }
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
  const uint32_t cap = pm.cap_mask + 1u;
  hipLaunchKernelGGL(portmap_init, dim3((cap + 255) / 256), dim3(256), 0, s, pm, first_port);
  return hipGetLastError();
}

hipError_t launch_nat64_6to4(const Nat64Args &a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  const uint32_t nb = nat64_num_blocks(a.n);
  hipLaunchKernelGGL(nat64_probe, dim3(nb), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(nat64_count, dim3(nb), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(nat64_scan, dim3(1), dim3(kScanBlock), 0, s, a, nb);
  hipLaunchKernelGGL(nat64_assign, dim3(nb), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(nat64_rewrite, dim3(nb), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace cgpu
