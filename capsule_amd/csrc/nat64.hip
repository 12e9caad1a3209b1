// nat64.hip — examples/nat64 on gfx950: the IPv6 -> IPv4 rewrite ("6to4")
// and the IPv4 -> IPv6 rewrite ("4to6").
//
// Reference: examples/nat64/main.rs:121-150 (nat_6to4), :86-118 (nat_4to6),
// :41-53 (assigned_port), :56-58 (assigned_addr), :62-83 (map4to6 /
// map6to4), :35 (V4_ADDR); Packet::remove (core/src/packets/mod.rs:242) ->
// Mbuf::shrink (mbuf.rs:256-275); Ethernet::push::<Ipv4|Ipv6> (ip/v4.rs:
// 455-469, default header :594-609; ip/v6/mod.rs:302-316, :453-464) ->
// Mbuf::extend (mbuf.rs:225-245); setters (ip/v4.rs:189-203, 293-357);
// Tcp::reconcile_all -> Tcp::compute_checksum (tcp.rs:462-477), then
// Ipv4::reconcile (ip/v4.rs:486-489) / Ipv6::reconcile (ip/v6/mod.rs:331-334).
//
// The reference assigns gateway ports from a global AtomicU16 (first 1025)
// in first-seen order of (v6 src, tcp src port).  A batch reproduces that
// order exactly.  Each direction is one fused kernel per 256-frame block:
//   phase 1  one lane per frame: classify by the reference control flow
//            (Act / Drop / Abort), look the key up in the device port map
//            (6to4: open-addressing PORT_MAP; 4to6: the ADDR_MAP reverse
//            array), and build the frame's new IP header into an LDS record.
//   phase 2  kFG lanes per frame: stream the frame to its output slot, 16-B
//            chunks interleaved across the group (chunk c = 16q + kFG*j + g),
//            each lane loading the input shifted by the header-size change,
//            the header words patched in registers, the TCP span summed with
//            v_sad_u16 and reduced across the group; the lane holding the
//            TCP checksum field stores it last.
// A 6to4 frame whose key is not yet committed (first seen in this batch)
// needs the batch-wide first-seen order, so phase 1 defers it: its header
// record goes to global scratch and its index to a deferred list, and
//   K2 count   per-workgroup count of "first packet of a new key"
//   K3 scan    exclusive scan of the counts (one workgroup) + NEXT_PORT
//   K4 assign  ballot/popcount prefix -> ordinal -> port = base + ordinal
//   K5 rewrite the deferred frames (phase 2's code, list-driven) + commit
// finish them.  When no key is new (the steady state) K2..K5 see an empty
// deferred list and return at once.  Kernel boundaries are the only
// cross-workgroup hand-offs besides device-scope atomics on the table.
#include "capsule_gpu.h"
#include "device_common.hpp"
#include "kernels.hpp"

namespace cgpu {

namespace {

constexpr uint32_t kBlock = 256;
#ifndef CGPU_NAT64_FG
#define CGPU_NAT64_FG 4
#endif
constexpr uint32_t kFG = CGPU_NAT64_FG;      // lanes per frame in the rewrite phase
constexpr uint32_t kFJ = 16u / kFG;          // 16-B chunks per lane per 256-B pass
constexpr uint32_t kNow = 4u;                // record info bit: rewrite in the fused kernel
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

// ---- phase 1 of 6to4: classify + probe + IPv4 header -----------------------
// The pushed IPv4 header (v4.rs:594-609) with the setters of main.rs:133-138
// and Ipv4::reconcile (v4.rs:486-489) already applied, as 5 LE dwords.
__device__ __forceinline__ void ipv4_header(const V6 &v, uint32_t len, uint32_t (&H)[5]) {
  const uint32_t w = be32(v.L[0]);
  const uint32_t dscp = (w & 0x0fc00000u) >> 22, ecn = (w & 0x00300000u) >> 20;
  const uint32_t ttl = ((v.L[1] >> 24) - 1u) & 0xffu;  // hop_limit - 1 (u8, wrapping)
  const uint32_t dscp_ecn = (((dscp << 2) & 0xfcu) | (ecn & 0x3u)) & 0xffu;
  const uint32_t new_len = len - 20u;
  H[0] = 0x45u | (dscp_ecn << 8) | (swap16((new_len - v.eth_len) & 0xffffu) << 16);
  H[1] = 0u;               // identification 0, flags/fragment 0
  H[2] = ttl | (6u << 8);  // protocol = next_header (6)
  H[3] = kV4Addr;          // V4_ADDR (main.rs:35)
  H[4] = v.L[9];           // map6to4(dst): low 32 bits (main.rs:79-83)
  const uint32_t ip_c = (~swap16(fold64((uint64_t)H[0] + H[1] + H[2] + H[3] + H[4]))) & 0xffffu;
  H[2] |= swap16(ip_c) << 16;
}

// assigned_port (main.rs:41-53) lookup for frame i: returns the table slot
// (kNoSlot: table full) and, for a key committed by an earlier batch, its
// port; a key first seen in this batch is claimed (CAS) or joined, and its
// first packet index recorded (atomicMin) for K2..K4.
__device__ __forceinline__ uint32_t probe_port(const Nat64Args &a, rsrc_t rs, uint32_t i, const V6 &v,
                                               uint32_t &port) {
  uint32_t key[5];
  make_key(v, key);
  uint32_t h = key_hash(key) & a.pm.cap_mask;
  port = 0xffffffffu;
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
      if (ref & kPersist) return h;
      atomicMin(&a.pm.slots[h].w[7], i);
      return h | kLocalBit;
    }
    h = (h + 1u) & a.pm.cap_mask;
  }
  return kNoSlot;
}

// ---- phase 2 / K5: the rewrite of one frame by its group of kFG lanes --------
// A frame record: info = k | kNow | port << 16 (6to4: the assigned port;
// 4to6: the original v6-side port); V = the new IP header as LE dwords (6to4:
// IPv4 H[0..4]; 4to6: the 40-B IPv6 header); ph = 4to6 pseudo-header residue.
struct FrameRec {
  uint32_t in_off, o_off, new_len, info;
  uint32_t V[10];
  uint32_t ph;
};

// Output dword at header-relative position r (frame dword - VLAN depth) in
// the header region; x is the input dword loaded for it.
template <bool TO4>
__device__ __forceinline__ uint32_t out_dword(int r, uint32_t x, const uint32_t (&V)[10],
                                              uint32_t port_be) {
  uint32_t d = x;
  if (TO4) {
    if (r == 3) d = __builtin_amdgcn_alignbyte(V[0], 0x00080000u, 2);  // ether_type 0x0800
#pragma unroll
    for (int h = 4; h <= 7; ++h)
      if (r == h) d = __builtin_amdgcn_alignbyte(V[h - 3], V[h - 4], 2);
    if (r == 8) d = (V[4] >> 16) | (port_be << 16);  // dst tail | TCP src port
    if (r == 12) d &= 0x0000ffffu;                     // TCP checksum zeroed
  } else {
    if (r == 3) d = __builtin_amdgcn_alignbyte(V[0], 0xdd860000u, 2);  // ether_type 0x86dd
#pragma unroll
    for (int h = 4; h <= 12; ++h)
      if (r == h) d = __builtin_amdgcn_alignbyte(V[h - 3], V[h - 4], 2);
    if (r == 13) d = (x & 0xffff0000u) | (V[9] >> 16);  // dst tail | TCP src port
    if (r == 14) d = (x & 0xffff0000u) | port_be;       // TCP dst port | seq
    if (r == 17) d &= 0x0000ffffu;                      // TCP checksum zeroed
  }
  return d;
}

// Store output chunk c (16 B) of a frame of nl bytes; never past nl.
template <bool FAST>
__device__ __forceinline__ void store_chunk(rsrc_t ors, uint8_t *out_arena, uint32_t o_off,
                                            uint32_t c, u32x4 v, uint32_t nl) {
  const uint32_t b0 = 16u * c;
  if (!FAST) {
    if (b0 < nl) store_out(ors, out_arena, o_off, c, v, nl, (o_off & 3u) == 0u);
    return;
  }
  __builtin_amdgcn_raw_buffer_store_b128(v, ors, (int)(b0 + 16u <= nl ? o_off + b0 : kNoRead), 0, 0);
  if (b0 < nl && b0 + 16u > nl) {  // the partial last chunk: dword and byte stores
#pragma unroll
    for (uint32_t t = 0; t < 4u; ++t) {
      const uint32_t b = b0 + 4u * t;
      __builtin_amdgcn_raw_buffer_store_b32(v[t], ors, (int)(b + 4u <= nl ? o_off + b : kNoRead), 0, 0);
#pragma unroll
      for (uint32_t x = 0; x < 3u; ++x)
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v[t] >> (8u * x)), ors,
                                             (int)(b + 4u > nl && b + x < nl ? o_off + b + x : kNoRead), 0, 0);
    }
  }
}

// Output byte b of the rewritten frame comes from input byte b (Ethernet,
// chunks 0-1), from the header record, or from input byte b + 20 (6to4) /
// b - 20 (4to6) (the TCP segment, chunks >= 2).  FAST (wave-uniform): every
// frame of the wave is dword-aligned on both sides and well inside both
// arenas, so loads and full-chunk stores are branch-free (an unneeded chunk
// gets an offset past num_records: zero load, dropped store).
template <bool TO4, bool FAST>
__device__ __forceinline__ void rewrite_frame(const Nat64Args &a, rsrc_t rs, rsrc_t ors, uint32_t g,
                                              const FrameRec &f, bool in_al_wave) {
  constexpr uint32_t kHdrC = TO4 ? 4u : 5u;  // chunks holding header words / patches
  constexpr uint32_t kHold = TO4 ? 3u : 4u;  // chunk holding the TCP checksum field
  constexpr int kSpanR = TO4 ? 8 : 13;       // first TCP dword (its high half)
  const uint32_t k = f.info & 3u, port_be = swap16(f.info >> 16), nl = f.new_len;
  uint32_t acc = 0;
  u32x4 held = {0u, 0u, 0u, 0u};
  for (uint32_t q = 0; 256u * q < nl; ++q) {
    u32x4 o[kFJ];
#pragma unroll
    for (uint32_t j = 0; j < kFJ; ++j) {
      const uint32_t c = 16u * q + kFG * j + g;
      const uint32_t src = c < 2u ? f.in_off + 16u * c
                                  : (TO4 ? f.in_off + 16u * c + 20u : f.in_off + 16u * c - 20u);
      const bool need = 16u * c < nl;
      if (FAST) {
        o[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(need ? src : kNoRead), 0, 0);
      } else {
        o[j] = u32x4{0u, 0u, 0u, 0u};
        if (need) o[j] = load_in(rs, a.arena_len, src, in_al_wave);
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < kFJ; ++j) {
      const uint32_t c = 16u * q + kFG * j + g;
      if (c < kHdrC) {
#pragma unroll
        for (uint32_t t = 0; t < 4u; ++t) {
          const int r = (int)(4u * c + t) - (int)k;
          const uint32_t d = out_dword<TO4>(r, o[j][t], f.V, port_be);
          uint32_t m = r < kSpanR ? 0u : (r == kSpanR ? 0xffff0000u : 0xffffffffu);
          m &= range_mask(16u * c + 4u * t, 0u, nl);
          acc = sad16(d & m, acc);
          o[j][t] = d;
        }
      } else {
        acc = sad16(o[j][3], sad16(o[j][2], sad16(o[j][1], sad16(o[j][0], acc))));
        if (16u * c < nl && 16u * c + 16u > nl) {  // bytes past the end of the frame
#pragma unroll
          for (uint32_t t = 0; t < 4u; ++t) {
            const uint32_t x = o[j][t] & ~range_mask(16u * c + 4u * t, 0u, nl);
            acc -= (x & 0xffffu) + (x >> 16);
          }
        }
      }
      if (c == kHold) held = o[j];
    }
#pragma unroll
    for (uint32_t j = 0; j < kFJ; ++j) {
      const uint32_t c = 16u * q + kFG * j + g;
      if (c != kHold) store_chunk<FAST>(ors, a.out_arena, f.o_off, c, o[j], nl);
    }
  }
#pragma unroll
  for (uint32_t d = kFG / 2; d > 0; d >>= 1) acc += __shfl_xor(acc, d, kFG);
  if (g == kHold % kFG) {
    uint32_t tcp_c;
    if (TO4) {
      // v4 pseudo-header (checksum.rs:93-103): 203.0.113.1, dst, 6, span
      const uint32_t span = (nl - (34u + 4u * k)) & 0xffffu;
      const uint32_t dst = be32(f.V[4]);
      const uint32_t ph = fold32(0xcb00u + 0x7101u + (dst >> 16) + (dst & 0xffffu) + 6u + span);
      tcp_c = (~fold32(ph + swap16(fold32(acc)))) & 0xffffu;
    } else {
      // v6 pseudo-header (checksum.rs:123-128): addresses (ph), span, 6
      const uint32_t span = (nl - (54u + 4u * k)) & 0xffffu;
      tcp_c = (~fold32(swap16(fold32(acc + f.ph)) + span + 6u)) & 0xffffu;
    }
    const uint32_t tw = TO4 ? k : k + 1u;  // dword of the checksum field in the held chunk
#pragma unroll
    for (uint32_t t = 0; t < 4u; ++t)
      if (t == tw) held[t] |= swap16(tcp_c) << 16;
    store_chunk<FAST>(ors, a.out_arena, f.o_off, kHold, held, nl);
  }
}

// Runs rewrite_frame with the wave-uniform FAST decision.
template <bool TO4>
__device__ __forceinline__ void rewrite_dispatch(const Nat64Args &a, rsrc_t rs, rsrc_t ors,
                                                 uint32_t g, const FrameRec &f) {
  const bool fast = !__ballot(!((f.in_off & 3u) == 0u && (f.o_off & 3u) == 0u &&
                                (uint64_t)f.in_off + f.new_len + 64u <= (uint64_t)a.arena_len &&
                                (uint64_t)f.o_off + f.new_len + 16u <= (uint64_t)a.out_arena_len));
  if (fast) {
    rewrite_frame<TO4, true>(a, rs, ors, g, f, true);
  } else {
    const bool in_al_wave = !__ballot((f.in_off & 3u) != 0u);
    rewrite_frame<TO4, false>(a, rs, ors, g, f, in_al_wave);
  }
}

// Phase 2 of the fused kernels: the block's ready frames, kBlock / kFG at a
// time.  LDS record (4 x 16 B): {in_off, o_off, new_len, info}, V[0..3],
// V[4..7], {V[8], V[9], ph, -}.
template <bool TO4>
__device__ __forceinline__ void rewrite_block(const Nat64Args &a, const u32x4 (*lrec)[4]) {
  const uint32_t g = threadIdx.x % kFG;
  const rsrc_t rs = make_rsrc(a.arena, a.arena_len);
  const rsrc_t ors = make_rsrc(a.out_arena, a.out_arena_len);
  for (uint32_t it = 0; it < kFG; ++it) {
    const uint32_t fl = it * (kBlock / kFG) + threadIdx.x / kFG;
    const u32x4 r0 = lrec[fl][0];
    if (!(r0[3] & kNow)) continue;  // uniform within the group
    const u32x4 r1 = lrec[fl][1], r2 = lrec[fl][2], r3 = lrec[fl][3];
    FrameRec f;
    f.in_off = r0[0];
    f.o_off = r0[1];
    f.new_len = r0[2];
    f.info = r0[3];
    f.V[0] = r1[0]; f.V[1] = r1[1]; f.V[2] = r1[2]; f.V[3] = r1[3];
    f.V[4] = r2[0]; f.V[5] = r2[1]; f.V[6] = r2[2]; f.V[7] = r2[3];
    f.V[8] = r3[0]; f.V[9] = r3[1];
    f.ph = r3[2];
    rewrite_dispatch<TO4>(a, rs, ors, g, f);
    if (g == 0u) a.out_len[blockIdx.x * kBlock + fl] = (uint16_t)f.new_len;
  }
}

// ---- 6to4 fused kernel ------------------------------------------------------
__global__ __launch_bounds__(kBlock) void nat64_6to4_fused(Nat64Args a) {
  __shared__ u32x4 lrec[kBlock][4];
  const uint32_t t = threadIdx.x, lane = t & 63u;
  const uint32_t i = blockIdx.x * kBlock + t;
  const bool valid = i < a.n;
  const rsrc_t rs = make_rsrc(a.arena, a.arena_len);
  const uint32_t off = valid ? a.off[i] : 0u, len = valid ? (uint32_t)a.len[i] : 0u;
  V6 v;
  classify(rs, a.arena_len, off, len, v);
  bool deferred = false;
  uint32_t info = 0u;
  if (valid) {
    uint32_t slot = kNoSlot;
    if (v.disp == CGPU_ACT) {
      uint32_t port;
      slot = probe_port(a, rs, i, v, port);
      if (slot == kNoSlot) {
        v.disp = CGPU_ABORT;
        v.st = CGPU_PKT_TABLE_FULL;
      } else {
        uint32_t H[5];
        ipv4_header(v, len, H);
        if (port != 0xffffffffu) {  // committed key: finished in phase 2
          info = v.k | kNow | (port << 16);
          lrec[t][0] = u32x4{off, a.out_off[i], len - 20u, info};
          lrec[t][1] = u32x4{H[0], H[1], H[2], H[3]};
          lrec[t][2] = u32x4{H[4], 0u, 0u, 0u};
          slot = kNoSlot;
        } else {  // new key: its port needs the batch-wide order (K2..K5)
          deferred = true;
          a.rec_h[i] = u32x4{H[0], H[1], H[2], H[3]};
          a.rec_b[i] = make_uint2(H[4], v.k);
        }
      }
    }
    if (v.disp != CGPU_ACT) a.out_len[i] = 0;
    a.pkt_slot[i] = slot;
    a.disposition[i] = (uint8_t)v.disp;
    a.status[i] = (uint8_t)v.st;
  }
  if (!(info & kNow)) lrec[t][0] = u32x4{0u, 0u, 0u, 0u};
  // append the deferred frames to the list (one atomic per wave)
  const uint64_t dm = __ballot(deferred);
  if (dm) {
    const uint32_t leader = (uint32_t)__builtin_ctzll(dm);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&a.pm.state[4u + a.par], (uint32_t)__popcll(dm));
    base = __shfl(base, (int)leader);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(dm >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0u));
    if (deferred) a.defer[base + rank] = i;
  }
  __syncthreads();
  rewrite_block<true>(a, lrec);
}

// Only packets whose key was first seen in this batch touch the table here.
__device__ __forceinline__ bool is_first_new(const Nat64Args &a, uint32_t i) {
  const uint32_t ps = a.pkt_slot[i];
  if (ps == kNoSlot || !(ps & kLocalBit)) return false;
  return a.pm.slots[ps & kSlotMask].w[7] == i;
}

// ---- K2: per-block count of first packets of new keys ----------------------
__global__ __launch_bounds__(kBlock) void nat64_count(Nat64Args a) {
  if (a.pm.state[4u + a.par] == 0u) return;  // nothing deferred: K3 ignores block_sums
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
  if (a.pm.state[4u + a.par] == 0u) {  // no new key in this batch
    if (threadIdx.x == 0) {
      a.pm.state[2] = a.pm.state[0];
      a.pm.state[3] = 0u;
    }
    return;
  }
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
  if (a.pm.state[4u + a.par] == 0u) return;
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


// ---- K5: the deferred frames (phase 2's rewrite, list-driven) + commit -------
__global__ __launch_bounds__(kBlock) void nat64_6to4_deferred(Nat64Args a) {
  const uint32_t cnt = a.pm.state[4u + a.par];
  const uint32_t g = threadIdx.x % kFG;
  const rsrc_t rs = make_rsrc(a.arena, a.arena_len);
  const rsrc_t ors = make_rsrc(a.out_arena, a.out_arena_len);
  for (uint32_t e = blockIdx.x * (kBlock / kFG) + threadIdx.x / kFG; e < cnt;
       e += gridDim.x * (kBlock / kFG)) {
    const uint32_t p = a.defer[e];
    const uint32_t ps = a.pkt_slot[p], slot = ps & kSlotMask;
    const u32x4 hv = a.rec_h[p];
    const uint2 bv = a.rec_b[p];
    FrameRec f;
    f.in_off = a.off[p];
    f.o_off = a.out_off[p];
    f.new_len = (uint32_t)a.len[p] - 20u;
    f.info = (bv.y & 3u) | (a.pm.slots[slot].w[6] << 16);  // port from K4
    f.V[0] = hv[0]; f.V[1] = hv[1]; f.V[2] = hv[2]; f.V[3] = hv[3]; f.V[4] = bv.x;
#pragma unroll
    for (int j = 5; j < 10; ++j) f.V[j] = 0u;
    f.ph = 0u;
    rewrite_dispatch<true>(a, rs, ors, g, f);
    if (g == 0u) {
      a.out_len[p] = (uint16_t)f.new_len;
      if (ps & kFirstBit) {  // commit the new key (PORT_MAP.insert_new, main.rs:49)
        a.pm.slots[slot].w[7] = 0xffffffffu;
        a.pm.slots[slot].w[0] = kPersist;
      }
    }
  }
  // the other parity's list counter is the next call's: clear it for that call
  if (blockIdx.x == 0 && threadIdx.x == 0) a.pm.state[4u + (a.par ^ 1u)] = 0u;
}

// ============================ 4to6 direction =================================
// Phase 1: classify, look the TCP destination port up in the reverse map
// ADDR_MAP (rev[port] -> slot -> the v6 key), build the IPv6 header; phase 2
// as in 6to4 with the input shifted by -20 bytes behind the 40-byte header
// (the TCP checksum field, output bytes 70+4k, is in chunk 4).
__global__ __launch_bounds__(kBlock) void nat64_4to6_fused(Nat64Args a) {
  __shared__ u32x4 lrec[kBlock][4];
  const uint32_t t = threadIdx.x;
  const uint32_t i = blockIdx.x * kBlock + t;
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
  uint32_t info = 0u;
  if (valid) {
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
              disp = CGPU_ACT;
              const u32x4 *sp = reinterpret_cast<const u32x4 *>(&a.pm.slots[(uint32_t)r]);
              const u32x4 s0 = sp[0], s1 = sp[1];
              const uint32_t de = (L[0] >> 8) & 0xffu;             // dscp_ecn (v4.rs:186-203)
              const uint32_t dscp = de >> 2, ecn = de & 3u;
              const uint32_t hop = ((L[2] & 0xffu) - 1u) & 0xffu;   // ttl - 1 (u8, wrapping)
              const uint32_t new_len = len + 20u;
              // Ipv6Header::default + set_dscp/ecn/next_header/hop_limit/src/dst
              const uint32_t w = (6u << 28) | ((dscp << 22) & 0x0fc00000u) | ((ecn << 20) & 0x00300000u);
              const uint32_t V0 = be32(w);
              const uint32_t V1 = swap16((new_len - eth_len - 40u) & 0xffffu) | (6u << 16) | (hop << 24);
              const uint32_t V2 = 0x9bff6400u;  // 64:ff9b::/96 (map4to6, main.rs:62-74)
              const uint32_t V5 = L[3];         // v4 source address
              // V6..V9: the ADDR_MAP key, the original v6 source
              uint32_t ph = 0;                  // v6 pseudo-header addresses, LE residue
              ph = sad16(V2, ph);
              ph = sad16(V5, ph);
              ph = sad16(s0[1], sad16(s0[2], sad16(s0[3], sad16(s1[0], ph))));
              info = k | kNow | (s1[1] << 16);  // the original v6-side port
              lrec[t][0] = u32x4{off, a.out_off[i], new_len, info};
              lrec[t][1] = u32x4{V0, V1, V2, 0u};
              lrec[t][2] = u32x4{0u, V5, s0[1], s0[2]};
              lrec[t][3] = u32x4{s0[3], s1[0], fold32(ph), 0u};
            }
          }
        }
      }
    }
    if (disp != CGPU_ACT) a.out_len[i] = 0;
    a.disposition[i] = (uint8_t)disp;
    a.status[i] = (uint8_t)st;
  }
  if (!(info & kNow)) lrec[t][0] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  rewrite_block<false>(a, lrec);
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
    pm.state[4] = 0u;  // deferred-list counters, by call parity
    pm.state[5] = 0u;
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
  const uint32_t nb5 = (a.n + kBlock / kFG - 1) / (kBlock / kFG);
  hipLaunchKernelGGL(nat64_6to4_fused, dim3(nb), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(nat64_count, dim3(nb), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(nat64_scan, dim3(1), dim3(kScanBlock), 0, s, a, nb);
  hipLaunchKernelGGL(nat64_assign, dim3(nb), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(nat64_6to4_deferred, dim3(nb5 < 2048u ? nb5 : 2048u), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_nat64_4to6(const Nat64Args &a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(nat64_4to6_fused, dim3(nat64_num_blocks(a.n)), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace cgpu
