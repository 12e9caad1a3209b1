// device_common.hpp — CDNA4 device helpers shared by the packet kernels.
//
// * Arena reads go through a raw buffer resource (T8 in the HIP guide): the
//   descriptor is built from kernel arguments only, so it is wave-uniform
//   and lives in SGPRs, and the hardware range check turns any read past
//   `arena_len` into zeros instead of a fault.
// * One's-complement sums are accumulated as little-endian dwords in a u64
//   and folded with end-around carry.  RFC 1071 sums are byte-order and
//   grouping independent modulo 0xFFFF, and a fold of a sum of non-negative
//   terms is zero only when every term is zero, so the result equals the
//   reference's u16-word loop (core/src/packets/checksum.rs:145-168)
//   exactly, including the 0x0000 / 0xFFFF distinction.  DESIGN.md §3 has
//   the derivation.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cgpu {

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ rsrc_t make_rsrc(const void *p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes,
                                           0x00020000);
}

// One dword at a 4-byte-aligned arena offset that may straddle the end of
// the arena.  The buffer range check drops a whole dword that crosses
// num_records, so the bytes still inside are fetched one by one.
__device__ __forceinline__ uint32_t load4_tail(rsrc_t rs, uint32_t byte_off, uint32_t arena_len) {
  if ((uint64_t)byte_off + 4u <= (uint64_t)arena_len)
    return __builtin_amdgcn_raw_buffer_load_b32(rs, (int)byte_off, 0, 0);
  uint32_t v = 0;
  for (uint32_t b = 0; b < 3u; ++b)
    if (byte_off + b < arena_len)
      v |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rs, (int)(byte_off + b), 0, 0) << (8u * b);
  return v;
}

// The dword at any arena byte offset (tail-safe: zero past the arena end).
__device__ __forceinline__ uint32_t load4_any(rsrc_t rs, uint32_t byte_off, uint32_t arena_len) {
  const uint32_t sh = byte_off & 3u, b = byte_off - sh;
  const uint32_t lo = load4_tail(rs, b, arena_len);
  const uint32_t hi = sh ? load4_tail(rs, b + 4u, arena_len) : 0u;
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// 16 bytes at a 4-byte-aligned arena offset.  Near the end of the arena the
// load is split so that bytes up to the last one are still returned (and
// zeros past it).
__device__ __forceinline__ u32x4 load16(rsrc_t rs, uint32_t byte_off, uint32_t arena_len) {
  if ((uint64_t)byte_off + 16u <= (uint64_t)arena_len) {
    return __builtin_amdgcn_raw_buffer_load_b128(rs, (int)byte_off, 0, 0);
  }
  u32x4 v;
  v[0] = load4_tail(rs, byte_off, arena_len);
  v[1] = load4_tail(rs, byte_off + 4u, arena_len);
  v[2] = load4_tail(rs, byte_off + 8u, arena_len);
  v[3] = load4_tail(rs, byte_off + 12u, arena_len);
  return v;
}

// Packet-relative dword window: P[j] = bytes [4j, 4j+4) of the packet that
// starts at arena offset `off`, for the first `wlen` bytes (later bytes are
// whatever follows in the arena, or zero past its end).  Loads are aligned
// to 4 bytes and realigned with v_alignbyte, so any packet offset works.
template <int NW>
__device__ __forceinline__ void load_window(rsrc_t rs, uint32_t arena_len, uint32_t off,
                                            uint32_t wlen, uint32_t (&P)[NW]) {
  constexpr int NC = (NW * 4 + 3 + 15) / 16;
  const uint32_t sh = off & 3u;
  const uint32_t base = off - sh;
  uint32_t D[NC * 4];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    u32x4 v = {0u, 0u, 0u, 0u};
    if ((uint32_t)(16 * c) < sh + wlen) v = load16(rs, base + 16u * c, arena_len);
    D[4 * c + 0] = v[0];
    D[4 * c + 1] = v[1];
    D[4 * c + 2] = v[2];
    D[4 * c + 3] = v[3];
  }
#pragma unroll
  for (int j = 0; j < NW; ++j) P[j] = __builtin_amdgcn_alignbyte(D[j + 1], D[j], sh);
}

// Mask of the bytes of dword j (relative bytes [4j, 4j+4)) that lie below
// `end` (relative).  Little-endian: byte b of the dword is bits [8b, 8b+8).
__device__ __forceinline__ uint32_t end_mask(int j, uint32_t end) {
  const uint32_t lo = 4u * (uint32_t)j;
  if (end >= lo + 4u) return 0xffffffffu;
  if (end <= lo) return 0u;
  return 0xffffffffu >> (8u * (lo + 4u - end));
}

// Fold a u64 sum of little-endian dwords to 16 bits, preserving residue mod
// 0xFFFF and non-zeroness.
__device__ __forceinline__ uint32_t fold64(uint64_t s) {
  uint64_t t = (s & 0xffffffffull) + (s >> 32);
  t = (t & 0xffffffffull) + (t >> 32);
  uint32_t x = (uint32_t)t;
  x = (x & 0xffffu) + (x >> 16);
  x = (x & 0xffffu) + (x >> 16);
  return x;
}

__device__ __forceinline__ uint32_t fold32(uint32_t x) {
  x = (x & 0xffffu) + (x >> 16);
  x = (x & 0xffffu) + (x >> 16);
  return x;
}

__device__ __forceinline__ uint32_t swap16(uint32_t x) {
  return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu);
}

// Big-endian u16 from the low / high half of a little-endian dword.
__device__ __forceinline__ uint32_t be16_lo(uint32_t w) { return swap16(w & 0xffffu); }
__device__ __forceinline__ uint32_t be16_hi(uint32_t w) { return swap16(w >> 16); }
__device__ __forceinline__ uint32_t be32(uint32_t w) { return __builtin_bswap32(w); }

// Little-endian residue sum of arena bytes [s, e) (absolute offsets), in the
// absolute-parity domain (byte at an even address has weight 1).
__device__ __forceinline__ uint64_t sum_abs(rsrc_t rs, uint32_t arena_len, uint32_t s,
                                            uint32_t e) {
  uint64_t acc = 0;
  uint32_t c = s & ~3u;
  // first chunk: mask off bytes below s
  while (c < e) {
    u32x4 v = load16(rs, c, arena_len);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint32_t a = c + 4u * t;
      uint32_t m = 0xffffffffu;
      if (a < s) m = (s - a >= 4u) ? 0u : (0xffffffffu << (8u * (s - a)));
      if (a + 4u > e) m &= (e <= a) ? 0u : (0xffffffffu >> (8u * (a + 4u - e)));
      acc += (uint64_t)(v[t] & m);
    }
    c += 16u;
  }
  return acc;
}

// ---- SipHash-1-3, key (0, 0): Rust std DefaultHasher::new() ---------------
// The 64-bit state words are kept as explicit 32-bit halves: a rotation by
// b < 32 is two v_alignbit_b32, a rotation by 32 is a rename, an add is
// v_add_co + v_addc.  (Letting the compiler see uint64_t produced 64-bit
// shift pairs plus register-pair moves for every rotation.)
struct W64 {
  uint32_t lo, hi;
};

__device__ __forceinline__ W64 w64(uint64_t x) { return W64{(uint32_t)x, (uint32_t)(x >> 32)}; }

__device__ __forceinline__ W64 add64(W64 a, W64 b) {
  W64 r;
  r.lo = a.lo + b.lo;
  r.hi = a.hi + b.hi + (r.lo < a.lo ? 1u : 0u);
  return r;
}

__device__ __forceinline__ W64 xor64(W64 a, W64 b) { return W64{a.lo ^ b.lo, a.hi ^ b.hi}; }

template <int B>
__device__ __forceinline__ W64 rotl64(W64 x) {
  static_assert(B > 0 && B < 32, "rotation by 32 is a swap");
  return W64{__builtin_amdgcn_alignbit(x.lo, x.hi, 32 - B),
             __builtin_amdgcn_alignbit(x.hi, x.lo, 32 - B)};
}

__device__ __forceinline__ W64 swap32(W64 x) { return W64{x.hi, x.lo}; }

struct Sip {
  W64 v0, v1, v2, v3;
};

__device__ __forceinline__ void sip_round(Sip &s) {
  s.v0 = add64(s.v0, s.v1);
  s.v1 = xor64(rotl64<13>(s.v1), s.v0);
  s.v0 = swap32(s.v0);
  s.v2 = add64(s.v2, s.v3);
  s.v3 = xor64(rotl64<16>(s.v3), s.v2);
  s.v0 = add64(s.v0, s.v3);
  s.v3 = xor64(rotl64<21>(s.v3), s.v0);
  s.v2 = add64(s.v2, s.v1);
  s.v1 = xor64(rotl64<17>(s.v1), s.v2);
  s.v2 = swap32(s.v2);
}

__device__ __forceinline__ Sip sip_init() {
  Sip s;
  s.v0 = w64(0x736f6d6570736575ull);
  s.v1 = w64(0x646f72616e646f6dull);
  s.v2 = w64(0x6c7967656e657261ull);
  s.v3 = w64(0x7465646279746573ull);
  return s;
}

__device__ __forceinline__ void sip_block(Sip &s, W64 m) {
  s.v3 = xor64(s.v3, m);
  sip_round(s);
  s.v0 = xor64(s.v0, m);
}

__device__ __forceinline__ uint64_t sip_finish(Sip &s, W64 b) {
  sip_block(s, b);
  s.v2.lo ^= 0xffu;
  sip_round(s);
  sip_round(s);
  sip_round(s);
  const W64 r = xor64(xor64(s.v0, s.v1), xor64(s.v2, s.v3));
  return (uint64_t)r.lo | ((uint64_t)r.hi << 32);
}

// The first compressions of both families absorb constant words (the IpAddr
// discriminant, and for v6 the slice length 16), so the state after them is a
// compile-time constant: sip_const evaluates SipHash on the host compiler.
struct SipC {
  uint64_t v0, v1, v2, v3;
};

constexpr uint64_t rotl_c(uint64_t x, int b) { return (x << b) | (x >> (64 - b)); }

constexpr SipC sip_round_c(SipC s) {
  s.v0 += s.v1;
  s.v1 = rotl_c(s.v1, 13) ^ s.v0;
  s.v0 = rotl_c(s.v0, 32);
  s.v2 += s.v3;
  s.v3 = rotl_c(s.v3, 16) ^ s.v2;
  s.v0 += s.v3;
  s.v3 = rotl_c(s.v3, 21) ^ s.v0;
  s.v2 += s.v1;
  s.v1 = rotl_c(s.v1, 17) ^ s.v2;
  s.v2 = rotl_c(s.v2, 32);
  return s;
}

constexpr SipC sip_block_c(SipC s, uint64_t m) {
  s.v3 ^= m;
  s = sip_round_c(s);
  s.v0 ^= m;
  return s;
}

constexpr SipC kSipInit{0x736f6d6570736575ull, 0x646f72616e646f6dull, 0x6c7967656e657261ull,
                        0x7465646279746573ull};
constexpr SipC kSip4 = sip_block_c(kSipInit, 0);                   // v4: [disc 0]
constexpr SipC kSip6 = sip_block_c(sip_block_c(kSipInit, 1), 16);  // v6: [disc 1][16u64]

__device__ __forceinline__ Sip sip_from(const SipC &c) {
  return Sip{w64(c.v0), w64(c.v1), w64(c.v2), w64(c.v3)};
}

// Hash of Flow{src_ip, dst_ip, src_port, dst_port, protocol} as Rust 1.50
// `#[derive(Hash)]` feeds it to DefaultHasher:
//   v4: [0u64][src 4B][0u64][dst 4B][sport le16][dport le16][proto]  = 29 B
//   v6: [1u64][16u64][src 16B][1u64][16u64][dst 16B][ports][proto]   = 69 B
// Addresses are the little-endian dwords of their wire bytes; sport/dport
// are host-order values.  The constant leading blocks start from kSip4 /
// kSip6.  An all-IPv4 wave (uniform branch) runs 2 compressions + finish on
// constants the compiler folds further (the first block's v0/v1/v2 are
// constant); a mixed wave shares the next two compressions' code and pays 4
// extra ones for its v6 lanes.
__device__ __forceinline__ uint64_t flow_hash(bool v6, const uint32_t (&src)[4],
                                              const uint32_t (&dst)[4], uint32_t sport,
                                              uint32_t dport, uint32_t proto) {
  Sip s;
  if (!__ballot(v6)) {
    s = sip_from(kSip4);
    sip_block(s, W64{src[0], 0u});  // [src][disc lo 0]
    sip_block(s, W64{0u, dst[0]});  // [disc hi 0][dst]
    return sip_finish(s, W64{sport | (dport << 16), proto | (29u << 24)});
  }
  const Sip s4 = sip_from(kSip4), s6 = sip_from(kSip6);
  s.v0 = v6 ? s6.v0 : s4.v0;
  s.v1 = v6 ? s6.v1 : s4.v1;
  s.v2 = v6 ? s6.v2 : s4.v2;
  s.v3 = v6 ? s6.v3 : s4.v3;
  // v4 [src][disc lo 0] [disc hi 0][dst] ; v6 [src 0..7] [src 8..15]
  sip_block(s, W64{src[0], v6 ? src[1] : 0u});
  sip_block(s, v6 ? W64{src[2], src[3]} : W64{0u, dst[0]});
  if (v6) {
    sip_block(s, W64{1u, 0u});
    sip_block(s, W64{16u, 0u});
    sip_block(s, W64{dst[0], dst[1]});
    sip_block(s, W64{dst[2], dst[3]});
  }
  return sip_finish(s, W64{sport | (dport << 16), proto | ((v6 ? 69u : 29u) << 24)});
}

}  // namespace cgpu
