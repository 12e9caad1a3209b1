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
struct Sip {
  uint64_t v0, v1, v2, v3;
};

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int b) {
  return (x << b) | (x >> (64 - b));
}

__device__ __forceinline__ void sip_round(Sip &s) {
  s.v0 += s.v1;
  s.v1 = rotl64(s.v1, 13);
  s.v1 ^= s.v0;
  s.v0 = rotl64(s.v0, 32);
  s.v2 += s.v3;
  s.v3 = rotl64(s.v3, 16);
  s.v3 ^= s.v2;
  s.v0 += s.v3;
  s.v3 = rotl64(s.v3, 21);
  s.v3 ^= s.v0;
  s.v2 += s.v1;
  s.v1 = rotl64(s.v1, 17);
  s.v1 ^= s.v2;
  s.v2 = rotl64(s.v2, 32);
}

__device__ __forceinline__ Sip sip_init() {
  Sip s;
  s.v0 = 0x736f6d6570736575ull;
  s.v1 = 0x646f72616e646f6dull;
  s.v2 = 0x6c7967656e657261ull;
  s.v3 = 0x7465646279746573ull;
  return s;
}

__device__ __forceinline__ void sip_block(Sip &s, uint64_t m) {
  s.v3 ^= m;
  sip_round(s);
  s.v0 ^= m;
}

__device__ __forceinline__ uint64_t sip_finish(Sip &s, uint64_t b) {
  sip_block(s, b);
  s.v2 ^= 0xffull;
  sip_round(s);
  sip_round(s);
  sip_round(s);
  return s.v0 ^ s.v1 ^ s.v2 ^ s.v3;
}

__device__ __forceinline__ uint64_t u64_of(uint32_t lo, uint32_t hi) {
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// Hash of Flow{src_ip, dst_ip, src_port, dst_port, protocol} as Rust 1.50
// `#[derive(Hash)]` feeds it to DefaultHasher:
//   v4: [0u64][src 4B][0u64][dst 4B][sport le16][dport le16][proto]  = 29 B
//   v6: [1u64][16u64][src 16B][1u64][16u64][dst 16B][ports][proto]   = 69 B
// Addresses are given as the little-endian dwords of their wire bytes.
__device__ __forceinline__ uint64_t flow_hash_v4(uint32_t src, uint32_t dst, uint32_t sport,
                                                 uint32_t dport, uint32_t proto) {
  Sip s = sip_init();
  sip_block(s, 0ull);
  sip_block(s, (uint64_t)src);
  sip_block(s, (uint64_t)dst << 32);
  const uint64_t b = (29ull << 56) | ((uint64_t)proto << 32) | ((uint64_t)dport << 16) |
                     (uint64_t)sport;
  return sip_finish(s, b);
}

__device__ __forceinline__ uint64_t flow_hash_v6(const uint32_t (&src)[4],
                                                 const uint32_t (&dst)[4], uint32_t sport,
                                                 uint32_t dport, uint32_t proto) {
  Sip s = sip_init();
  sip_block(s, 1ull);
  sip_block(s, 16ull);
  sip_block(s, u64_of(src[0], src[1]));
  sip_block(s, u64_of(src[2], src[3]));
  sip_block(s, 1ull);
  sip_block(s, 16ull);
  sip_block(s, u64_of(dst[0], dst[1]));
  sip_block(s, u64_of(dst[2], dst[3]));
  const uint64_t b = (69ull << 56) | ((uint64_t)proto << 32) | ((uint64_t)dport << 16) |
                     (uint64_t)sport;
  return sip_finish(s, b);
}

}  // namespace cgpu
