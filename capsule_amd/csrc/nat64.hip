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
// order exactly.  6to4 is three launches (the fused kernel, the tail's order
// and patch launches), 4to6 one.
//
// The fused kernels (nat64_6to4_fused, nat64_4to6_fused): a wave owns 32
// frames.  Waves whose frames are 16-B aligned in the input, dword-aligned
// in the output and short enough for one 256-B row pass take the ROWS path:
// 16-lane row j loads frame 4r + j in round r (four whole frames per load
// instruction), bytes 0..95 of each frame reach its own lane through
// wave-private LDS, the lane classifies the frame by the reference control
// flow and looks its key up (6to4: the PORT_MAP slot table; 4to6: the
// ADDR_MAP arrays), the payload is moved by 20 B with DPP row shifts and
// summed by a DPP row reduction while the lookup is in flight, and row j
// stores frame 4r + j in one instruction with the header chunks and the TCP
// checksum patched in.  Other waves take the QUAD path: a quad of lanes per
// frame (any alignment, any length), DPP quad broadcasts of the header.
//
// A 6to4 frame whose key is not yet committed (first seen in this batch) is
// written with source port 0 and deferred (its checksum stashed): its key is
// claimed in the slot table or joined on the claim's tag (probe_port_at),
// and the tail (nat64_tail_order, nat64_tail_patch) verifies the tag joins,
// orders the batch's new keys by their first packet, assigns NEXT_PORT +
// ordinal, commits them, and patches only the deferred frames' port and
// checksum.  With no new key (the steady state) both tail launches return at
// once.
#include <hip/hip_ext.h>

#include "capsule_gpu.h"
#include "device_common.hpp"
#include "kernels.hpp"

namespace cgpu {

namespace {

constexpr uint32_t kBlock = 256;
// cache policy bits of the frame-stream loads and stores: the default
// policy (nontemporal and sc1 variants were slower)
constexpr int kAux = 0;
#define NAT64_OCC __attribute__((amdgpu_waves_per_eu(1)))
constexpr uint32_t kFG = 4u;                 // lanes per frame in the rewrite phase
constexpr uint32_t kFJ = 16u / kFG;          // 16-B chunks per lane per 256-B pass
constexpr uint32_t kNow = 4u;                // record info bit: rewrite in the fused kernel
constexpr uint32_t kNoSlot = 0xffffffffu;
constexpr uint32_t kLocalBit = 0x40000000u;  // pkt_slot: key first seen in this batch
constexpr uint32_t kClaimBit = 0x20000000u;  // pkt_slot: this packet claimed the slot
constexpr uint32_t kPatchBit = 0x80000000u;  // pkt_slot (tail repair): a committed key's port
constexpr uint32_t kSlotMask = 0x1fffffffu;  // slot index (capacity_log2 <= 29)
constexpr uint32_t kV4Addr = 0x017100cbu;    // 203.0.113.1 as LE dword of wire bytes
// The tailroom model of Mbuf::extend (mbuf.rs:225-233) is Nat64Args::room:
// RTE_MBUF_DEFAULT_DATAROOM = 2048 for device batches; on the mbuf path the
// host passes 65535 and the scatter checks each mbuf's real tailroom.
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

// Both hashes are keyed per map (cgpu_portmap_create: a random seed and a
// random odd multiplier per key word for each), so that keys sharing a
// probe chain or a claim tag cannot be chosen from outside (crafted
// collisions would send every such packet through the tail's serial
// repair).  Each key word enters the state multiplied by its own secret
// multiplier: the state difference two keys leave after word j depends on
// m_j, so no pair of keys -- and no difference between words j and j + 1 --
// cancels for every map (with one fixed multiplier, a bit-31 difference in
// word j and a matching one in word j + 1 cancelled for every seed).  This
// is a universal-hash argument against keys chosen without knowledge of
// the map's secrets, not a cryptographic PRF; correctness never depends on
// it (equal tags are verified on the key words by the tail).
__device__ __forceinline__ uint32_t key_hash(const uint32_t (&key)[5], const PortMapDev &pm) {
  uint32_t h = 0x9e3779b9u ^ pm.seed_hash;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    h ^= key[j] * pm.mul_hash[j];
    h = rotl32(h, 13) * 5u + 0xe6546b64u;
  }
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

// The claim tag: a second, independent hash of the key (a batch-local slot
// whose tag differs holds another key; an equal tag is confirmed on the key
// words).
__device__ __forceinline__ uint32_t key_tag(const uint32_t (&key)[5], const PortMapDev &pm) {
  uint32_t h = 0x2545f491u ^ pm.seed_tag;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    h = (h ^ key[j]) * pm.mul_tag[j];
    h ^= h >> 15;
  }
  h *= 0x85ebca77u;
  h ^= h >> 13;
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

// V6 from frame-relative dwords P[3..16] (bytes 12..67: the VLAN marker
// through the TCP source port at QinQ depth); the checks follow the
// reference nat_6to4 control flow in order.
// NOVLAN: the caller knows that no frame of the wave carries a VLAN marker
// (static header positions, no per-dword selects).
template <bool NOVLAN = false>
__device__ __forceinline__ void classify_dwords(const uint32_t (&P)[20], uint32_t len,
                                                uint32_t room, V6 &v) {
  const uint32_t marker = be16_lo(P[3]);
  v.k = NOVLAN ? 0u : (marker == 0x8100u ? 1u : (marker == 0x88a8u ? 2u : 0u));
  v.eth_len = 14u + 4u * v.k;
  const uint32_t et = NOVLAN ? marker : be16_lo(sel3(v.k, P[3], P[4], P[5]));
  uint32_t A[13];
#pragma unroll
  for (int j = 0; j < (NOVLAN ? 11 : 13); ++j) A[j] = __builtin_amdgcn_alignbyte(P[4 + j], P[3 + j], 2);
#pragma unroll
  for (int j = 0; j < 11; ++j) v.L[j] = NOVLAN ? A[j] : sel3(v.k, A[j], A[j + 1], A[j + 2]);
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
  if (!(20u < (shrunk < room ? room - shrunk : 0u))) {
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

// One lane's own classification of a frame (the port-map probe reads a
// batch-local key's representative frame with it): tail-safe dword loads of
// bytes 0..79, zero past the frame end.
__device__ __forceinline__ void classify(rsrc_t rs, uint32_t arena_len, uint32_t off,
                                         uint32_t len, uint32_t room, V6 &v) {
  constexpr int NW = 20;
  uint32_t P[NW];
  if ((off & 3u) == 0u && (uint64_t)off + 80u <= (uint64_t)arena_len) {
    // a dword-aligned frame well inside the arena: five 16-B loads (bytes
    // past the frame's end are never used: classify checks len first)
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      const u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off + 16u * c), 0, 0);
      P[4 * c] = t[0]; P[4 * c + 1] = t[1]; P[4 * c + 2] = t[2]; P[4 * c + 3] = t[3];
    }
    classify_dwords(P, len, room, v);
    return;
  }
  const uint32_t sh = off & 3u, base = off - sh;
  const uint32_t need = sh + (len < 80u ? len : 80u);
  uint32_t D[NW + 1];
#pragma unroll
  for (int j = 0; j < NW + 1; ++j)
    D[j] = (uint32_t)(4 * j) < need ? load4_tail(rs, base + 4u * j, arena_len) : 0u;
#pragma unroll
  for (int j = 0; j < NW; ++j) P[j] = __builtin_amdgcn_alignbyte(D[j + 1], D[j], sh);
  classify_dwords(P, len, room, v);
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
    __builtin_amdgcn_raw_buffer_store_b128(v, ors, (int)o, 0, kAux);
    return;
  }
#pragma unroll
  for (uint32_t t = 0; t < 4u; ++t) {
    const uint32_t b = 16u * c + 4u * t;
    if (aligned && b + 4u <= len) {
      __builtin_amdgcn_raw_buffer_store_b32(v[t], ors, (int)(o + 4u * t), 0, kAux);
    } else {
      for (uint32_t q = 0; q < 4u; ++q)
        if (b + q < len) out_arena[o + 4u * t + q] = (uint8_t)(v[t] >> (8u * q));
    }
  }
}

// ---- 6to4: the new IPv4 header, the port-map probe ---------------------------
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
// port; a key first seen in this batch is claimed or joined, and its first
// packet index recorded (atomicMin) for the tail kernel.
//
// A claim is one 64-bit CAS of {ref = i + 1, tag} into an empty slot; the
// claimer then writes the key words (plain stores: nothing in this launch
// reads them) and its index into w[7].  A packet that finds a batch-local
// claim with its own tag joins it on the tag alone: it stashes its key, and
// the tail compares the stash with the slot's key words behind the kernel
// boundary, where they are coherent, and repairs the rare collision (two
// keys of one tag in one probe chain).  No lane waits for another: a wait on
// a claimer's publish would need the key words read at the coherence point
// (atomics; plain and sc1 loads can be served a stale copy of the slot line
// by the XCD's L2, which this lane's own probe load filled), and costs more
// than the stash.  A different tag is a different key: next slot.  Keys
// committed by earlier batches are matched from the 32-B slot load (their
// words were written by an earlier launch).  refs only ever go 0 -> (i + 1)
// -> kPersist, and a claim's tag never changes, so a stale probe load at
// worst leads to the CAS, which returns the coherent word.
__device__ __forceinline__ uint32_t probe_port_at(const Nat64Args &a, uint32_t i,
                                                  const uint32_t (&key)[5], uint32_t h, u32x4 s0,
                                                  u32x4 s1, uint32_t &port) {
  port = 0xffffffffu;
  uint32_t tag = 0;  // computed when a slot is not a committed key (never in the steady state)
  bool have_tag = false;
  for (uint32_t probe = 0; probe <= a.pm.cap_mask; ++probe) {
    if (probe != 0u) {  // the first slot was loaded by the caller
      const u32x4 *sp = reinterpret_cast<const u32x4 *>(&a.pm.slots[h]);
      s0 = sp[0];
      s1 = sp[1];
    }
    uint32_t *w = a.pm.slots[h].w;
    uint32_t ref = s0[0], stag = s0[1];
    if (!(ref & kPersist) && !have_tag) {
      tag = key_tag(key, a.pm) & a.pm.tag_mask;
      have_tag = true;
    }
    if (ref == 0u) {
      const unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long *>(w), 0ull,
                                               (unsigned long long)(i + 1u) |
                                                   ((unsigned long long)tag << 32));
      if (old == 0ull) {  // claimed: the key words, read behind the kernel boundary only
        *reinterpret_cast<u32x2 *>(&w[2]) = u32x2{key[0], key[1]};
        *reinterpret_cast<u32x2 *>(&w[4]) = u32x2{key[2], key[3]};
        w[6] = key[4];
        atomicMin(&w[7], i);
        return h | kLocalBit | kClaimBit;
      }
      ref = (uint32_t)old;
      stag = (uint32_t)(old >> 32);
    }
    if (ref & kPersist) {
      const uint32_t other[5] = {s0[2], s0[3], s1[0], s1[1], s1[2] & 0xffffu};
      if (key_eq(key, other)) {
        port = s1[2] >> 16;
        return h;
      }
    } else if (stag == tag) {
      // joined on the tag alone: the key goes to the stash; the key's first
      // packet index.  w[7] only decreases and never exceeds the claimer's
      // index (ref - 1), so a packet after the claimer, or after a w[7]
      // loaded with the slot, needs no atomic: with the packets probing in
      // about their own order, most joiners of a key skip it
      a.stash_key[i] = u32x4{key[0], key[1], key[2], key[3]};
      a.stash_port[i] = (uint16_t)key[4];
      if (s1[3] > i && i + 1u < ref) atomicMin(&w[7], i);
      return h | kLocalBit;
    }
    h = (h + 1u) & a.pm.cap_mask;
  }
  return kNoSlot;
}

__device__ __forceinline__ uint32_t probe_port(const Nat64Args &a, uint32_t i, const V6 &v,
                                               uint32_t &port) {
  uint32_t key[5];
  make_key(v, key);
  const uint32_t h = key_hash(key, a.pm) & a.pm.cap_mask;
  const u32x4 *sp = reinterpret_cast<const u32x4 *>(&a.pm.slots[h]);
  return probe_port_at(a, i, key, h, sp[0], sp[1], port);
}

// ---- the rewrite of one frame by its quad (the fused kernel's quad path) -----
// A frame record: info = k | kNow | port << 16 (6to4: the assigned port;
// 4to6: the original v6-side port); V = the new IP header as LE dwords (6to4:
// IPv4 H[0..4]; 4to6: the 40-B IPv6 header); ph = 4to6 pseudo-header residue.
struct FrameRec {
  uint32_t in_off, o_off, new_len, info;
  uint32_t V[10];
  uint32_t ph;
  uint32_t defer_i;  // 6to4: the packet index of a deferred frame (its checksum is
                     // stashed for the tail), else kNoSlot
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
  if (b0 + 16u <= nl) {
    __builtin_amdgcn_raw_buffer_store_b128(v, ors, (int)(o_off + b0), 0, kAux);
  } else if (b0 < nl) {
    // The partial last chunk, r = 1..15 bytes: its whole dwords in one
    // b32/b64/b96 store, then a b16 and/or b8 for the trailing bytes.  With
    // a wave-uniform frame length only one of the paths below is issued.
    const uint32_t r = nl - b0, d = r >> 2, tb = r & 3u, o = o_off + b0;
    if (d == 3u) {
      __builtin_amdgcn_raw_buffer_store_b96(u32x3{v[0], v[1], v[2]}, ors, (int)o, 0, kAux);
    } else if (d == 2u) {
      __builtin_amdgcn_raw_buffer_store_b64(u32x2{v[0], v[1]}, ors, (int)o, 0, kAux);
    } else if (d == 1u) {
      __builtin_amdgcn_raw_buffer_store_b32(v[0], ors, (int)o, 0, kAux);
    }
    if (tb != 0u) {
      const uint32_t w = d == 0u ? v[0] : (d == 1u ? v[1] : (d == 2u ? v[2] : v[3]));
      const uint32_t ob = o + 4u * d;
      if (tb >= 2u) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)w, ors, (int)ob, 0, kAux);
      if (tb & 1u) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(w >> (8u * (tb & 2u))), ors,
                                                       (int)(ob + (tb & 2u)), 0, kAux);
    }
  }
}

// Output byte b of the rewritten frame comes from input byte b (Ethernet,
// chunks 0-1), from the header record, or from input byte b + 20 (6to4) /
// b - 20 (4to6) (the TCP segment, chunks >= 2).  A group of kFG = 16 lanes
// owns a frame; lane g owns output chunks c = 16q + g.
constexpr uint32_t kHdrC4 = 4u, kHdrC6 = 5u;  // chunks holding header words / patches
constexpr uint32_t kHold4 = 3u, kHold6 = 4u;  // chunk holding the TCP checksum field

// Output chunk c of frame f, its 16 bytes o as taken from the input: patch
// the header dwords, add the TCP span bytes to acc, store it (or keep it in
// `held` if it carries the checksum field).
template <bool TO4, bool FAST>
__device__ __forceinline__ void chunk_out(const Nat64Args &a, rsrc_t ors, const FrameRec &f,
                                          uint32_t c, u32x4 o, uint32_t &acc, u32x4 &held) {
  constexpr uint32_t kHdrC = TO4 ? kHdrC4 : kHdrC6;
  constexpr uint32_t kHold = TO4 ? kHold4 : kHold6;
  constexpr int kSpanR = TO4 ? 8 : 13;  // first TCP dword (its high half)
  const uint32_t k = f.info & 3u, port_be = swap16(f.info >> 16), nl = f.new_len;
  if (16u * c >= nl) return;
  if (c < kHdrC) {
#pragma unroll
    for (uint32_t t = 0; t < 4u; ++t) {
      const int r = (int)(4u * c + t) - (int)k;
      const uint32_t d = out_dword<TO4>(r, o[t], f.V, port_be);
      uint32_t m = r < kSpanR ? 0u : (r == kSpanR ? 0xffff0000u : 0xffffffffu);
      m &= range_mask(16u * c + 4u * t, 0u, nl);
      acc = sad16(d & m, acc);
      o[t] = d;
    }
  } else {
    acc = sad16(o[3], sad16(o[2], sad16(o[1], sad16(o[0], acc))));
    if (16u * c + 16u > nl) {  // bytes past the end of the frame
#pragma unroll
      for (uint32_t t = 0; t < 4u; ++t) {
        const uint32_t x = o[t] & ~range_mask(16u * c + 4u * t, 0u, nl);
        acc -= (x & 0xffffu) + (x >> 16);
      }
    }
  }
  if (c == kHold) held = o;
  else store_chunk<FAST>(ors, a.out_arena, f.o_off, c, o, nl);
}

// The group's TCP sum, the checksum (v4 or v6 pseudo-header) into the held
// chunk, and its store by the lane that owns it.
template <bool TO4, bool FAST>
__device__ __forceinline__ void finish_frame(const Nat64Args &a, rsrc_t ors, const FrameRec &f,
                                             uint32_t g, uint32_t acc, u32x4 held) {
  constexpr uint32_t kHold = TO4 ? kHold4 : kHold6;
  const uint32_t k = f.info & 3u, nl = f.new_len;
#pragma unroll
  for (uint32_t d = kFG / 2; d > 0; d >>= 1) acc += __shfl_xor(acc, d, kFG);
  if (g != kHold % kFG) return;
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
  if (TO4 && f.defer_i != kNoSlot) a.stash_c0[f.defer_i] = tcp_c | (k << 16);
  const uint32_t tw = TO4 ? k : k + 1u;  // dword of the checksum field in the held chunk
#pragma unroll
  for (uint32_t t = 0; t < 4u; ++t)
    if (t == tw) held[t] |= swap16(tcp_c) << 16;
  store_chunk<FAST>(ors, a.out_arena, f.o_off, kHold, held, nl);
}

// Input position of output chunk c (16 input bytes at the shifted position).
template <bool TO4>
__device__ __forceinline__ uint32_t chunk_src(uint32_t in_off, uint32_t c) {
  return c < 2u ? in_off + 16u * c : (TO4 ? in_off + 16u * c + 20u : in_off + 16u * c - 20u);
}

// A group of kFG lanes rewrites frame f; lane g owns output chunks
// c = 16q + kFG j + g (interleaved: each load instruction covers whole 64-B
// pieces of kBlock / kFG frames).  FAST (wave-uniform): every frame of the
// wave is dword-aligned on both sides and well inside both arenas, so loads
// and full-chunk stores are branch-free (an unneeded chunk gets an offset
// past num_records: zero load, dropped store).  PRE: the pass-0 chunks were
// loaded by the caller (FAST only).
template <bool TO4, bool FAST, bool PRE>
__device__ __forceinline__ void rewrite_frame(const Nat64Args &a, rsrc_t rs, rsrc_t ors, uint32_t g,
                                              const FrameRec &f, bool in_al_wave,
                                              const u32x4 (&pre)[kFJ]) {
  const uint32_t nl = f.new_len;
  uint32_t acc = 0;
  u32x4 held = {0u, 0u, 0u, 0u};
  for (uint32_t q = 0; 256u * q < nl; ++q) {
    u32x4 o[kFJ];
#pragma unroll
    for (uint32_t j = 0; j < kFJ; ++j) {
      const uint32_t c = 16u * q + kFG * j + g;
      const bool need = 16u * c < nl;
      if (PRE && q == 0u) {
        o[j] = pre[j];
      } else if (FAST) {
        o[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(need ? chunk_src<TO4>(f.in_off, c) : kNoRead), 0, kAux);
      } else {
        o[j] = u32x4{0u, 0u, 0u, 0u};
        if (need) o[j] = load_in(rs, a.arena_len, chunk_src<TO4>(f.in_off, c), in_al_wave);
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < kFJ; ++j) chunk_out<TO4, FAST>(a, ors, f, 16u * q + kFG * j + g, o[j], acc, held);
  }
  finish_frame<TO4, FAST>(a, ors, f, g, acc, held);
}

// ---- fused kernels: one 4-lane quad per frame -----------------------------
// Lane g of the quad owns output chunks c = 16q + 4j + g.  The quad issues
// its frame's pass-0 loads (4 x 16 B per lane, at the shifted input
// positions) together with the header chunks 0..3 (and lane 0: chunk 4),
// unshifted, which hit the same lines; the header dwords reach every lane of
// the quad by DPP quad broadcasts; every lane classifies (the work is 4x
// redundant, but no LDS, no barrier, and a frame's bytes are read while its
// lines are hot); lane 0 probes the port map; then the quad rewrites.

// Lane K of each quad, to all four lanes (DPP quad_perm [K, K, K, K]).
template <int K>
__device__ __forceinline__ uint32_t qbc(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, K * 0x55, 0xf, 0xf, true);
}

// Header chunk g (lanes 0..3) and, in lane 0, chunk 4: frame bytes 0..79.
__device__ __forceinline__ void header_loads(rsrc_t rs, uint32_t arena_len, uint32_t off, uint32_t g,
                                             bool valid, bool hdr_fast, bool al_wave, u32x4 &Y,
                                             u32x4 &Y4) {
  Y = u32x4{0u, 0u, 0u, 0u};
  Y4 = u32x4{0u, 0u, 0u, 0u};
  if (hdr_fast) {
    Y = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(valid ? off + 16u * g : kNoRead), 0, kAux);
    Y4 = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(valid && g == 0u ? off + 64u : kNoRead), 0, kAux);
  } else if (valid) {
    Y = load_in(rs, arena_len, off + 16u * g, al_wave);
    if (g == 0u) Y4 = load_in(rs, arena_len, off + 64u, al_wave);
  }
}

// Frame dwords P[3..16] (bytes 12..67) in every lane of the quad.
__device__ __forceinline__ void gather_header(u32x4 Y, u32x4 Y4, uint32_t (&P)[20]) {
#pragma unroll
  for (int j = 0; j < 20; ++j) P[j] = 0u;
  P[3] = qbc<0>(Y[3]);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    P[4 + t] = qbc<1>(Y[t]);
    P[8 + t] = qbc<2>(Y[t]);
    P[12 + t] = qbc<3>(Y[t]);
  }
  P[16] = qbc<0>(Y4[0]);
}

// Pass-0 chunk loads of the quad's frame (FAST only; zero otherwise).
template <bool TO4>
__device__ __forceinline__ void pass0_loads(rsrc_t rs, uint32_t off, uint32_t nl, uint32_t g, bool fast,
                                            u32x4 (&X)[kFJ]) {
#pragma unroll
  for (uint32_t j = 0; j < kFJ; ++j) {
    const uint32_t c = kFG * j + g;
    X[j] = u32x4{0u, 0u, 0u, 0u};
    if (fast) X[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(16u * c < nl ? chunk_src<TO4>(off, c) : kNoRead), 0, kAux);
  }
}

// One quad's frame descriptor for a round and the wave-uniform load modes.
struct QuadDesc {
  uint32_t i, off, len, o_off, nl;
  bool valid, fast, hdr_fast, al_wave;
};

// TO4: 6to4 (an Act frame has 74 <= len, new length len - 20); else 4to6
// (54 <= len < 2028, new length len + 20).
template <bool TO4>
__device__ __forceinline__ QuadDesc quad_desc(const Nat64Args &a, uint32_t i) {
  QuadDesc d;
  d.i = i;
  d.valid = i < a.n;
  d.off = d.valid ? a.off[i] : 0u;
  d.len = d.valid ? (uint32_t)a.len[i] : 0u;
  d.o_off = d.valid ? a.out_off[i] : 0u;
  return d;
}

template <bool TO4>
__device__ __forceinline__ void quad_modes(const Nat64Args &a, QuadDesc &d) {
  const bool cand = TO4 ? (d.valid && d.len >= 74u) : (d.valid && d.len >= 54u && d.len < a.room - 20u);
  d.nl = cand ? (TO4 ? d.len - 20u : d.len + 20u) : 0u;
  d.fast = !__ballot(cand && !((d.off & 3u) == 0u && (d.o_off & 3u) == 0u &&
                               (uint64_t)d.off + d.nl + 64u <= (uint64_t)a.arena_len &&
                               (uint64_t)d.o_off + d.nl + 16u <= (uint64_t)a.out_arena_len));
  d.hdr_fast = !__ballot(d.valid && ((d.off & 3u) != 0u || (uint64_t)d.off + 80u > (uint64_t)a.arena_len));
  d.al_wave = !__ballot(d.valid && (d.off & 3u) != 0u);
}

// ---- realignment within the quad ---------------------------------------------
// 20 bytes = one chunk + one dword, so when the input frame is 16-B aligned
// every output chunk c >= 2 is three dwords of one aligned input chunk and
// one dword of its neighbour, which another lane of the quad loaded:
//   6to4: out c = {in(c+1).y, .z, .w, in(c+2).x}: lane g loads in(c+1) and
//         takes in(c+2).x from lane g+1 (lane 3: from lane 0's next chunk);
//   4to6: out c = {in(c-2).w, in(c-1).x, .y, .z}: lane g loads in(c-1) and
//         takes in(c-2).w from lane g-1 (lane 0: lane 3's previous chunk).
// Chunks 0 and 1 are the input's own.  Aligned loads cost one 16-B piece of
// one line each; the shifted ones straddled two (measured 134 vs 92 us for
// the bare copy of 1 M 256-B frames).
template <int CTRL>
__device__ __forceinline__ uint32_t qdpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, true);
}
constexpr int kQNext = 1 | (2 << 2) | (3 << 4) | (0 << 6);  // lane g <- lane (g + 1) % 4
constexpr int kQPrev = 3 | (0 << 2) | (1 << 4) | (2 << 6);  // lane g <- lane (g + 3) % 4

template <bool TO4>
__device__ __forceinline__ uint32_t aligned_src(uint32_t in_off, uint32_t c) {
  if (c < 2u) return in_off + 16u * c;
  return TO4 ? in_off + 16u * (c + 1u) : in_off + 16u * (c - 1u);
}

// Pass q's aligned loads A[j] (chunk c = 16q + 4j + g) and, 6to4, lane 3's
// extra dword E = in(16q + 17).x for output chunk 16q + 15.
template <bool TO4>
__device__ __forceinline__ void aligned_loads(rsrc_t rs, uint32_t in_off, uint32_t nl, uint32_t q,
                                              uint32_t g, u32x4 (&A)[kFJ], uint32_t &E) {
#pragma unroll
  for (uint32_t j = 0; j < kFJ; ++j) {
    const uint32_t c = 16u * q + kFG * j + g;
    // 6to4: chunk c's load also serves output chunk c - 1's last dword
    const bool need = TO4 ? 16u * c < nl + 4u : 16u * c < nl;
    A[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(need ? aligned_src<TO4>(in_off, c) : kNoRead), 0, kAux);
  }
  E = 0u;
  if (TO4) {
    const uint32_t c = 16u * q + 15u;
    E = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(g == 3u && 16u * c < nl ? in_off + 16u * (c + 2u) : kNoRead), 0, kAux);
  }
}

// The shifted chunks X[j] of pass q from the aligned loads.  carry (4to6):
// lane 3's A[3].w of the previous pass, as seen by lane 0.
template <bool TO4>
__device__ __forceinline__ void realign(const u32x4 (&A)[kFJ], uint32_t E, uint32_t q, uint32_t g,
                                        uint32_t &carry, u32x4 (&X)[kFJ]) {
#pragma unroll
  for (uint32_t j = 0; j < kFJ; ++j) {
    if (TO4) {
      const uint32_t n1 = qdpp<kQNext>(A[j][0]);
      const uint32_t n2 = j + 1 < kFJ ? qdpp<kQNext>(A[j + 1 < kFJ ? j + 1 : j][0]) : E;
      const uint32_t nx = g == 3u ? n2 : n1;
      X[j] = (q == 0u && j == 0u && g < 2u) ? A[j] : u32x4{A[j][1], A[j][2], A[j][3], nx};
    } else {
      const uint32_t p1 = qdpp<kQPrev>(A[j][3]);
      const uint32_t p0 = j > 0 ? qdpp<kQPrev>(A[j > 0 ? j - 1 : 0][3]) : carry;
      uint32_t pw = g == 0u ? p0 : p1;
      if (q == 0u && j == 0u) {
        const uint32_t c0w = qbc<0>(A[0][3]);  // in(0).w for output chunk 2
        if (g == 2u) pw = c0w;
      }
      X[j] = (q == 0u && j == 0u && g < 2u) ? A[j] : u32x4{pw, A[j][0], A[j][1], A[j][2]};
    }
  }
  if (!TO4) carry = qdpp<kQPrev>(A[kFJ - 1][3]);  // lane 0 <- lane 3's last chunk
}

// rewrite_frame for a 16-B-aligned input frame: aligned loads + realign.
// Pass 0's loads were issued by the caller (A0, E0).
template <bool TO4>
__device__ __forceinline__ void rewrite_frame_al(const Nat64Args &a, rsrc_t rs, rsrc_t ors, uint32_t g,
                                                 const FrameRec &f, const u32x4 (&A0)[kFJ], uint32_t E0) {
  const uint32_t nl = f.new_len;
  uint32_t acc = 0, carry = 0;
  u32x4 held = {0u, 0u, 0u, 0u};
  u32x4 X[kFJ];
  realign<TO4>(A0, E0, 0u, g, carry, X);
#pragma unroll
  for (uint32_t j = 0; j < kFJ; ++j) chunk_out<TO4, true>(a, ors, f, kFG * j + g, X[j], acc, held);
  for (uint32_t q = 1; 256u * q < nl; ++q) {  // frames longer than 256 B
    u32x4 A[kFJ];
    uint32_t E;
    aligned_loads<TO4>(rs, f.in_off, nl, q, g, A, E);
    realign<TO4>(A, E, q, g, carry, X);
#pragma unroll
    for (uint32_t j = 0; j < kFJ; ++j) chunk_out<TO4, true>(a, ors, f, 16u * q + kFG * j + g, X[j], acc, held);
  }
  finish_frame<TO4, true>(a, ors, f, g, acc, held);
}

// The quad's frame: aligned (16-B input, FAST), FAST (shifted loads issued
// early) or general; the pass-0 loads go out with the header loads.
template <bool TO4>
__device__ __forceinline__ void issue_frame_loads(rsrc_t rs, const QuadDesc &d, uint32_t g, bool al16,
                                                  u32x4 (&X)[kFJ], uint32_t &E) {
  E = 0u;
  if (al16) aligned_loads<TO4>(rs, d.off, d.nl, 0u, g, X, E);
  else pass0_loads<TO4>(rs, d.off, d.nl, g, d.fast, X);
}

template <bool TO4>
__device__ __forceinline__ void rewrite_quad(const Nat64Args &a, rsrc_t rs, rsrc_t ors, uint32_t g,
                                             const QuadDesc &d, bool al16, const FrameRec &f,
                                             const u32x4 (&X)[kFJ], uint32_t E) {
  if (al16) rewrite_frame_al<TO4>(a, rs, ors, g, f, X, E);
  else if (d.fast) rewrite_frame<TO4, true, true>(a, rs, ors, g, f, true, X);
  else rewrite_frame<TO4, false, false>(a, rs, ors, g, f, d.al_wave, X);
}

// Count the wave's deferred frames (flag set in their lane), one atomic per
// wave: the tail kernel returns at once when the count is 0.
// Flag that the batch has deferred frames (the tail returns at once
// without).  A plain store of 1 by one lane of each such wave: an atomic add
// on one word from every wave of a cold batch (32 k waves) serialized at
// that word's memory-side atomic unit, about 90 adds per us, and took the
// fused kernel from 110 to 400 us; plain stores of the same value merge in
// the XCDs' L2s and reach memory at the kernel boundary.
__device__ __forceinline__ void defer_append(const Nat64Args &a, uint32_t lane, bool flag,
                                             uint32_t i) {
  (void)i;
  const uint64_t dm = __ballot(flag);
  if (!dm) return;
  if (lane == (uint32_t)__builtin_ctzll(dm)) a.pm.state[4u + a.par] = 1u;
}

// The general path: one quad per frame (any alignment, any length); `i` is
// the quad's frame, lane the wave lane.
__device__ __forceinline__ void quad_6to4(const Nat64Args &a, rsrc_t rs, rsrc_t ors, uint32_t i,
                                          uint32_t lane) {
  const uint32_t g = lane & (kFG - 1u);
  QuadDesc d = quad_desc<true>(a, i);
  quad_modes<true>(a, d);
  const bool al16 = d.fast && !__ballot(d.nl != 0u && (d.off & 15u) != 0u);
  u32x4 X[kFJ], Y, Y4;
  uint32_t E;
  issue_frame_loads<true>(rs, d, g, al16, X, E);
  header_loads(rs, a.arena_len, d.off, g, d.valid, d.hdr_fast, d.al_wave, Y, Y4);
  uint32_t P[20];
  gather_header(Y, Y4, P);
  V6 v;
  classify_dwords(P, d.len, a.room, v);
  // assigned_port (main.rs:41-53): lane 0 of the quad probes the table
  uint32_t slot = kNoSlot, port = 0xffffffffu;
  if (d.valid && g == 0u && v.disp == CGPU_ACT) {
    slot = probe_port(a, d.i, v, port);
  }
  slot = qbc<0>(slot);
  port = qbc<0>(port);
  if (v.disp == CGPU_ACT && slot == kNoSlot) {
    v.disp = CGPU_ABORT;
    v.st = CGPU_PKT_TABLE_FULL;
  }
  const bool act = d.valid && v.disp == CGPU_ACT;
  uint32_t H[5];
  ipv4_header(v, d.len, H);
  const bool now = act && port != 0xffffffffu;  // committed key: its port is known
  const bool deferred = act && !now;            // new key: its port needs the batch order (tail)
  if (d.valid && g == 0u) {
    a.out_len[d.i] = act ? (uint16_t)d.nl : 0;
    a.pkt_slot[d.i] = now ? kNoSlot : slot;
    a.disposition[d.i] = (uint8_t)v.disp;
    a.status[d.i] = (uint8_t)v.st;
  }
  defer_append(a, lane, deferred && g == 0u, d.i);
  if (act) {  // a deferred frame is written with source port 0; the tail patches it
    FrameRec f;
    f.in_off = d.off;
    f.o_off = d.o_off;
    f.new_len = d.nl;
    f.info = v.k | kNow | ((now ? port : 0u) << 16);
#pragma unroll
    for (int j = 0; j < 5; ++j) f.V[j] = H[j];
#pragma unroll
    for (int j = 5; j < 10; ++j) f.V[j] = 0u;
    f.ph = 0u;
    f.defer_i = deferred ? d.i : kNoSlot;
    rewrite_quad<true>(a, rs, ors, g, d, al16, f, X, E);
  }
}

// ---- the rows path: F frames per wave ---------------------------------------
// When every frame of a wave is 16-B aligned in the input, dword-aligned in
// the output and at most 256 B long (one input pass), the wave moves its frames in rows of 16 lanes, four
// whole frames per load and store instruction (full lines), and decides per
// frame in one lane:
//   A. row j loads frame 4r + j in round r, lane l its 16-B chunk l; the
//      rows pass bytes 0..95 of every frame through wave-private LDS to the
//      frame's own lane, which classifies its frame, probes the port map
//      (the probe's latency hides behind the row loads) and builds output
//      bytes 0..63 (Ethernet, the IPv4 header, the start of the rewritten TCP
//      header) and their part of the TCP sum into a wave-private LDS record;
//   B. the payload moved by 20 B (in(l+1).yzw and in(l+2).x by DPP row
//      shifts) and its TCP sum (a DPP row reduction), while the port-map
//      probes are in flight; then row j writes frame 4r + j in one store
//      instruction (whole lines): lanes 0-3 the chunks built in A, lanes
//      4-14 the payload, lane 3 with the TCP checksum patched in.
// Wave-uniform specialisations: no VLAN tag in the wave (static header
// layout), one output length for the wave (per-lane chunk masks computed
// once).
constexpr uint32_t kRowW = 20;  // LDS dwords per frame record
constexpr uint32_t kRowFrames = 32;  // frames per wave (64: 152 us, 3 waves per SIMD)

template <int CTRL>
__device__ __forceinline__ uint32_t dppz(uint32_t v) {  // lanes without a source get 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, true);
}
constexpr int kRowShl1 = 0x101, kRowShl2 = 0x102;
constexpr int kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118;

// Record layout (dwords of the frame's LDS slot, written in phase A):
//   0..15  output bytes 0..63 (TCP checksum field zero)
//   16     output length if the frame is finished here, else 0
//   17     TCP sum (LE words) of the span bytes among output bytes 0..63
//          (after A5: the whole span's sum)
//   18     v4 pseudo-header sum | VLAN depth << 16 (after A5: the finished
//          TCP checksum field | VLAN depth << 16)
//   19     output offset
// FULL: every Act frame of the wave has at least 64 output bytes (no byte
// mask at the output length within bytes 0..63; the bench's frames, and any
// TCP frame with 10 B of payload or more).
template <bool K0, bool FULL>
__device__ __forceinline__ void rows_build(const uint32_t (&D)[24], const uint32_t (&H)[10],
                                           uint32_t k, uint32_t port_be, uint32_t nl,
                                           uint32_t (&O)[16], uint32_t &acc) {
  acc = 0;
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    const int r = w - (K0 ? 0 : (int)k);
    const uint32_t x = w < 8 ? D[w] : D[w + 5];  // output bytes >= 32: input + 20
    const uint32_t d = out_dword<true>(r, x, H, port_be);
    uint32_t m = r < 8 ? 0u : (r == 8 ? 0xffff0000u : 0xffffffffu);
    if (!FULL) m &= range_mask(4u * (uint32_t)w, 0u, nl);
    acc = sad16(d & m, acc);
    O[w] = d;
  }
}

// Row-path cache policy of the frame loads and of the whole-row stores: the
// default (nontemporal, aux 2, was slower: DESIGN.md §3.2)
constexpr int kRowAux = 0;    // whole-row stores of 6to4's packed output (partial lines: default)
constexpr int kRowLdAux = 2;  // frame loads: nontemporal (whole lines per instruction)
// 4to6 writes its frames into 256-B slots, a whole slot per row store:
// nontemporal, so the output stream does not push ADDR_MAP's lines out of
// the L2 (round 5, A/B on one box: 99.3 -> 90.3 us, reads 313 -> 283 MB)
constexpr int kRow46StAux = 2;

// B1: the payload of every round -- output chunks 4.. realigned in place
// (X[r] becomes output chunk l of frame 4r + row) and their TCP sum, reduced
// over the row into lane 15, which leaves it in the frame's record (rec[17]).
// Needs only the frames' lengths, not the port map, so it runs while the
// probes are in flight.
template <bool UNI>
__device__ __forceinline__ void rows_payload(u32x4 (&X)[kRowFrames / 4], uint32_t *lds, uint32_t row,
                                             uint32_t l, uint32_t nl0) {
  // UNI: every ACT frame of the wave has output length nl0, so this lane's
  // byte masks are the same in every round
  u32x4 M0;
#pragma unroll
  for (uint32_t t = 0; t < 4u; ++t) M0[t] = range_mask(16u * l + 4u * t, 0u, nl0);
#pragma unroll
  for (uint32_t r = 0; r < kRowFrames / 4u; ++r) {
    uint32_t *fr = lds + (4u * r + row) * kRowW;
    const uint32_t fnl = fr[16];
    if (!__ballot(fnl != 0u)) continue;  // no ACT frame in this round
    const u32x4 A = X[r];
    u32x4 o;
    o[0] = dppz<kRowShl1>(A[1]);
    o[1] = dppz<kRowShl1>(A[2]);
    o[2] = dppz<kRowShl1>(A[3]);
    o[3] = dppz<kRowShl2>(A[0]);
    uint32_t acc = 0;
    if (l >= 4u) {
#pragma unroll
      for (uint32_t t = 0; t < 4u; ++t)
        acc = sad16(o[t] & (UNI ? M0[t] : range_mask(16u * l + 4u * t, 0u, fnl)), acc);
    }
    acc += dppz<kRowShr1>(acc);
    acc += dppz<kRowShr2>(acc);
    acc += dppz<kRowShr4>(acc);
    acc += dppz<kRowShr8>(acc);
    if (l == 15u) fr[17] = acc;
    X[r] = o;
  }
}

// B2: row j writes frame 4r + j in one store instruction (whole lines):
// lanes 0-3 the chunks built in A, lanes 4.. the realigned payload; lane 3
// patches the TCP checksum into its chunk.  The chunk of lane l of frame
// 4r + row, as stored.
__device__ __forceinline__ u32x4 rows_chunk(const u32x4 (&X)[kRowFrames / 4], const uint32_t *fr, uint32_t r,
                                            uint32_t l, const u32x4 &meta) {
  const u32x4 hc = *reinterpret_cast<const u32x4 *>(fr + 4u * (l & 3u));
  u32x4 o = l < 4u ? hc : X[r];
  if (l == 3u) {  // the checksum, finished by the frame's own lane in A5
    const uint32_t fk = meta[2] >> 16, tcp_c = meta[2] & 0xffffu;
#pragma unroll
    for (uint32_t t = 0; t < 4u; ++t)
      if (t == fk) o[t] |= swap16(tcp_c) << 16;
  }
  return o;
}

__device__ __forceinline__ void rows_store(const Nat64Args &a, rsrc_t ors, const u32x4 (&X)[kRowFrames / 4],
                                           const uint32_t *lds, uint32_t row, uint32_t l) {
#pragma unroll
  for (uint32_t r = 0; r < kRowFrames / 4u; ++r) {
    const uint32_t *fr = lds + (4u * r + row) * kRowW;
    const u32x4 meta = *reinterpret_cast<const u32x4 *>(fr + 16);
    const uint32_t fnl = meta[0];
    if (!__ballot(fnl != 0u)) continue;  // no frame of this round is finished here
    const u32x4 o = rows_chunk(X, fr, r, l, meta);
    if (fnl != 0u) {
      const uint32_t b0 = 16u * l;
      if (b0 + 16u <= fnl) __builtin_amdgcn_raw_buffer_store_b128(o, ors, (int)(meta[3] + b0), 0, kRowAux);
      else if (b0 < fnl) store_chunk<true>(ors, a.out_arena, meta[3], l, o, fnl);
    }
  }
}

// B2 for a wave whose 32 frames are all Act and packed back to back in the
// output (out_off[f + 1] = out_off[f] + new length, lengths multiples of 4:
// the bench's egress image, a TX ring): each half of the wave (16 frames,
// at most 3,776 B) is assembled in wave-private LDS by the rows and then
// stored linearly, 1 KiB per instruction.  The stage holds the half's bytes
// at their output address modulo 16 (stage dword 0 is the 16-B chunk the
// half starts in), so a lane reads each whole output chunk with one aligned
// 16-B LDS read; only the half's first and last chunks are masked.  The
// 128-B lines that lie wholly inside the half's span are stored nontemporal
// (whole lines: the output stream then does not push the port map's probe
// lines out of the L2, as whole-slot nontemporal stores did for 4to6); the
// half's two boundary lines, which the neighbouring half or wave also
// writes, keep the default policy.
constexpr uint32_t kStageDw = 16u * 236u / 4u + 8u;  // one half-wave's output + alignment, dwords
constexpr int kStageNT = 2;

__device__ __forceinline__ void rows_store_staged(rsrc_t ors, const u32x4 (&X)[kRowFrames / 4], const uint32_t *lds,
                                                  uint32_t *stage, uint32_t row, uint32_t l, uint32_t lane) {
#pragma unroll
  for (uint32_t h = 0; h < 2u; ++h) {
    const uint32_t S = lds[16u * h * kRowW + 19u];  // the half's first frame's output offset
    const uint32_t *lr = lds + (16u * h + 15u) * kRowW;
    const uint32_t E = lr[19] + lr[16];  // its last frame's end
    const uint32_t A = S & ~15u;         // the chunk the half starts in: stage dword 0
#pragma unroll
    for (uint32_t rr = 0; rr < 4u; ++rr) {
      const uint32_t r = 4u * h + rr;
      const uint32_t *fr = lds + (4u * r + row) * kRowW;
      const u32x4 meta = *reinterpret_cast<const u32x4 *>(fr + 16);
      const u32x4 o = rows_chunk(X, fr, r, l, meta);
      const uint32_t d0 = (meta[3] - A) / 4u + 4u * l;  // the chunk's first dword in the stage
#pragma unroll
      for (uint32_t t = 0; t < 4u; ++t)
        if (16u * l + 4u * t < meta[0]) stage[d0 + t] = o[t];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const uint32_t nch = (E - A + 15u) >> 4;
    for (uint32_t c = lane; c < nch; c += 64u) {
      const uint32_t g = A + 16u * c;
      const u32x4 v = *reinterpret_cast<const u32x4 *>(stage + 4u * c);
      if (g >= S && g + 16u <= E) {
        const uint32_t line = g & ~127u;
        if (line >= S && line + 128u <= E)
          __builtin_amdgcn_raw_buffer_store_b128(v, ors, (int)g, 0, kStageNT);
        else
          __builtin_amdgcn_raw_buffer_store_b128(v, ors, (int)g, 0, 0);
      } else {  // the half's first or last chunk: its bytes in [S, E) only
#pragma unroll
        for (uint32_t t = 0; t < 4u; ++t) {
          const uint32_t b = g + 4u * t;
          if (b >= S && b < E) __builtin_amdgcn_raw_buffer_store_b32(v[t], ors, (int)b, 0, 0);
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
}

__device__ __forceinline__ bool rows_6to4(const Nat64Args &a, rsrc_t rs, rsrc_t ors, uint32_t base,
                                          uint32_t lane, uint32_t *lds, uint32_t *stage) {
  constexpr uint32_t R = kRowFrames / 4u;  // rounds
  const uint32_t i = base + lane;
  const bool mine = lane < kRowFrames;
  const bool valid = mine && i < a.n;
  const uint32_t off = valid ? a.off[i] : 0u;
  const uint32_t len = valid ? (uint32_t)a.len[i] : 0u;
  const uint32_t o_off = valid ? a.out_off[i] : 0u;
  // 16-B aligned input (aligned loads, DPP realignment), dword-aligned output
  // (b128 stores at any dword: packed output frames stay on this path)
  if (__ballot(valid && ((off & 15u) != 0u || (o_off & 3u) != 0u || len > 256u))) return false;
  const uint32_t row = lane >> 4, l = lane & 15u;
  uint32_t D[24];
  // A2: the frames in rows, four whole frames per load instruction; in
  // flight while the headers are classified and the port map is probed
  u32x4 X[R];
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t f = 4u * r + row;
    const uint32_t fo = __shfl(off, (int)f), fl = __shfl(len, (int)f);
    X[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(16u * l < fl ? fo + 16u * l : kNoRead), 0, kRowLdAux);
  }
  // A1: bytes 0..95 of every frame from its row, through wave-private LDS
  // (the record area, not yet in use) to the frame's own lane: no strided
  // per-lane loads of the header lines the rows have just fetched
#pragma unroll
  for (uint32_t r = 0; r < R; ++r)
    if (l < 6u) *reinterpret_cast<u32x4 *>(lds + (4u * r + row) * 24u + 4u * l) = X[r];
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
  for (uint32_t m = 0; m < 6u; ++m) {
    const u32x4 t = *reinterpret_cast<const u32x4 *>(lds + (mine ? lane : 0u) * 24u + 4u * m);
    D[4 * m] = t[0]; D[4 * m + 1] = t[1]; D[4 * m + 2] = t[2]; D[4 * m + 3] = t[3];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  uint32_t *rec = lds + (mine ? lane : 0u) * kRowW;
  // A3: the reference control flow; the first port-map slot of the key is
  // loaded now and examined after B1
  uint32_t P[20];
#pragma unroll
  for (int j = 0; j < 20; ++j) P[j] = D[j];
  V6 v;
  const uint32_t mk = be16_lo(P[3]);
  if (!__ballot(mine && (mk == 0x8100u || mk == 0x88a8u))) classify_dwords<true>(P, len, a.room, v);
  else classify_dwords<false>(P, len, a.room, v);
  const bool act0 = valid && v.disp == CGPU_ACT;
  uint32_t key[5];
  make_key(v, key);
  const uint32_t h = key_hash(key, a.pm) & a.pm.cap_mask;
  u32x4 s0 = {0u, 0u, 0u, 0u}, s1 = {0u, 0u, 0u, 0u};
  if (act0) {
    const u32x4 *sp = reinterpret_cast<const u32x4 *>(&a.pm.slots[h]);
    s0 = sp[0];
    s1 = sp[1];
  }
  const uint32_t nl = len - 20u;  // meaningful for ACT frames
  if (mine) {
    rec[16] = act0 ? nl : 0u;
    rec[19] = o_off;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // B1: realign and sum the payload of every round (port-independent)
  const uint32_t nl0 = __shfl(nl, (int)(__builtin_ctzll(__ballot(act0) | (1ull << 63))));
  if (!__ballot(act0 && nl != nl0)) rows_payload<true>(X, lds, row, l, nl0);
  else rows_payload<false>(X, lds, row, l, nl0);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // A4: assigned_port (main.rs:41-53), the IPv4 header
  uint32_t slot = kNoSlot, port = 0xffffffffu;
  if (act0) {
    slot = probe_port_at(a, i, key, h, s0, s1, port);
  }
  if (v.disp == CGPU_ACT && slot == kNoSlot) {
    v.disp = CGPU_ABORT;
    v.st = CGPU_PKT_TABLE_FULL;
  }
  const bool act = valid && v.disp == CGPU_ACT;
  uint32_t H[10];
  ipv4_header(v, len, reinterpret_cast<uint32_t(&)[5]>(H));
#pragma unroll
  for (int j = 5; j < 10; ++j) H[j] = 0u;
  const bool now = act && port != 0xffffffffu;
  const bool deferred = act && !now;
  // pkt_slot only where the wave has a deferred frame (the tail reads the
  // wave's flag first): the steady state writes none
  const bool wdef = __ballot(deferred) != 0ull;
  if (valid) {
    a.out_len[i] = act ? (uint16_t)nl : 0;
    if (wdef) a.pkt_slot[i] = now ? kNoSlot : slot;
    a.disposition[i] = (uint8_t)v.disp;
    a.status[i] = (uint8_t)v.st;
  }
  if (lane == 0u) a.wave_flag[base / kRowFrames] = wdef ? 1u : 0u;
  defer_append(a, lane, deferred, i);
  // A5: output bytes 0..63 and their share of the TCP sum; the record.  A
  // deferred frame is written with source port 0 (the tail patches the port
  // and the checksum once the batch order has assigned it).
  const uint32_t k = v.k, port_be = now ? swap16(port & 0xffffu) : 0u;
  uint32_t O[16], accA;
  const bool k0 = !__ballot(act && k != 0u), full = !__ballot(act && nl < 64u);
  if (k0 && full) rows_build<true, true>(D, H, k, port_be, nl, O, accA);
  else if (k0) rows_build<true, false>(D, H, k, port_be, nl, O, accA);
  else rows_build<false, false>(D, H, k, port_be, nl, O, accA);
  const uint32_t span = (nl - (34u + 4u * k)) & 0xffffu;
  const uint32_t dst = be32(H[4]);
  const uint32_t ph = fold32(0xcb00u + 0x7101u + (dst >> 16) + (dst & 0xffffu) + 6u + span);
  if (mine) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
      *reinterpret_cast<u32x4 *>(rec + 4 * m) = u32x4{O[4 * m], O[4 * m + 1], O[4 * m + 2], O[4 * m + 3]};
    const uint32_t payload = rec[17];
    // the TCP checksum field (a deferred frame's with port 0, stashed with
    // its VLAN depth for the tail), once per frame rather than per row store
    const uint32_t c0k = ((~fold32(ph + swap16(fold32(payload + accA)))) & 0xffffu) | (k << 16);
    *reinterpret_cast<u32x4 *>(rec + 16) = u32x4{act ? nl : 0u, payload + accA, c0k, o_off};
    if (deferred) a.stash_c0[i] = c0k;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // the staged store: every frame of the wave Act, the outputs tiling one
  // span in frame order (dword lengths)
  const uint32_t nxt = __shfl_down(o_off, 1);
  const bool untiled = mine && (!act || (nl & 3u) != 0u || (lane + 1u < kRowFrames && nxt != o_off + nl));
  if (!__ballot(untiled)) rows_store_staged(ors, X, lds, stage, row, l, lane);
  else rows_store(a, ors, X, lds, row, l);
  return true;
}

__global__ __launch_bounds__(kBlock) NAT64_OCC void nat64_6to4_fused(Nat64Args a) {
  __shared__ uint32_t lds[kBlock / 64][kRowFrames * (kRowW > 24u ? kRowW : 24u)];
  __shared__ __attribute__((aligned(16))) uint32_t stage[kBlock / 64][kStageDw];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t base = (blockIdx.x * (kBlock / 64u) + wave) * kRowFrames;
  if (base >= a.n) return;  // wave-uniform
  const rsrc_t rs = make_rsrc(a.arena, a.arena_len);
  const rsrc_t ors = make_rsrc(a.out_arena, a.out_arena_len);
  if (rows_6to4(a, rs, ors, base, lane, lds[wave], stage[wave])) return;
  // the general path: rounds of 16 frames, a quad per frame (every frame's
  // pkt_slot written)
  for (uint32_t q = 0; q < kRowFrames / 16u; ++q) quad_6to4(a, rs, ors, base + 16u * q + lane / 4u, lane);
  if (lane == 0u) a.wave_flag[base / kRowFrames] = 1u;
}

// ---- the tail: order the batch's new keys, finish their frames --------------
// The batch's keys first seen in it get NEXT_PORT + (rank of their first
// packet among the first packets of all new keys): AtomicU16::fetch_add in
// the reference's packet order (main.rs:45-51).  The fused kernel left each
// such key's first packet index in its slot (w[7], by atomicMin), each
// deferred packet's slot in pkt_slot, and the key of each packet that
// joined a slot on its claim tag alone in the stash.  Two launches of nb
// workgroups (nb = chunks of kBlock packets), one chunk each:
//   nat64_tail_order     each tag-joined packet's key is compared with its
//                        slot's key words (a tag collision is listed for the
//                        repair below), and the packets that are a new key's
//                        first packet (w[7] == i) give a 256-bit mask and a
//                        count per chunk; the workgroup that arrives last
//                        (arrivals counted in 32 shards of their own lines,
//                        then one counter: an atomic on one word serializes
//                        at its memory-side unit, ~90 per us) repairs any
//                        collisions, scans the counts into each chunk's
//                        base ordinal and advances NEXT_PORT;
//   nat64_tail_patch     every deferred packet computes its key's port from
//                        the first packet's chunk base and mask -- no hand-off
//                        between packets of one key -- and patches its frame
//                        (the fused kernel wrote it with source port 0); a
//                        first packet also commits the key (port, kPersist,
//                        ADDR_MAP).
// Both are grid-stride loops over the chunks on grids of at most kOrderGrid
// / kPatchGrid workgroups (in the steady state each workgroup only reads the
// flag and returns: 1.5-1.9 us per launch on the stream, nearly independent
// of the grid up to 1024 workgroups, tools/launch_gap.hip).  Inside
// nat64_tail_order, the counts and the collision list are stored sc1,
// drained before the arrival atomics and loaded sc1 by the last workgroup
// (MI355X_MICROARCH.md, inter-workgroup visibility: the last arriver, told
// by its add); everything else crosses a launch boundary.  The arrivals are
// counted per XCD (blockIdx % 8 under round-robin placement, a speed choice
// only), on counters 4 KiB apart, then the XCD counts on one: atomics on one
// line, and on lines 128 B apart, serialized at ~13 ns each (4096
// workgroups arriving on 32 counters 128 B apart took 48 us).
// state (line 0): [0] NEXT_PORT [1] entries [4+p] the batch has deferred
// frames (p = call parity; the previous call's flag is cleared by this
// call's order launch).  The arrival counters, the collision count and the
// port base live in the scratch (TailCtl), zeroed again by the last arriver.
__device__ __forceinline__ void st_sc1(uint32_t *p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t *p) {
  return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t add_agent(uint32_t *p, uint32_t v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The tail's control words in the scratch: 8 arrival shards 4 KiB apart,
// then a line with the shard-completion counter, the collision count and
// the port base.
constexpr uint32_t kShards = 8u, kShardW = 1024u;
constexpr uint32_t kOrderGrid = 1024u, kPatchGrid = 1024u;  // patch 4096 -> 1024: steady 110.7 -> 110.0 us, cold unchanged (round 5)
struct TailCtl {
  uint32_t *shard;  // [kShards * kShardW]: shard s counts at shard[s * kShardW]
  uint32_t *top;    // [0] shards complete, [1] collisions, [2] port base
};
__device__ __forceinline__ TailCtl tail_ctl(const Nat64Args &a) {
  return TailCtl{a.ctl, a.ctl + kShards * kShardW};
}

// Whether packet i's stashed key is its slot's key (w = the slot's words).
__device__ __forceinline__ bool stash_matches(const Nat64Args &a, uint32_t i, const uint32_t *w) {
  const u32x4 k = a.stash_key[i];
  return k[0] == w[2] && k[1] == w[3] && k[2] == w[4] && k[3] == w[5] &&
         (uint32_t)a.stash_port[i] == (w[6] & 0xffffu);
}

// Packet i's pkt_slot entry as the fused kernel left it: a wave without a
// deferred frame skips the stores and clears its flag (its entries are
// stale from an earlier call).
__device__ __forceinline__ uint32_t pkt_slot_of(const Nat64Args &a, uint32_t i) {
  return a.wave_flag[i / kRowFrames] ? a.pkt_slot[i] : kNoSlot;
}
// The same inside the repair, which rewrites entries (thread 0) that the
// workgroup's other threads then read: at the coherence point.
__device__ __forceinline__ uint32_t pkt_slot_sc1(const Nat64Args &a, uint32_t i) {
  return a.wave_flag[i / kRowFrames] ? ld_sc1(&a.pkt_slot[i]) : kNoSlot;
}

// One chunk's first packets (all kBlock threads): the mask words and the
// count, sc1.  Tag-joined packets whose key is not their slot's (collisions)
// go to the list `mism` (sc1 entries, counted in ctl.top[1]); they are never
// a first packet here.
__device__ __forceinline__ void chunk_firsts(const Nat64Args &a, uint32_t c, bool verify,
                                             uint32_t *cnt, uint32_t *cmask, uint32_t *mism,
                                             const TailCtl &ctl) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t i = c * kBlock + threadIdx.x;
  const uint32_t ps = i < a.n ? pkt_slot_sc1(a, i) : kNoSlot;
  const bool loc = ps != kNoSlot && (ps & kLocalBit);
  bool bad = false, f = false;
  if (loc) {
    const uint32_t *w = a.pm.slots[ps & kSlotMask].w;
    if (verify && !(ps & kClaimBit)) bad = !stash_matches(a, i, w);
    // w[7] as the repair left it, at the coherence point (its atomics)
    f = !bad && ld_sc1(&w[7]) == i;
  }
  const uint64_t m = __ballot(f);
  if (lane == 0) {
    st_sc1(&cmask[8u * c + 2u * wave], (uint32_t)m);
    st_sc1(&cmask[8u * c + 2u * wave + 1u], (uint32_t)(m >> 32));
  }
  const uint64_t bm = __ballot(bad);
  if (bm) {  // rare: list the wave's collisions
    const uint32_t first = (uint32_t)__builtin_ctzll(bm);
    uint32_t at = 0;
    if (lane == first) at = add_agent(&ctl.top[1], (uint32_t)__popcll(bm));
    at = __shfl(at, (int)first);
    if (bad) st_sc1(&mism[at + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull))], i);
  }
  const uint32_t n_first = (uint32_t)__syncthreads_count(f);
  if (threadIdx.x == 0) st_sc1(&cnt[c], n_first);
}

// kOrderU chunks per workgroup (c0 + j * stride): every load of the U chunks
// is issued before the first compare, so a workgroup waits on one chain of
// dependent loads (pkt_slot -> slot) instead of U; the counts per wave go
// through LDS (s_wc), one barrier for the U chunks.
constexpr uint32_t kOrderU = 4;
__device__ __forceinline__ void chunks_firsts(const Nat64Args &a, uint32_t c0, uint32_t stride,
                                              uint32_t nb, uint32_t *cnt, uint32_t *cmask,
                                              uint32_t *mism, const TailCtl &ctl,
                                              uint32_t (*s_wc)[kBlock / 64]) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t ps[kOrderU], w7[kOrderU];
  bool bad[kOrderU];
#pragma unroll
  for (uint32_t j = 0; j < kOrderU; ++j) {
    const uint32_t c = c0 + j * stride, i = c * kBlock + threadIdx.x;
    ps[j] = c < nb && i < a.n ? pkt_slot_of(a, i) : kNoSlot;
  }
#pragma unroll
  for (uint32_t j = 0; j < kOrderU; ++j) {
    const uint32_t i = (c0 + j * stride) * kBlock + threadIdx.x;
    w7[j] = kNoSlot;
    bad[j] = false;
    if (ps[j] != kNoSlot && (ps[j] & kLocalBit)) {
      // the slot in two 16-B loads (w[2..7]: key words and first packet):
      // a gather costs per instruction and per line, not per byte
      const u32x4 *sp = reinterpret_cast<const u32x4 *>(&a.pm.slots[ps[j] & kSlotMask]);
      const u32x4 s1 = sp[1];
      w7[j] = s1[3];
      if (!(ps[j] & kClaimBit)) {
        const u32x4 s0 = sp[0];
        const u32x4 k = a.stash_key[i];
        bad[j] = k[0] != s0[2] || k[1] != s0[3] || k[2] != s1[0] || k[3] != s1[1] ||
                 (uint32_t)a.stash_port[i] != (s1[2] & 0xffffu);
      }
    }
  }
#pragma unroll
  for (uint32_t j = 0; j < kOrderU; ++j) {
    const uint32_t c = c0 + j * stride, i = c * kBlock + threadIdx.x;
    const bool f = !bad[j] && w7[j] == i;
    const uint64_t m = __ballot(f);
    if (lane == 0 && c < nb) {
      st_sc1(&cmask[8u * c + 2u * wave], (uint32_t)m);
      st_sc1(&cmask[8u * c + 2u * wave + 1u], (uint32_t)(m >> 32));
      s_wc[j][wave] = (uint32_t)__popcll(m);
    }
    const uint64_t bm = __ballot(bad[j]);
    if (bm) {  // rare: list the wave's collisions
      const uint32_t first = (uint32_t)__builtin_ctzll(bm);
      uint32_t at = 0;
      if (lane == first) at = add_agent(&ctl.top[1], (uint32_t)__popcll(bm));
      at = __shfl(at, (int)first);
      if (bad[j]) st_sc1(&mism[at + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull))], i);
    }
  }
  __syncthreads();
  if (threadIdx.x < kOrderU) {
    const uint32_t c = c0 + threadIdx.x * stride;
    uint32_t t = 0;
#pragma unroll
    for (uint32_t w = 0; w < kBlock / 64u; ++w) t += s_wc[threadIdx.x][w];
    if (c < nb) st_sc1(&cnt[c], t);
  }
  __syncthreads();  // s_wc is reused
}

// The repair of tag collisions (rare: distinct keys whose claim tags are
// equal met in a probe chain), by the last arriver: each listed packet looks
// its key up exactly (its slot's key words were written by the fused kernel;
// slots this repair claims, by this workgroup) and joins that slot or claims
// a new one; the first packet of every slot a colliding packet had joined is
// recomputed (a collision may have lowered it), and the chunks whose first
// packets may have changed are counted again.  The patch launch reads the
// result behind the launch boundary.
constexpr uint32_t kRepairSet = 256;  // wrong slots per pass
__device__ void tail_repair(const Nat64Args &a, uint32_t nb, uint32_t nmism, const uint32_t *mism,
                            uint32_t *cnt, uint32_t *cmask, const TailCtl &ctl) {
  __shared__ uint32_t s_slot[kRepairSet], s_min[kRepairSet], s_chunk[4 * kRepairSet];
  __shared__ uint32_t s_ns, s_nc, s_all;
  if (threadIdx.x == 0) {
    s_ns = 0u;
    s_nc = 0u;
    s_all = 0u;
  }
  __syncthreads();
  // 1. the listed packets, one by one (thread 0): exact lookups
  if (threadIdx.x == 0) {
    auto add_chunk = [&](uint32_t pkt) {
      if (pkt >= a.n) return;  // (no packet: nothing to count again)
      const uint32_t ch = pkt / kBlock;
      for (uint32_t q = 0; q < s_nc; ++q)
        if (s_chunk[q] == ch) return;
      if (s_nc < 4u * kRepairSet) s_chunk[s_nc++] = ch;
      else s_all = 1u;
    };
    for (uint32_t q = 0; q < nmism; ++q) {
      const uint32_t m = ld_sc1(&mism[q]);
      const uint32_t wrong = a.pkt_slot[m] & kSlotMask;
      uint32_t k = 0;
      for (; k < s_ns; ++k)
        if (s_slot[k] == wrong) break;
      if (k == s_ns) {
        if (s_ns < kRepairSet) {
          s_slot[s_ns] = wrong;
          s_min[s_ns] = 0xffffffffu;
          ++s_ns;
        } else {
          s_all = 1u;  // more wrong slots than a pass holds: recount every chunk
        }
      }
      add_chunk(m);
      add_chunk(a.pm.slots[wrong].w[7]);  // the wrong slot's first packet so far
      const u32x4 sk = a.stash_key[m];
      const uint32_t key[5] = {sk[0], sk[1], sk[2], sk[3], (uint32_t)a.stash_port[m]};
      uint32_t h = key_hash(key, a.pm) & a.pm.cap_mask, res = kNoSlot;
      for (uint32_t probe = 0; probe <= a.pm.cap_mask; ++probe, h = (h + 1u) & a.pm.cap_mask) {
        uint32_t *w = a.pm.slots[h].w;
        const uint32_t other[5] = {w[2], w[3], w[4], w[5], w[6] & 0xffffu};
        if (w[0] == 0u) {  // a new key after all: claim it
          w[1] = key_tag(key, a.pm) & a.pm.tag_mask;
          w[2] = key[0];
          w[3] = key[1];
          w[4] = key[2];
          w[5] = key[3];
          w[6] = key[4];
          w[7] = m;
          w[0] = m + 1u;
          res = h | kLocalBit | kClaimBit;
          break;
        }
        if (!key_eq(key, other)) continue;
        if (w[0] & kPersist) {  // a committed key: its port (the frame is patched with it)
          res = h | kPatchBit;
        } else {
          add_chunk(w[7]);
          if (m < w[7]) w[7] = m;
          res = h | kLocalBit;
        }
        break;
      }
      if (res == kNoSlot) {  // no room: the packet aborts (TABLE_FULL)
        a.disposition[m] = CGPU_ABORT;
        a.status[m] = CGPU_PKT_TABLE_FULL;
        a.out_len[m] = 0;
      }
      a.pkt_slot[m] = res;
    }
  }
  __syncthreads();
  // 2. the first packet of each slot a collision had joined: the minimum
  // over the packets that belong to it now.  More such slots than the set
  // holds (s_all): the first packet of every slot of the batch is computed
  // again, from all packets (a slot outside the set would otherwise keep a
  // first packet that has moved to another slot, and its key no port).
  const uint32_t ns = s_ns;
  if (s_all) {
    for (uint32_t i = threadIdx.x; i < a.n; i += kBlock) {
      const uint32_t ps = pkt_slot_sc1(a, i);
      if (ps != kNoSlot && (ps & kLocalBit)) st_sc1(&a.pm.slots[ps & kSlotMask].w[7], 0xffffffffu);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < a.n; i += kBlock) {
      const uint32_t ps = pkt_slot_sc1(a, i);
      if (ps != kNoSlot && (ps & kLocalBit)) atomicMin(&a.pm.slots[ps & kSlotMask].w[7], i);
    }
    __builtin_amdgcn_s_waitcnt(0);
  } else {
    for (uint32_t i = threadIdx.x; i < a.n; i += kBlock) {
      const uint32_t ps = pkt_slot_of(a, i);
      if (ps == kNoSlot || !(ps & kLocalBit)) continue;
      const uint32_t sl = ps & kSlotMask;
      for (uint32_t k = 0; k < ns; ++k)
        if (s_slot[k] == sl) atomicMin(&s_min[k], i);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && !s_all)
    for (uint32_t k = 0; k < ns; ++k) {
      a.pm.slots[s_slot[k]].w[7] = s_min[k];
      const uint32_t ch = s_min[k] / kBlock;
      bool have = false;
      for (uint32_t q = 0; q < s_nc; ++q) have |= s_chunk[q] == ch;
      if (!have && s_min[k] < a.n) {
        if (s_nc < 4u * kRepairSet) s_chunk[s_nc++] = ch;
        else s_all = 1u;
      }
    }
  __syncthreads();
  // 3. count the affected chunks again (every chunk when the sets overflowed)
  const uint32_t nc = s_all ? nb : s_nc;
  for (uint32_t q = 0; q < nc; ++q) {
    const uint32_t c = s_all ? q : s_chunk[q];  // < nb (add_chunk keeps packets < n)
    chunk_firsts(a, c, false, cnt, cmask, nullptr, ctl);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
}

// The last arriver: exclusive scan of the chunk counts into the chunk bases
// (read by the patch launch), the port base, NEXT_PORT advanced (AtomicU16
// wrap), and the control words zeroed for the next call.
__device__ __forceinline__ void tail_scan(const Nat64Args &a, uint32_t nb, const uint32_t *cnt,
                                          uint32_t *cbase, const TailCtl &ctl, uint32_t *s_part) {
  uint32_t *const st = a.pm.state;
  const uint32_t per = (nb + kBlock - 1u) / kBlock;
  const uint32_t b0 = threadIdx.x * per, b1 = b0 + per < nb ? b0 + per : nb;
  // Up to 16 counts per thread (1 Mi packets) are read at once, 16 B per
  // sc1 load (aux 16), and kept in registers for the second pass: atomic
  // loads one after the other were a round trip each, 6.8 us.
  constexpr uint32_t kReg = 16;
  uint32_t v[kReg];
  uint32_t sum = 0;
  const bool reg = per <= kReg;
  if (reg) {
    const rsrc_t rc = make_rsrc(cnt, 4u * nb);  // counts past nb read as 0
#pragma unroll
    for (uint32_t q = 0; q < kReg / 4u; ++q) {
      const u32x4 t = 4u * q < per ? __builtin_amdgcn_raw_buffer_load_b128(rc, (int)(4u * (b0 + 4u * q)), 0, 16)
                                   : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
      for (uint32_t j = 0; j < 4u; ++j) v[4u * q + j] = 4u * q + j < per && b0 + 4u * q + j < nb ? t[j] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < kReg; ++j) sum += v[j];
  } else {
    for (uint32_t b = b0; b < b1; ++b) sum += ld_sc1(&cnt[b]);
  }
  // exclusive scan of the 256 partial sums: within each wave by shuffles,
  // then the four wave totals
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t incl = sum;
#pragma unroll
  for (uint32_t d = 1; d < 64u; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d);
    if (lane >= d) incl += y;
  }
  if (lane == 63u) s_part[wave] = incl;
  __syncthreads();
  uint32_t run = incl - sum, total = 0;
#pragma unroll
  for (uint32_t w = 0; w < kBlock / 64u; ++w) {
    if (w < wave) run += s_part[w];
    total += s_part[w];
  }
  if (reg) {
#pragma unroll
    for (uint32_t j = 0; j < kReg; ++j) {
      if (b0 + j < b1) cbase[b0 + j] = run;
      run += v[j];
    }
  } else {
    for (uint32_t b = b0; b < b1; ++b) {
      const uint32_t c = ld_sc1(&cnt[b]);
      cbase[b] = run;
      run += c;
    }
  }
  if (threadIdx.x < kShards) ctl.shard[threadIdx.x * kShardW] = 0u;
  if (threadIdx.x == 0) {
    const uint32_t base = st[0];
    ctl.top[0] = 0u;
    ctl.top[1] = 0u;
    ctl.top[2] = base;
    st[0] = (base + total) & 0xffffu;  // read by the next call's launches
    st[1] += total;
  }
}


__device__ __forceinline__ uint32_t shard_size(uint32_t grid, uint32_t s) {
  return s < grid ? (grid - s + kShards - 1u) / kShards : 0u;
}

__global__ __launch_bounds__(kBlock) void nat64_tail_order(Nat64Args a, uint32_t nb) {
  __shared__ uint32_t s_last, s_nm;
  __shared__ uint32_t s_part[kBlock / 64];
  __shared__ uint32_t s_wc[kOrderU][kBlock / 64];
  uint32_t *const st = a.pm.state;
  // the previous call's flag, cleared only if set: in the steady state the
  // flag line is never written, so every workgroup's read of it can hit
  if (blockIdx.x == 0 && threadIdx.x == 0 && st[4u + (a.par ^ 1u)] != 0u) st[4u + (a.par ^ 1u)] = 0u;
  if (st[4u + a.par] == 0u) return;  // nothing deferred: no new key
  uint32_t *const cnt = a.chunks, *const cbase = a.chunks + nb, *const cmask = a.chunks + 2u * nb;
  uint32_t *const mism = a.chunks + 10u * nb;  // the tag collisions (packet indices)
  const TailCtl ctl = tail_ctl(a);
  for (uint32_t c0 = blockIdx.x; c0 < nb; c0 += kOrderU * gridDim.x)
    chunks_firsts(a, c0, gridDim.x, nb, cnt, cmask, mism, ctl, s_wc);
  __builtin_amdgcn_s_waitcnt(0);  // every storing wave drains before the arrival
  __syncthreads();
  if (threadIdx.x == 0) {
    // arrival: the workgroup's shard, then (its last arriver) the shard count
    const uint32_t s = blockIdx.x % kShards, g = gridDim.x;
    bool last = false;
    if (add_agent(&ctl.shard[s * kShardW], 1u) == shard_size(g, s) - 1u) {
      const uint32_t used = g < kShards ? g : kShards;
      last = add_agent(&ctl.top[0], 1u) == used - 1u;
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  if (threadIdx.x == 0) s_nm = atomicCAS(&ctl.top[1], 0u, 0u);  // the collisions, read at the coherence point
  __syncthreads();
  if (s_nm) tail_repair(a, nb, s_nm, mism, cnt, cmask, ctl);
  tail_scan(a, nb, cnt, cbase, ctl, s_part);
}

// One deferred packet: its key's port, the commit of a first packet, and
// the frame's port and checksum.
__device__ __forceinline__ void patch_packet(const Nat64Args &a, uint32_t i, uint32_t ps,
                                             uint32_t o_off, uint32_t ck, uint32_t port_base, const uint32_t *cbase,
                                             const uint32_t *cmask) {
  uint32_t *w = a.pm.slots[ps & kSlotMask].w;
  uint32_t port;
  if (ps & kLocalBit) {
    const uint32_t fi = w[7];  // the key's first packet
    const uint32_t fc = fi / kBlock, fb = fi % kBlock;
    const u32x4 m0 = *reinterpret_cast<const u32x4 *>(cmask + 8u * fc);
    const u32x4 m1 = *reinterpret_cast<const u32x4 *>(cmask + 8u * fc + 4u);
    const uint32_t mw[8] = {m0[0], m0[1], m0[2], m0[3], m1[0], m1[1], m1[2], m1[3]};
    uint32_t below = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8u; ++j) {
      const uint32_t lo = 32u * j;
      below += (uint32_t)__builtin_popcount(fb >= lo + 32u ? mw[j] : (fb > lo ? mw[j] & ((1u << (fb - lo)) - 1u) : 0u));
    }
    const uint32_t ordinal = cbase[fc] + below;
    port = (port_base + ordinal) & 0xffffu;  // NEXT_PORT.fetch_add order
    if (fi == i) {
      const uint32_t kw[5] = {w[2], w[3], w[4], w[5], w[6]};
      // ADDR_MAP.insert_new(port, key) (main.rs:50): the first mapping of a
      // port wins, also after NEXT_PORT wraps.  This call's ordinals o and
      // o + 65536k share a port, so only its first lap (o < 65536) can be
      // first, and only if no earlier call mapped the port: one writer per
      // entry, no race.
      uint32_t *e = a.pm.rev + 5u * port;
      if (ordinal < 65536u && !(e[4] & kRevValid)) {
#pragma unroll
        for (int j = 0; j < 4; ++j) e[j] = kw[j];
        e[4] = (kw[4] & 0xffffu) | kRevValid;
      }
      // PORT_MAP.insert_new (main.rs:49): the key, committed for later batches
      w[6] = (kw[4] & 0xffffu) | (port << 16);
      w[0] = kPersist;
    }
  } else {  // (repair) a committed key found for a colliding packet
    port = w[6] >> 16;
  }
  // The fused kernel wrote the frame with source port 0 and stashed that
  // frame's checksum c0 and VLAN depth; set the port and patch the checksum,
  // ~fold(~c0 + port) -- exact: the sum behind c0 includes the
  // pseudo-header's protocol 6, so it is never 0 and ~c0 recovers its fold
  // (DESIGN.md §3.3).  Only the 4 bytes are touched: the frame is not read.
  const uint32_t c0 = ck & 0xffffu, k = ck >> 16;
  const uint32_t c = (~fold32(((~c0) & 0xffffu) + port)) & 0xffffu;
  // (the fused kernel wrote the frame and its stash: k <= 2, the TCP header
  // inside the output arena; checked all the same, a bad stash must not
  // turn into a stray store)
  if (k > 2u || (uint64_t)o_off + 52u + 4u * k > a.out_arena_len) return;
  uint8_t *tcp = a.out_arena + o_off + 34u + 4u * k;  // the TCP header
  if (!((o_off + 34u) & 1u)) {  // (packed 6to4 output: even) two 16-bit stores
    *reinterpret_cast<uint16_t *>(tcp) = (uint16_t)swap16(port);
    *reinterpret_cast<uint16_t *>(tcp + 16) = (uint16_t)swap16(c);
  } else {
    tcp[0] = (uint8_t)(port >> 8);
    tcp[1] = (uint8_t)port;
    tcp[16] = (uint8_t)(c >> 8);
    tcp[17] = (uint8_t)c;
  }
}

__global__ __launch_bounds__(kBlock) void nat64_tail_patch(Nat64Args a, uint32_t nb) {
  if (a.pm.state[4u + a.par] == 0u) return;  // nothing deferred: no new key
  const uint32_t *const cbase = a.chunks + nb, *const cmask = a.chunks + 2u * nb;
  const uint32_t port_base = tail_ctl(a).top[2];
  for (uint32_t c = blockIdx.x; c < nb; c += gridDim.x) {
    const uint32_t i = c * kBlock + threadIdx.x;
    if (i >= a.n) break;
    // loaded together: the slot reference, the frame's place and its stash
    const uint32_t ps = pkt_slot_of(a, i), o_off = a.out_off[i], ck = a.stash_c0[i];
    if (ps != kNoSlot && (ps & (kLocalBit | kPatchBit))) patch_packet(a, i, ps, o_off, ck, port_base, cbase, cmask);
  }
}

// ============================ 4to6 direction =================================
// Classify, look the TCP destination port up in ADDR_MAP (rev[port]: the v6
// key itself, one 20-B entry), build the
// IPv6 header, then the quad
// rewrite with the input shifted by -20 bytes behind the 40-byte header (the
// TCP checksum field, output bytes 70+4k, is in chunk 4).
// 4to6 classification of one frame (main.rs:86-118) up to the ADDR_MAP
// lookup: disposition, status, VLAN depth, the TCP destination port, and
// the L3-relative dwords L[0..5].
struct V4 {
  uint32_t k, eth_len, disp, st, gw_port;
  uint32_t L[6];
};

__device__ __forceinline__ void classify4(const uint32_t (&P)[20], uint32_t len, V4 &v) {
  const uint32_t marker = be16_lo(P[3]);
  v.k = marker == 0x8100u ? 1u : (marker == 0x88a8u ? 2u : 0u);
  v.eth_len = 14u + 4u * v.k;
  const uint32_t et = be16_lo(sel3(v.k, P[3], P[4], P[5]));
  uint32_t A[8];  // L3-relative dwords 0..6 (IPv4 header, TCP ports)
#pragma unroll
  for (int j = 0; j < 8; ++j) A[j] = __builtin_amdgcn_alignbyte(P[4 + j], P[3 + j], 2);
#pragma unroll
  for (int j = 0; j < 6; ++j) v.L[j] = sel3(v.k, A[j], j + 1 < 8 ? A[j + 1] : 0u, j + 2 < 8 ? A[j + 2] : 0u);
  v.disp = CGPU_ABORT;
  v.gw_port = 0u;
  if (len == 0u) v.st = CGPU_PKT_ETH_BAD_OFFSET;                 // parse::<Ethernet>()?
  else if (len < v.eth_len) v.st = CGPU_PKT_ETH_OUT_OF_BUFFER;
  else if (et != 0x0800u) v.st = CGPU_PKT_NOT_IPV4;              // parse::<Ipv4>()?
  else if (v.eth_len >= len) v.st = CGPU_PKT_L3_BAD_OFFSET;
  else if (v.eth_len + 20u > len) v.st = CGPU_PKT_L3_OUT_OF_BUFFER;
  else {
    v.st = CGPU_PKT_OK;
    v.disp = CGPU_DROP;
    const uint32_t flags_frag = be16_hi(v.L[1]);  // flags/fragment offset: L3 bytes 6-7
    const uint32_t proto = (v.L[2] >> 8) & 0xffu;
    if (proto == 6u && (flags_frag & 0x1fffu) == 0u && !(flags_frag & 0x2000u)) {
      const uint32_t tcp_off = v.eth_len + 20u;
      if (tcp_off >= len) { v.st = CGPU_PKT_L4_BAD_OFFSET; v.disp = CGPU_ABORT; }   // peek::<Tcp4>()?
      else if (tcp_off + 20u > len) { v.st = CGPU_PKT_L4_OUT_OF_BUFFER; v.disp = CGPU_ABORT; }
      else {
        v.gw_port = be16_hi(v.L[5]);  // TCP destination port (L3 bytes 22-23)
        v.disp = CGPU_ACT;            // pending the ADDR_MAP lookup
      }
    }
  }
}

// ADDR_MAP[port]: the v6 address and the port word (| kRevValid), one 20-B
// entry read as a dwordx4 and a dword (buffer loads: any dword alignment)
__device__ __forceinline__ void rev_read(const PortMapDev &pm, uint32_t port, u32x4 &addr,
                                         uint32_t &rport) {
  const rsrc_t rr = make_rsrc(pm.rev, 65536u * 20u);
  addr = __builtin_amdgcn_raw_buffer_load_b128(rr, (int)(20u * port), 0, 0);
  rport = __builtin_amdgcn_raw_buffer_load_b32(rr, (int)(20u * port + 16u), 0, 0);
}

// The IPv6 header of a 4to6 frame (Ipv6Header::default + set_dscp / ecn /
// next_header / hop_limit / src / dst, main.rs:92-105; payload_length by
// Ipv6::reconcile, v6/mod.rs:331-334) as 10 LE dwords, from its IPv4
// classification and its ADDR_MAP value (the original v6 source address
// s0); ph = the LE residue of the pseudo-header's address words.
__device__ __forceinline__ void ipv6_header(const V4 &v, uint32_t nl, u32x4 s0, uint32_t (&V)[10],
                                            uint32_t &ph) {
  const uint32_t de = (v.L[0] >> 8) & 0xffu;            // dscp_ecn (v4.rs:186-203)
  const uint32_t dscp = de >> 2, ecn = de & 3u;
  const uint32_t hop = ((v.L[2] & 0xffu) - 1u) & 0xffu;  // ttl - 1 (u8, wrapping)
  const uint32_t w = (6u << 28) | ((dscp << 22) & 0x0fc00000u) | ((ecn << 20) & 0x00300000u);
  V[0] = be32(w);
  V[1] = swap16((nl - v.eth_len - 40u) & 0xffffu) | (6u << 16) | (hop << 24);
  V[2] = 0x9bff6400u;  // 64:ff9b::/96 (map4to6, main.rs:62-74)
  V[3] = 0u;
  V[4] = 0u;
  V[5] = v.L[3];       // v4 source address
  V[6] = s0[0];        // the ADDR_MAP value: the original v6 source
  V[7] = s0[1];
  V[8] = s0[2];
  V[9] = s0[3];
  uint32_t x = sad16(V[2], 0u);
  x = sad16(V[5], x);
  x = sad16(s0[0], sad16(s0[1], sad16(s0[2], sad16(s0[3], x))));
  ph = fold32(x);
}

// assigned_addr(port) (main.rs:56-58) and the push's tailroom check for a
// frame the classification left ACT: ADDR_MAP holds the value (the port
// word: the v6-side port and the valid bit).
__device__ __forceinline__ void addr_map_check(const Nat64Args &a, uint32_t len, uint32_t rport, V4 &v) {
  if (!(rport & kRevValid)) {
    v.disp = CGPU_DROP;  // no mapping: Either::Drop
  } else if (len >= a.room - 20u) {  // push::<Ipv6>(): extend 40 needs 40 < tailroom
    v.st = CGPU_PKT_NOT_RESIZED;
    v.disp = CGPU_ABORT;
  }
}

// ---- 4to6 rows path -----------------------------------------------------------
// The 6to4 rows design mirrored: every frame of the wave 16-B aligned in the
// input, dword-aligned in the output and at most 236 B long (output at most
// 256 B, one row pass).  Row j loads frame 4r + j in round r, four whole
// frames per load instruction; bytes 0..95 reach the frame's own lane through
// LDS, which classifies it by nat_4to6's control flow, reads its ADDR_MAP
// entry (issued here, examined after B1) and builds output bytes 0..79
// (Ethernet, the IPv6 header, the TCP header with the original port, the
// checksum field zero) into an LDS record.  B1: output chunk l >= 5 is
// in(l-2).w, in(l-1).xyz (DPP row shifts right: the frame grows by 20 B
// behind the new header) and its TCP sum a DPP row reduction.  B2: row j
// stores frame 4r + j in one instruction; lanes 0-4 take the record, lane 4
// with the TCP checksum patched in (output bytes 70 + 4k).
constexpr uint32_t kRowW6 = 24;  // LDS dwords per 4to6 record: output bytes 0..79 + 4 meta

// Output dwords 0..19 of the rewritten frame (header-relative r = w - k)
// and the TCP sum (LE words) of the span bytes among them.
template <bool K0>
__device__ __forceinline__ void rows_build6(const uint32_t (&D)[24], const uint32_t (&V)[10],
                                            uint32_t k, uint32_t port_be, uint32_t nl,
                                            uint32_t (&O)[20], uint32_t &acc) {
  acc = 0;
#pragma unroll
  for (int w = 0; w < 20; ++w) {
    const int r = w - (K0 ? 0 : (int)k);
    const uint32_t x = w < 8 ? D[w] : D[w - 5];  // output bytes >= 32: input - 20
    const uint32_t d = out_dword<false>(r, x, V, port_be);
    uint32_t m = r < 13 ? 0u : (r == 13 ? 0xffff0000u : 0xffffffffu);
    m &= range_mask(4u * (uint32_t)w, 0u, nl);
    acc = sad16(d & m, acc);
    O[w] = d;
  }
}

// B1 (4to6): output chunks 5.. from the row's input chunks, and their sum.
template <bool UNI>
__device__ __forceinline__ void rows_payload6(u32x4 (&X)[kRowFrames / 4], uint32_t *lds, uint32_t row,
                                              uint32_t l, uint32_t nl0) {
  u32x4 M0;
#pragma unroll
  for (uint32_t t = 0; t < 4u; ++t) M0[t] = range_mask(16u * l + 4u * t, 0u, nl0);
#pragma unroll
  for (uint32_t r = 0; r < kRowFrames / 4u; ++r) {
    uint32_t *fr = lds + (4u * r + row) * kRowW6;
    const uint32_t fnl = fr[20];
    if (!__ballot(fnl != 0u)) continue;  // no ACT frame in this round
    const u32x4 A = X[r];
    u32x4 o;
    o[0] = dppz<kRowShr2>(A[3]);
    o[1] = dppz<kRowShr1>(A[0]);
    o[2] = dppz<kRowShr1>(A[1]);
    o[3] = dppz<kRowShr1>(A[2]);
    uint32_t acc = 0;
    if (l >= 5u) {
#pragma unroll
      for (uint32_t t = 0; t < 4u; ++t)
        acc = sad16(o[t] & (UNI ? M0[t] : range_mask(16u * l + 4u * t, 0u, fnl)), acc);
    }
    acc += dppz<kRowShr1>(acc);
    acc += dppz<kRowShr2>(acc);
    acc += dppz<kRowShr4>(acc);
    acc += dppz<kRowShr8>(acc);
    if (l == 15u) fr[21] = acc;
    X[r] = o;
  }
}

// B2 (4to6): lanes 0-4 the record's chunks, lanes 5.. the payload; lane 4
// patches the checksum (record meta: fnl, TCP sum, fph_be | k << 16, o_off).
__device__ __forceinline__ void rows_store6(const Nat64Args &a, rsrc_t ors, const u32x4 (&X)[kRowFrames / 4],
                                            const uint32_t *lds, uint32_t row, uint32_t l) {
#pragma unroll
  for (uint32_t r = 0; r < kRowFrames / 4u; ++r) {
    const uint32_t *fr = lds + (4u * r + row) * kRowW6;
    const u32x4 meta = *reinterpret_cast<const u32x4 *>(fr + 20);
    const uint32_t fnl = meta[0];
    if (!__ballot(fnl != 0u)) continue;
    const u32x4 hc = *reinterpret_cast<const u32x4 *>(fr + 4u * (l < 5u ? l : 0u));
    u32x4 o = l < 5u ? hc : X[r];
    if (l == 4u) {  // the checksum, finished by the frame's own lane in A5
      const uint32_t fk = meta[2] >> 16, tcp_c = meta[2] & 0xffffu;
#pragma unroll
      for (uint32_t t = 0; t < 4u; ++t)
        if (t == fk + 1u) o[t] |= swap16(tcp_c) << 16;
    }
    if (fnl != 0u) {
      const uint32_t b0 = 16u * l;
      if (b0 + 16u <= fnl) __builtin_amdgcn_raw_buffer_store_b128(o, ors, (int)(meta[3] + b0), 0, kRow46StAux);
      else if (b0 < fnl) store_chunk<true>(ors, a.out_arena, meta[3], l, o, fnl);
    }
  }
}

__device__ __forceinline__ bool rows_4to6(const Nat64Args &a, rsrc_t rs, rsrc_t ors, uint32_t base,
                                          uint32_t lane, uint32_t *lds) {
  constexpr uint32_t R = kRowFrames / 4u;  // rounds
  const uint32_t i = base + lane;
  const bool mine = lane < kRowFrames;
  const bool valid = mine && i < a.n;
  const uint32_t off = valid ? a.off[i] : 0u;
  const uint32_t len = valid ? (uint32_t)a.len[i] : 0u;
  const uint32_t o_off = valid ? a.out_off[i] : 0u;
  if (__ballot(valid && ((off & 15u) != 0u || (o_off & 3u) != 0u || len > 236u))) return false;
  const uint32_t row = lane >> 4, l = lane & 15u;
  // A2: the frames in rows, four whole frames per load instruction
  u32x4 X[R];
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t f = 4u * r + row;
    const uint32_t fo = __shfl(off, (int)f), fl = __shfl(len, (int)f);
    X[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(16u * l < fl ? fo + 16u * l : kNoRead), 0, kRowLdAux);
  }
  // A1: bytes 0..95 of every frame, through LDS to the frame's own lane
  uint32_t D[24];
#pragma unroll
  for (uint32_t r = 0; r < R; ++r)
    if (l < 6u) *reinterpret_cast<u32x4 *>(lds + (4u * r + row) * 24u + 4u * l) = X[r];
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
  for (uint32_t m = 0; m < 6u; ++m) {
    const u32x4 t = *reinterpret_cast<const u32x4 *>(lds + (mine ? lane : 0u) * 24u + 4u * m);
    D[4 * m] = t[0]; D[4 * m + 1] = t[1]; D[4 * m + 2] = t[2]; D[4 * m + 3] = t[3];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  uint32_t *rec = lds + (mine ? lane : 0u) * kRowW6;
  // A3: nat_4to6's control flow; the ADDR_MAP entry is read now and examined
  // after B1
  uint32_t P[20];
#pragma unroll
  for (int j = 0; j < 20; ++j) P[j] = D[j];
  V4 v;
  classify4(P, len, v);
  const bool act0 = valid && v.disp == CGPU_ACT;
  u32x4 s0 = {0u, 0u, 0u, 0u};
  uint32_t rport = 0u;
  if (act0) {
    rev_read(a.pm, v.gw_port, s0, rport);
  }
  const uint32_t nl = len + 20u;  // meaningful for ACT frames
  if (mine) {
    rec[20] = act0 ? nl : 0u;
    rec[23] = o_off;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // B1: realign and sum the payload of every round (lookup-independent)
  const uint32_t nl0 = __shfl(nl, (int)(__builtin_ctzll(__ballot(act0) | (1ull << 63))));
  if (!__ballot(act0 && nl != nl0)) rows_payload6<true>(X, lds, row, l, nl0);
  else rows_payload6<false>(X, lds, row, l, nl0);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // A4: the ADDR_MAP value, the IPv6 header
  if (act0) addr_map_check(a, len, rport, v);
  const bool act = valid && v.disp == CGPU_ACT;
  if (valid) {
    a.out_len[i] = act ? (uint16_t)nl : 0;
    a.disposition[i] = (uint8_t)v.disp;
    a.status[i] = (uint8_t)v.st;
  }
  uint32_t V[10], ph;
  ipv6_header(v, nl, s0, V, ph);
  // A5: output bytes 0..79 and their share of the TCP sum; the record
  const uint32_t k = v.k, port_be = swap16(rport & 0xffffu);  // the original v6-side port
  uint32_t O[20], accA;
  if (!__ballot(act && k != 0u)) rows_build6<true>(D, V, k, port_be, nl, O, accA);
  else rows_build6<false>(D, V, k, port_be, nl, O, accA);
  const uint32_t span = (nl - (54u + 4u * k)) & 0xffffu;
  // the pseudo-header in the big-endian domain of the final fold
  const uint32_t fph = fold32(swap16(ph) + span + 6u);
  if (mine) {
#pragma unroll
    for (int m = 0; m < 5; ++m)
      *reinterpret_cast<u32x4 *>(rec + 4 * m) = u32x4{O[4 * m], O[4 * m + 1], O[4 * m + 2], O[4 * m + 3]};
    const uint32_t payload = rec[21];
    const uint32_t tcp_c = (~fold32(fph + swap16(fold32(payload + accA)))) & 0xffffu;
    *reinterpret_cast<u32x4 *>(rec + 20) = u32x4{act ? nl : 0u, payload + accA, tcp_c | (k << 16), o_off};
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  rows_store6(a, ors, X, lds, row, l);
  return true;
}

// The general 4to6 path: one quad per frame (any alignment, any length).
__device__ __forceinline__ void quad_4to6(const Nat64Args &a, rsrc_t rs, rsrc_t ors, uint32_t i,
                                          uint32_t lane) {
  const uint32_t g = lane & (kFG - 1u);
  QuadDesc d = quad_desc<false>(a, i);
  quad_modes<false>(a, d);
  const bool al16 = d.fast && !__ballot(d.nl != 0u && (d.off & 15u) != 0u);
  u32x4 X[kFJ], Y, Y4;
  uint32_t E;
  issue_frame_loads<false>(rs, d, g, al16, X, E);
  header_loads(rs, a.arena_len, d.off, g, d.valid, d.hdr_fast, d.al_wave, Y, Y4);
  uint32_t P[20];
  gather_header(Y, Y4, P);
  V4 v;
  classify4(P, d.len, v);
  // assigned_addr(port): the quad's lanes read the same words (one request)
  u32x4 s0 = {0u, 0u, 0u, 0u};
  uint32_t rport = 0u;
  if (d.valid && v.disp == CGPU_ACT) {
    rev_read(a.pm, v.gw_port, s0, rport);
    addr_map_check(a, d.len, rport, v);
  }
  const bool act = d.valid && v.disp == CGPU_ACT;
  if (d.valid && g == 0u) {
    a.out_len[d.i] = act ? (uint16_t)d.nl : 0;
    a.disposition[d.i] = (uint8_t)v.disp;
    a.status[d.i] = (uint8_t)v.st;
  }
  if (!act) return;
  FrameRec f;
  f.in_off = d.off;
  f.o_off = d.o_off;
  f.new_len = d.nl;
  ipv6_header(v, d.nl, s0, f.V, f.ph);
  f.info = v.k | kNow | ((rport & 0xffffu) << 16);  // the original v6-side port
  f.defer_i = kNoSlot;
  rewrite_quad<false>(a, rs, ors, g, d, al16, f, X, E);
}

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
void nat64_4to6_fused(Nat64Args a) {
  __shared__ uint32_t lds[kBlock / 64][kRowFrames * kRowW6];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t base = (blockIdx.x * (kBlock / 64u) + wave) * kRowFrames;
  if (base >= a.n) return;  // wave-uniform
  const rsrc_t rs = make_rsrc(a.arena, a.arena_len);
  const rsrc_t ors = make_rsrc(a.out_arena, a.out_arena_len);
  if (rows_4to6(a, rs, ors, base, lane, lds[wave])) return;
  for (uint32_t q = 0; q < kRowFrames / 16u; ++q) quad_4to6(a, rs, ors, base + 16u * q + lane / 4u, lane);
}

__global__ void portmap_init(PortMapDev pm, uint32_t first_port) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= pm.cap_mask) {
    u32x4 *s = reinterpret_cast<u32x4 *>(&pm.slots[i]);
    s[0] = u32x4{0u, 0u, 0u, 0u};
    s[1] = u32x4{0u, 0u, 0u, 0xffffffffu};
  }
  if (i < 65536u) {
#pragma unroll
    for (uint32_t j = 0; j < 5u; ++j) pm.rev[5u * i + j] = 0u;
  }
  if (i == 0) {
    pm.state[0] = first_port;  // NEXT_PORT
    // entries and the per-call-parity deferred flags
    for (uint32_t j = 1; j < 64u; ++j) pm.state[j] = 0u;
  }
}

}  // namespace

uint32_t nat64_num_blocks(uint32_t n) { return (n + kBlock - 1) / kBlock; }
size_t nat64_ctl_offset(uint32_t n) {  // 4 KiB aligned within the scratch's chunk area
  return (4ull * (10ull * nat64_num_blocks(n) + n) + 4095ull) & ~4095ull;
}
size_t nat64_chunk_bytes(uint32_t n) { return nat64_ctl_offset(n) + 4ull * (kShards * kShardW + 32u); }

hipError_t launch_portmap_init(const PortMapDev &pm, uint32_t first_port, hipStream_t s) {
  // one thread per slot and ADDR_MAP entry
  const uint32_t cap = pm.cap_mask + 1u > 65536u ? pm.cap_mask + 1u : 65536u;
  hipLaunchKernelGGL(portmap_init, dim3((cap + 255) / 256), dim3(256), 0, s, pm, first_port);
  return hipGetLastError();
}

// done (may be null): recorded when the call's last kernel completes, as
// the kernel's own completion (hipExtLaunchKernelGGL's stop event) rather
// than a separate marker packet behind it
hipError_t launch_nat64_6to4(const Nat64Args &a, hipStream_t s, hipEvent_t done) {
  if (a.n == 0) return hipSuccess;
  const uint32_t nb = nat64_num_blocks(a.n);
  const uint32_t fpb = (kBlock / 64u) * kRowFrames;  // fused: kRowFrames frames per wave
  const uint32_t nbf = (a.n + fpb - 1) / fpb;
  hipLaunchKernelGGL(nat64_6to4_fused, dim3(nbf), dim3(kBlock), 0, s, a);
  // the tail: the order of the new keys, then their frames' ports; in the
  // steady state (no new key) both grids return at once
  const uint32_t og = (nb + kOrderU - 1u) / kOrderU;
  hipLaunchKernelGGL(nat64_tail_order, dim3(og < kOrderGrid ? og : kOrderGrid), dim3(kBlock), 0, s, a, nb);
  hipExtLaunchKernelGGL(nat64_tail_patch, dim3(nb < kPatchGrid ? nb : kPatchGrid), dim3(kBlock), 0, s,
                        nullptr, done, 0, a, nb);
  return hipGetLastError();
}

hipError_t launch_nat64_4to6(const Nat64Args &a, hipStream_t s, hipEvent_t done) {
  if (a.n == 0) return hipSuccess;
  const uint32_t fpb = (kBlock / 64u) * kRowFrames;  // kRowFrames frames per wave
  hipExtLaunchKernelGGL(nat64_4to6_fused, dim3((a.n + fpb - 1) / fpb), dim3(kBlock), 0, s, nullptr, done, 0, a);
  return hipGetLastError();
}

}  // namespace cgpu
