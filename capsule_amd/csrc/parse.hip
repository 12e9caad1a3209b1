// parse.hip — batched Ethernet -> IPv4/IPv6 -> UDP/TCP parse, Internet
// checksums and 5-tuple flow hash on gfx950.
//
// One packet per lane.  A wave whose packets all sit at dword-aligned offsets
// well inside the arena (the normal case: packets in 64-byte slots) loads
// its 96-byte windows with unconditional buffer_load_dwordx4s (the last two
// only when some lane's packet is that long: a wave-uniform ballot), and
// reads every header field straight out of the loaded dwords; a wave with a
// misaligned packet or one near the end of the arena takes the general,
// tail-safe loader.  The window is shifted by the VLAN tag depth only when
// some lane has a tagged frame.  Checksums are exact integer sums of u16
// words accumulated with v_sad_u16 over the same registers (bytes past the
// window are streamed from memory); with a wave-uniform frame length the end
// masks are scalar.  Outputs are SoA: u32 meta, optional u32 (ip_csum |
// l4_csum << 16), u64 flow hash, optional 96-byte header record.
//
// Reference chain restated (file:line in /root/reference):
//   Ethernet::try_parse        core/src/packets/ethernet.rs:279-300, 164-181, 253-261
//   Ipv4::try_parse            core/src/packets/ip/v4.rs:427-442 (header fixed at 20 B, :403)
//   Ipv6::try_parse            core/src/packets/ip/v6/mod.rs:274-289 (40 B)
//   Udp/Tcp::try_parse         core/src/packets/udp.rs:287-302, tcp.rs:558-573 (8 / 20 B)
//   Mbuf::read_data bounds     core/src/dpdk/mbuf.rs:313-327
//   Ipv4::compute_checksum     core/src/packets/ip/v4.rs:322-333
//   Udp::compute_checksum      core/src/packets/udp.rs:204-219, set_checksum :132-141
//   Tcp::compute_checksum      core/src/packets/tcp.rs:462-477
//   PseudoHeader::sum          core/src/packets/checksum.rs:56-128
//   Udp/Tcp::flow              core/src/packets/udp.rs:151-159, tcp.rs:409-417
//   Icmpv4/Icmpv6::try_parse   core/src/packets/icmp/v4/mod.rs:205-220, icmp/v6/mod.rs:217-232 (4 B)
//   Icmpv4::compute_checksum   icmp/v4/mod.rs:118-129 (no pseudo-header)
//   Icmpv6::compute_checksum   icmp/v6/mod.rs:123-138 (pseudo-header, protocol 58)
//   SegmentRouting::try_parse  core/src/packets/ip/v6/srh.rs:299-327, dst()/pseudo_header :421-470
//   Fragment::try_parse        core/src/packets/ip/v6/fragment.rs:187-202
#include "capsule_gpu.h"
#include "device_common.hpp"
#include "kernels.hpp"

namespace cgpu {

namespace {

constexpr uint32_t kBlock = 256;
constexpr int kWin = 24;        // packet-relative window dwords (96 B)
constexpr uint32_t kQEnd = 88;  // normalized window bytes valid after a QinQ shift
constexpr uint32_t kNoRead = 0xffffff00u;  // > any arena_len the ABI accepts
// Cache policy of the loads whose instruction reads whole lines (the rows,
// stream and tail paths: 256 B or 1 KiB contiguous per instruction, each
// line once): nontemporal, so the frame stream does not push the lines that
// are still to be used out of the L2.  Measured (round 5, A/B on one box):
// parse256 59.7 -> 53.8 us, parse1500 289.4 -> 272.7, IMIX with checksums
// 92.0 -> 87.6, reconcile IMIX 125.9 -> 113.2, reconcile64 29.6 -> 27.3.
// The per-lane window loads (64 B of a frame in four strided instructions,
// whose lines the next instruction reuses) keep the default policy: with
// nontemporal loads parse64 went from 16.4 to 22.6 us.
constexpr int kNT = 2;
constexpr uint32_t kSlotPieces = 2;  // longest tail (256-B pieces) summed in slots
constexpr uint32_t kSlotIt = 4;  // slots per 16-lane row and round (loads in flight)
constexpr uint32_t kRowMaxLen = 512;  // the rows path: frames up to 2 pieces
// the rows variant of the checksum configs: batches whose mean slot (arena
// bytes per packet) is 128..kRowsMeanMax B (long frames, but not jumbo ones)
constexpr uint32_t kRowsMeanMax = 2200;
// frames of at least this many bytes sum the rest of their window's line
// early (below: bound by HBM bytes rather than by strided requests)
constexpr uint32_t kLine0Min = 512;

__device__ __forceinline__ uint32_t sel3(uint32_t k, uint32_t a, uint32_t b, uint32_t c) {
  return k == 0u ? a : (k == 1u ? b : c);
}

// (x & 0xffff) + (x >> 16) + acc in one v_sad_u16: exact sum of the two
// little-endian u16 words of a dword.
__device__ __forceinline__ uint32_t sad16(uint32_t x, uint32_t acc) {
  return __builtin_amdgcn_sad_u16(x, 0u, acc);
}

// General window loader: any byte offset, tail-safe at the end of the arena
// (only waves with a misaligned packet or one near the arena end run it).
__device__ __forceinline__ void load_window_general(rsrc_t rs, uint32_t arena_len, uint32_t off,
                                                    uint32_t len, uint32_t (&P)[kWin]) {
  const uint32_t sh = off & 3u;
  const uint32_t base = off - sh;
  const uint32_t need = sh + (len < 96u ? len : 96u);
  uint32_t D[kWin + 1];
#pragma unroll
  for (int j = 0; j < kWin + 1; ++j)
    D[j] = (uint32_t)(4 * j) < need ? load4_tail(rs, base + 4u * j, arena_len) : 0u;
#pragma unroll
  for (int j = 0; j < kWin; ++j) P[j] = __builtin_amdgcn_alignbyte(D[j + 1], D[j], sh);
}

// Sum of normalized window dwords j in [J0, 22) restricted to bytes < wend.
template <int J0>
__device__ __forceinline__ uint32_t sum_to_end(const uint32_t (&Q)[kWin - 2], uint32_t wend,
                                               uint32_t acc) {
#pragma unroll
  for (int j = J0; j < (int)(kQEnd / 4); ++j) {
    const uint32_t lo = 4u * (uint32_t)j;
    uint32_t m = 0xffffffffu;
    if (wend < lo + 4u) m = wend <= lo ? 0u : (0xffffffffu >> (8u * (lo + 4u - wend)));
    acc = sad16(Q[j] & m, acc);
  }
  return acc;
}

// The same for a wave-uniform wend (an SGPR): whole words are summed without
// a mask, and the words past the end are skipped by scalar branches.
template <int J0>
__device__ __forceinline__ uint32_t sum_to_end_s(const uint32_t (&Q)[kWin - 2], uint32_t wend,
                                                 uint32_t acc) {
#pragma unroll
  for (int j = J0; j < (int)(kQEnd / 4); ++j) {
    const uint32_t lo = 4u * (uint32_t)j;
    if (wend <= lo) break;
    acc = sad16(wend < lo + 4u ? Q[j] & (0xffffffffu >> (8u * (lo + 4u - wend))) : Q[j], acc);
  }
  return acc;
}

// Tail sums.  A 1 KiB piece [b, b + 1024) of a tail [from, to) (absolute
// arena offsets, b = from & ~15 + 1024 j) is loaded by the whole wave, 16 B
// per lane; a lane loads its chunk only if the chunk overlaps [from, to), and
// sums all 16 bytes without masks.  The bytes of the first and last chunk that
// lie outside [from, to) are subtracted afterwards from wave-uniform copies of
// those two chunks (v_readlane + scalar arithmetic).
__device__ __forceinline__ uint32_t sum4(u32x4 v, uint32_t acc) {
  return sad16(v[3], sad16(v[2], sad16(v[1], sad16(v[0], acc))));
}

// u16-word sum of the bytes of chunk [c, c + 16) outside [from, to).
__device__ __forceinline__ uint32_t chunk_excess(u32x4 v, uint32_t c, uint32_t from, uint32_t to) {
  uint32_t e = 0;
#pragma unroll
  for (uint32_t t = 0; t < 4u; ++t) {
    const uint32_t d = c + 4u * t;
    uint32_t keep = 0xffffffffu;
    if (from > d) keep = from >= d + 4u ? 0u : (0xffffffffu << (8u * (from - d)));
    if (to < d + 4u) keep &= to <= d ? 0u : (0xffffffffu >> (8u * (d + 4u - to)));
    const uint32_t x = v[t] & ~keep;
    e += (x & 0xffffu) + (x >> 16);
  }
  return e;
}

// Masks a 16-B chunk at its frame's end: bytes [rem, 16) become 0 (rem >= 16:
// none).  Dword t keeps its low 8 * clamp(rem - 4 t, 0, 4) bits: the low half
// of 2^32 - 1 shifted right by the dropped bits as a 64-bit value (a shift by
// 32 gives 0, where a 32-bit shift would wrap), 4 VALU per dword against 7
// for two compares and two selects.
__device__ __forceinline__ void mask_chunk(u32x4 &v, uint32_t rem) {
  const int r8 = 8 * (int)(rem < 16u ? rem : 16u);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    int sh = 32 * t + 32 - r8;
    sh = sh < 0 ? 0 : (sh > 32 ? 32 : sh);
    v[t] &= (uint32_t)(0xffffffffull >> sh);
  }
}

// ---- the rows path (L4 checksum configs, waves of long frames) -----------
// A wave whose frames are 16-B aligned and at least 7/8 of them 128 B or
// longer reads each frame's first 512 B once, in rows: 16 lanes
// take one 256-B piece of one frame per load instruction (four whole frames
// per instruction, full lines), sum its u16 words (the frame's last chunk
// masked at its end) and reduce them over the row with DPP; the first 96 B
// of every frame pass through wave-private LDS to the frame's own lane.  The
// lane then has its window P and the exact word sum of the whole frame;
// the checksum span's sum is that sum minus the words before the span, plus
// the checksum tail's sum of bytes [512, len) for longer frames.  No line is
// fetched twice, as the per-lane window + tail passes can for line 0 of long
// frames (window: bytes 0..63; tail: bytes 64..127, later).
// Frames are processed in two halves of 32 (LDS: 32 x 96 B + sums per wave).
constexpr uint32_t kRowHalf = 32;
constexpr uint32_t kRowLds = kRowHalf * kWin + kRowHalf;  // dwords per wave

__device__ __forceinline__ void rows_prologue(rsrc_t rs, uint32_t off, uint32_t len, uint32_t lane,
                                              uint32_t *L, uint32_t (&P)[kWin], uint32_t &s_all) {
  const uint32_t row = lane >> 4, l = lane & 15u;
  // a frame longer than kRowMaxLen is summed here up to kRowMaxLen; the
  // checksum tail takes the rest
  len = len < kRowMaxLen ? len : kRowMaxLen;
  uint32_t npass = 0;  // 256-B pieces of the wave's longest (clipped) frame
#pragma unroll
  for (uint32_t p = 0; p < kRowMaxLen / 256u; ++p)
    if (__ballot(len > 256u * p)) npass = p + 1u;
  uint32_t *sums = L + kRowHalf * kWin;
#pragma unroll
  for (uint32_t half = 0; half < 2u; ++half) {
    for (uint32_t p = 0; p < npass; ++p) {
      // the half's 8 rounds in two groups of 4 loads in flight (the kernel
      // runs at 8 waves per SIMD: 64 VGPRs)
#pragma unroll
      for (uint32_t rg = 0; rg < kRowHalf / 16u; ++rg) {
        u32x4 v[4];
        uint32_t fl[4];
#pragma unroll
        for (uint32_t u = 0; u < 4u; ++u) {
          const uint32_t f = kRowHalf * half + 16u * rg + 4u * u + row;
          const uint32_t fo = __shfl(off, (int)f);
          fl[u] = __shfl(len, (int)f);
          const uint32_t c = 16u * p + l;
          v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(16u * c < fl[u] ? fo + 16u * c : kNoRead), 0, kNT);
        }
#pragma unroll
        for (uint32_t u = 0; u < 4u; ++u) {
          const uint32_t fr = 16u * rg + 4u * u + row;  // frame within the half
          if (p == 0u && l < 6u) *reinterpret_cast<u32x4 *>(L + fr * kWin + 4u * l) = v[u];
          const uint32_t b0 = 256u * p + 16u * l;
          const uint32_t rem = fl[u] > b0 ? fl[u] - b0 : 0u;
          u32x4 x4 = v[u];
          if (__ballot(rem < 16u)) mask_chunk(x4, rem);
          uint32_t x = sum4(x4, 0u);
          x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, true);  // row_shr:1
          x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, true);  // row_shr:2
          x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, true);  // row_shr:4
          x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, true);  // row_shr:8
          if (l == 15u) sums[fr] = p == 0u ? x : sums[fr] + x;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if ((lane >> 5) == half) {
      const uint32_t fr = lane & (kRowHalf - 1u);
#pragma unroll
      for (int m = 0; m < kWin / 4; ++m) {
        const u32x4 t = *reinterpret_cast<const u32x4 *>(L + fr * kWin + 4u * m);
        P[4 * m] = t[0];
        P[4 * m + 1] = t[1];
        P[4 * m + 2] = t[2];
        P[4 * m + 3] = t[3];
      }
      s_all = npass ? sums[fr] : 0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
}

// ---- the stream path (L4 checksum configs, waves of consecutive frames) ----
// A wave whose 64 frames are 16-B aligned and lie in ascending,
// non-overlapping order within kStreamMax bytes (a burst gathered into an
// arena: IMIX in 64-B slots, 256-B frames) reads that span as one stream,
// 1 KiB per load instruction (16 B per lane, whole lines, each line once),
// and attributes every 16-B chunk to the frame it belongs to: a bitmap of
// frame starts (one bit per chunk) with per-word prefix counts in LDS gives
// a chunk's owner in two LDS reads.  A chunk is loaded only if it lies
// before its owner's end (slot padding is skipped) and masked at that end.
// The chunk sums are added into per-frame accumulators by a segmented scan:
// one inclusive wave scan (DPP), then the last lane of each owner's run of
// lanes adds its prefix and the first one subtracts the prefix before it.
// The result is each frame's exact word sum, as the rows path produces
// (the checksum span is that minus the words before it).  Unlike the
// window + tail path, no line is read twice: a long frame's last line is
// often the next frame's first, which the tail pass fetched again after
// the window pass had let it go.
constexpr uint32_t kStreamU = 3;  // 1 KiB loads in flight per lane and step
constexpr uint32_t kStreamMax = 32768;  // span bytes per wave: 2048 chunks, one bitmap word per lane


__device__ __forceinline__ uint32_t dpp_wave_shr1(uint32_t v) {  // lane l <- lane l - 1 (lane 0: 0)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_wave_shl1(uint32_t v) {  // lane l <- lane l + 1 (lane 63: 0)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);
}

// Inclusive prefix sum over the 64 lanes (row shifts, then the row
// broadcasts of lanes 15 and 31).
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

// Whether the wave takes the stream path (wave-uniform); base = the first
// frame's offset, span = bytes to the last frame's end.
__device__ __forceinline__ bool stream_wave(uint32_t off, uint32_t len, bool valid, uint32_t lane,
                                            uint32_t arena_len, uint32_t &base, uint32_t &span) {
  const uint32_t noff = __shfl_down(off, 1);
  const bool ok = valid && (off & 15u) == 0u && (lane == 63u || (noff > off && noff - off >= len));
  if (__ballot(ok) != ~0ull || !__ballot(len > 96u)) return false;
  // the chunk grid starts at the first frame's line: every load instruction
  // of the stream then covers 8 whole lines, none shared with the next one
  base = __builtin_amdgcn_readfirstlane(off) & ~127u;
  const uint32_t end = __builtin_amdgcn_readlane(off + len, 63);
  span = end - base;
  return span <= kStreamMax && (uint64_t)end + 16u <= (uint64_t)arena_len;
}

// One 64-chunk step of the stream: chunk c of the span (relative to base)
// for this lane, its owner frame and that frame's end.
struct StreamChunk {
  uint32_t c, own, fe;
};

// Chunks at or past `hi` (the end of the half's range) take the owner of
// chunk hi - 1, and chunks before `lo` (the line-aligned start of a step
// grid) the owner of chunk lo: a valid frame of the half, whose sum they add
// 0 to (they are not loaded).  Their own bitmap word may lie past the bitmap.
__device__ __forceinline__ StreamChunk stream_chunk(const uint32_t *bm, const uint32_t *pre,
                                                    const uint32_t *fend, uint32_t c, uint32_t lo,
                                                    uint32_t hi) {
  const uint32_t q = c < lo ? lo : (c < hi ? c : hi - 1u), w = q >> 5;
  StreamChunk k;
  k.c = c;
  k.own = pre[w] + (uint32_t)__builtin_popcount(bm[w] & ((2u << (q & 31u)) - 1u)) - 1u;
  k.fe = fend[k.own];
  return k;
}

// Every frame's window P (bytes 0..95) and exact u16-word sum s_all (bytes
// [0, len)) from the wave's span.  The frames are taken in two halves of 32
// (the windows of one half in LDS at a time); within a half the span is read
// kStreamU KiB per step (kStreamU loads in flight per lane).  L: the wave's LDS,
// kStreamLds dwords.
constexpr uint32_t kStreamLds = 5u * 64u + kRowHalf * kWin;

__device__ __forceinline__ void stream_prologue(rsrc_t rs, uint32_t base, uint32_t span, uint32_t off,
                                                uint32_t len, uint32_t lane, uint32_t *L,
                                                uint32_t (&P)[kWin], uint32_t &s_all) {
  uint32_t *bm = L, *pre = L + 64, *fst = L + 128, *fend = L + 192, *acc = L + 256, *win = L + 320;
  bm[lane] = 0u;
  acc[lane] = 0u;
  fst[lane] = off - base;
  fend[lane] = off - base + len;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const uint32_t cs = (off - base) >> 4;  // the frame's first chunk
  atomicOr(&bm[cs >> 5], 1u << (cs & 31u));
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const uint32_t pc = (uint32_t)__builtin_popcount(bm[lane]);
  pre[lane] = wave_scan_incl(pc) - pc;  // frames starting before word `lane`
  const uint32_t nch = (span + 15u) >> 4;
  const uint32_t first = __builtin_amdgcn_readfirstlane(cs);          // frame 0's first chunk
  const uint32_t mid = __builtin_amdgcn_readlane(cs, (int)kRowHalf);  // half 1's first chunk
#pragma unroll
  for (uint32_t half = 0; half < 2u; ++half) {
    // a half's steps start on the line of its first chunk (base is a line)
    const uint32_t lo = half ? mid : first, hi = half ? nch : mid;
#pragma unroll
    for (uint32_t m = 0; m < kRowHalf * kWin / 256u; ++m)
      *reinterpret_cast<u32x4 *>(win + 4u * (64u * m + lane)) = u32x4{0u, 0u, 0u, 0u};
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (uint32_t c0 = lo & ~7u; c0 < hi; c0 += 64u * kStreamU) {
      StreamChunk k[kStreamU];
      u32x4 v[kStreamU];
#pragma unroll
      for (uint32_t u = 0; u < kStreamU; ++u) {
        k[u] = stream_chunk(bm, pre, fend, c0 + 64u * u + lane, lo, hi);
        const uint32_t rel = 16u * k[u].c;
        const bool in = k[u].c >= lo && k[u].c < hi && rel < k[u].fe;
        v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(in ? base + rel : kNoRead), 0, kNT);
      }
#pragma unroll
      for (uint32_t u = 0; u < kStreamU; ++u) {
        const uint32_t rel = 16u * k[u].c;
        const uint32_t rem = k[u].c >= lo && k[u].c < hi && rel < k[u].fe ? k[u].fe - rel : 16u;
        if (__ballot(rem < 16u)) mask_chunk(v[u], rem);
        // bytes 0..95 of a frame of this half: its window
        const uint32_t pos = rel - fst[k[u].own], fh = k[u].own - kRowHalf * half;
        if (k[u].c < hi && pos < 96u && fh < kRowHalf)
          *reinterpret_cast<u32x4 *>(win + __umul24(fh, kWin) + (pos >> 2)) = v[u];
        const uint32_t p = wave_scan_incl(sum4(v[u], 0u));
        const uint32_t own = k[u].own;
        const uint32_t own_prev = dpp_wave_shr1(own), own_next = dpp_wave_shl1(own);
        const uint32_t p_prev = dpp_wave_shr1(p);
        if (lane == 63u || own_next != own) atomicAdd(&acc[own], p);
        if (lane != 0u && own_prev != own) atomicSub(&acc[own], p_prev);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if ((lane >> 5) == half) {
      const uint32_t fh = lane & (kRowHalf - 1u);
#pragma unroll
      for (int m = 0; m < kWin / 4; ++m) {
        const u32x4 t = *reinterpret_cast<const u32x4 *>(win + fh * kWin + 4u * m);
        P[4 * m] = t[0];
        P[4 * m + 1] = t[1];
        P[4 * m + 2] = t[2];
        P[4 * m + 3] = t[3];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  s_all = acc[lane];
}

// ---- Longest span first: the order of the later waves ---------------------
// A wave takes 64 consecutive frames, and on the stream / rows paths its time
// follows its span (the bytes from its first frame's start to its last
// frame's end): for shuffled IMIX 11 to 37 KB.  A 1 Mi-packet launch is
// 16,384 waves, two per wave slot of the chip, and the waves dispatched last
// decide when it ends: with the groups taken in their own order the launch
// took 86.7 us, with the last half of them taken longest span first 77.3 us,
// with all after the first quarter 76.5 us (tools/imix_order_probe.py,
// DESIGN.md section 3.1; the host orders from half a round on).  So the launch's first
// sched_n / 256 workgroups each order 256 of the last sched_n groups by span,
// longest first (64 classes a quarter octave wide; a counting sort in LDS,
// one atomic per class present in a wave, never one per lane), and the k-th
// group of list b goes to the wave at position k * lists + b of the ordered
// range: the lists interleave into about the global order with no exchange
// between workgroups.  A wave learns its group from granule q: 8 bytes
// {tag, group} written by ONE write-through (sc1) store and polled by ONE
// lane with sc1 loads, so no fence orders anything (the R2 granule of
// cdna_hip_programming.md Guideline 16).  The tag is the call's own (the host
// counts calls per buffer), and the wave that takes a granule clears it, so
// an entry an earlier launch left never matches.  Calls captured into a
// graph run without the schedule (capi.hip set_schedule): replays of one
// graph would share a buffer and a tag.
// Which wave takes which group changes no output: every frame's results are
// its own.
typedef __attribute__((address_space(1))) unsigned long long gu64;
constexpr uint32_t kSchedClasses = 64;

__device__ __forceinline__ uint32_t span_class(uint32_t span) {
  // quarter octaves, longest first: class 0 holds spans of 16 MiB and more,
  // class 63 those below 304 B
  const uint32_t s = span < 16u ? 16u : span;
  const uint32_t msb = 31u - (uint32_t)__builtin_clz(s);
  const uint32_t q = 4u * msb + ((s >> (msb - 2u)) & 3u);  // 16 .. 127
  return q >= 96u ? 0u : (q <= 33u ? kSchedClasses - 1u : 96u - q);
}

// Adds each lane's count to ctr[its class] with one LDS atomic per class the
// wave holds; returns the counter's value before this wave's add plus the
// lane's rank among the wave's lanes of its class (lanes with in == false
// take no part).
__device__ __forceinline__ uint32_t class_add(uint32_t *ctr, uint32_t c, bool in) {
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t left = __ballot(in);
  uint32_t pos = 0;
  while (left) {
    const uint32_t first = (uint32_t)__builtin_ctzll(left);
    const uint32_t cc = __builtin_amdgcn_readlane(c, (int)first);
    const uint64_t m = __ballot(in && c == cc);
    uint32_t base = 0;
    if (lane == first) base = atomicAdd(&ctr[cc], (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, (int)first);
    if (in && c == cc) pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    left &= ~m;
  }
  return pos;
}

__device__ void schedule_waves(const ParseArgs &a, uint32_t *L) {
  uint32_t *cnt = L, *cur = L + kSchedClasses;
  const uint32_t t = threadIdx.x, lists = a.sched_n / kBlock, j = kBlock * blockIdx.x + t;
  if (t < kSchedClasses) cnt[t] = 0u;
  const uint64_t nb = (uint64_t)a.n;
  const rsrc_t r_off = make_rsrc(a.off, (uint32_t)(4u * nb < 0xffffffffull ? 4u * nb : 0xffffffffull));
  const rsrc_t r_len = make_rsrc(a.len, (uint32_t)(2u * nb < 0xffffffffull ? 2u * nb : 0xffffffffull));
  const uint32_t g = a.sched_from + j;
  const uint32_t f0 = 64u * g, f1 = (f0 + 63u < a.n ? f0 + 63u : a.n - 1u);
  const uint32_t o0 = __builtin_amdgcn_raw_buffer_load_b32(r_off, (int)(4u * f0), 0, 0);
  const uint32_t o1 = __builtin_amdgcn_raw_buffer_load_b32(r_off, (int)(4u * f1), 0, 0);
  const uint32_t l1 = __builtin_amdgcn_raw_buffer_load_b16(r_len, (int)(2u * f1), 0, 0);
  // frames out of order (no stream path): the lightest class
  const uint32_t c = o1 >= o0 ? span_class(o1 + l1 - o0) : kSchedClasses - 1u;
  __syncthreads();
  (void)class_add(cnt, c, true);
  __syncthreads();
  if (t < 64u) {  // exclusive prefix over the classes (one wave, 64 classes)
    const uint32_t x = cnt[t];
    // the first list tells the host whether this batch's spans vary (one
    // class: the order buys nothing, and the host orders the stream's next
    // batch from the second round on only, so that no first-round wave waits)
    const uint64_t present = __ballot(x != 0u);
    if (blockIdx.x == 0 && t == 0 && a.sched_spread != nullptr)
      __hip_atomic_store(a.sched_spread, __popcll(present) > 1 ? 1u : 0u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t y = x;
#pragma unroll
    for (uint32_t d = 1; d < 64u; d <<= 1) {
      const uint32_t z = (uint32_t)__shfl_up((int)y, d);
      if (t >= d) y += z;
    }
    cur[t] = y - x;
  }
  __syncthreads();
  const uint32_t k = class_add(cur, c, true);  // the group's rank in this list, longest first
  __hip_atomic_store((gu64 *)(a.sched + k * lists + blockIdx.x), ((unsigned long long)a.sched_tag << 32) | g,
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The group of 64 frames this wave takes (wave-uniform); ~0u: none (a wave
// that gave up waiting for its granule).  A give-up is never silent: the
// wave ORs kDevErrSched into the context's device error word, and the call
// (or the next cgpu_ctx_check) fails with CGPU_EIO.  Forward progress
// (DESIGN.md §3.1): the ordering workgroups are the launch's lowest
// workgroup ids and wait on nothing; each XCD places its workgroups in id
// order, so no wave of this launch can take the slot an ordering workgroup
// of its own XCD is waiting for.  A kernel of another stream that fills an
// XCD delays that XCD's ordering workgroup until its own waves end; it
// cannot block it.
__device__ __forceinline__ uint32_t wave_group(const ParseArgs &a) {
  if (a.sched == nullptr) return blockIdx.x * (kBlock / 64u) + (threadIdx.x >> 6);
  const uint32_t v = (blockIdx.x - a.sched_n / kBlock) * (kBlock / 64u) + (threadIdx.x >> 6);
  const uint32_t q = v - a.sched_from;
  if (v < a.sched_from || q >= a.sched_n) return v;
  uint32_t g = ~0u;
  if ((threadIdx.x & 63u) == 0u) {
    for (uint32_t spins = 0; spins < a.sched_spins; ++spins) {
      const unsigned long long x = __hip_atomic_load((gu64 *)(a.sched + q), __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
      if ((uint32_t)(x >> 32) == a.sched_tag) {
        g = (uint32_t)x;
        // consumed: cleared for the next launch, so that no later launch
        // can read this one's entry
        __hip_atomic_store((gu64 *)(a.sched + q), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
    if (g == ~0u) __hip_atomic_fetch_or(a.dev_err, kDevErrSched, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  return (uint32_t)__shfl((int)g, 0);
}

// V4U: the accept set has no IPv6, TCP, ICMP or extension bit (the typed
// parse::<Ipv4>() -> parse::<Udp<Ipv4>>() chain of the reference bench,
// bench/packets.rs:65-69): every IPv6 / TCP / ICMP branch is compiled out,
// as Rust monomorphises the typed chain.
// A big-endian u16 field store into a frame (any byte offset).
__device__ __forceinline__ void st16be(uint8_t *p, uint32_t v) {
  if (((uintptr_t)p & 1u) == 0u) {
    *reinterpret_cast<uint16_t *>(p) = (uint16_t)swap16(v);
  } else {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
  }
}

// RECON: the cgpu_reconcile variant (Packet::reconcile_all, packets/mod.rs:
// 297-300).  The layers come from the parse's meta words instead of the
// frame's bytes (a typed packet keeps its parse's offsets), the sums are the
// parse's, adjusted for the fields reconcile rewrites first (UDP length,
// IPv4 total_length), and the lane stores the new fields into its frame.
template <bool IPC, bool L4C, bool HASH, bool FIELDS, bool EXT, bool V4U, bool ROWS, bool RECON>
__device__ __forceinline__ void parse_body(const ParseArgs &a) {
  constexpr uint32_t kPathLds = kRowLds > kStreamLds ? kRowLds : kStreamLds;
  __shared__ uint32_t rlds[ROWS ? kBlock / 64 : 1][ROWS ? kPathLds : 1];
  if constexpr (ROWS) {
    static_assert((kBlock / 64) * kPathLds >= 2u * kSchedClasses, "the schedule's LDS");
    if (a.sched != nullptr && blockIdx.x < a.sched_n / kBlock) {
      schedule_waves(a, &rlds[0][0]);
      return;
    }
  }
  const uint32_t grp = ROWS ? wave_group(a) : blockIdx.x * (kBlock / 64u) + (threadIdx.x >> 6);
  const uint32_t i = grp == ~0u ? ~0u : 64u * grp + (threadIdx.x & 63u);
  // No early exit: lanes past n run with len 0 (status BadOffset) and store
  // nothing, so the wave stays whole for the cooperative tail sum below.
  const bool valid = i < a.n;
  const rsrc_t rs = make_rsrc(a.arena, a.arena_len);
  // descriptors through buffer resources: lanes past n read 0 (no branch)
  const uint64_t nb = (uint64_t)a.n;
  const rsrc_t r_off = make_rsrc(a.off, (uint32_t)(4u * nb < 0xffffffffull ? 4u * nb : 0xffffffffull));
  const rsrc_t r_len = make_rsrc(a.len, (uint32_t)(2u * nb < 0xffffffffull ? 2u * nb : 0xffffffffull));
  const uint32_t off = __builtin_amdgcn_raw_buffer_load_b32(r_off, (int)(4u * i), 0, 0);
  const uint32_t len = __builtin_amdgcn_raw_buffer_load_b16(r_len, (int)(2u * i), 0, 0);
  // RECON: the parse's meta word and the layers it records
  uint32_t mi = 0;
  if constexpr (RECON) {
    const rsrc_t r_meta = make_rsrc(a.meta_in, (uint32_t)(4u * nb < 0xffffffffull ? 4u * nb : 0xffffffffull));
    mi = __builtin_amdgcn_raw_buffer_load_b32(r_meta, (int)(4u * i), 0, 0);
  }
  const uint32_t m_k = (mi & CGPU_META_QINQ) ? 2u : ((mi & CGPU_META_DOT1Q) ? 1u : 0u);
  const uint32_t m_l3 = (mi >> 16) & 3u, m_l4 = (mi >> 18) & 3u, m_x = (mi >> 24) & 3u;

  // --- the packet-relative window P ---------------------------------------
  uint32_t P[kWin];
  uint32_t wlim = 96u;  // packet bytes the window holds
  uint32_t l0_sum = 0, l0_adv = 0;  // the window line's rest, summed early (below)
  bool rows = false;     // the rows path (above): window and frame sum from rows
  bool stream = false;   // the stream path (above): frame sums from the wave's span
  uint32_t s_all = 0, st_base = 0, st_span = 0;
  if (ROWS) {
    const bool bad = valid && ((off & 15u) != 0u || (uint64_t)off + len + 16u > (uint64_t)a.arena_len);
    const uint64_t vm = __ballot(valid);
    rows = vm && !__ballot(bad) &&
           8u * (uint32_t)__popcll(__ballot(valid && len >= 128u)) >= 7u * (uint32_t)__popcll(vm);
    // waves of long frames keep the rows (as fast, fewer VALU per byte); the
    // stream takes mixed waves (IMIX), whose short frames would leave 12 of a
    // row's 16 lanes idle, and whose long frames' lines past byte 512 the
    // rows' tail pass would fetch a second time
    stream = !rows && stream_wave(off, len, valid, threadIdx.x & 63u, a.arena_len, st_base, st_span);
  }
  const bool slow = (off & 3u) != 0u || (uint64_t)off + 96u > (uint64_t)a.arena_len;
  if (ROWS && rows) {
    rows_prologue(rs, valid ? off : 0u, valid ? len : 0u, threadIdx.x & 63u, rlds[threadIdx.x >> 6], P, s_all);
  } else if (ROWS && stream) {
    stream_prologue(rs, st_base, st_span, off, len, threadIdx.x & 63u, rlds[threadIdx.x >> 6], P, s_all);
  } else if (__ballot(slow)) {
    load_window_general(rs, a.arena_len, off, len, P);
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off + 16u * c), 0, 0);
      P[4 * c] = v[0];
      P[4 * c + 1] = v[1];
      P[4 * c + 2] = v[2];
      P[4 * c + 3] = v[3];
    }
    // Bytes 64..95, per lane, only where a frame's headers end past byte 64
    // (IPv6/TCP, or IPv6 behind VLAN tags) -- decided from the first 64 B --
    // or, with an L4 checksum, where the whole frame fits in 96 B.  A longer
    // frame's checksum span continues at byte 64 in the coalesced tail loop,
    // so it pays no strided loads past its first 64 B.  An instruction is
    // skipped when no lane of the wave needs it.
    wlim = 64u;
    if (__ballot(len > 64u)) {
      const uint32_t mk = be16_lo(P[3]);
      const uint32_t kk = RECON ? m_k : (mk == 0x8100u ? 1u : (mk == 0x88a8u ? 2u : 0u));
      const uint32_t et = be16_lo(sel3(kk, P[3], P[4], P[5]));
      const uint32_t w5 = sel3(kk, P[5], P[6], P[7]);  // normalized bytes 20..23
      const bool is6 = !V4U && (RECON ? m_l3 == CGPU_L3_IPV6 : et == 0x86ddu);
      const uint32_t pr = V4U ? 17u
                          : RECON ? (m_l4 == CGPU_L4_TCP ? 6u : 17u)
                                  : (is6 ? (w5 & 0xffu) : (w5 >> 24));
      const uint32_t hdr_end = (is6 ? 54u + 4u * kk : 0u) + (pr == 6u ? 20u : 8u);
#pragma unroll
      for (int c = 4; c < 6; ++c) {
        const bool need = len > 16u * c && (hdr_end > 16u * c || (L4C && len <= 96u));
        if (need) wlim = 16u * c + 16u;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (__ballot(need))
          v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(need ? off + 16u * c : kNoRead), 0, 0);
        P[4 * c] = v[0];
        P[4 * c + 1] = v[1];
        P[4 * c + 2] = v[2];
        P[4 * c + 3] = v[3];
      }
      // A long frame's checksum tail would start at (off + 64) & ~15 and
      // fetch the rest of this 128-B line again, after the 4 MB L2 has
      // evicted it: the lane sums those chunks now, with the window in
      // flight (at most 4, all inside the frame), and the tail starts on the
      // next line.  Frames of kLine0Min bytes and more only, where
      // the kernel is bound by HBM bytes rather than by strided requests.
      if (L4C) {
        const uint32_t tb = (off + 64u) & ~15u, lb = (tb + 127u) & ~127u;
        const uint32_t nc = wlim == 64u && len >= kLine0Min && lb < off + len ? (lb - tb) >> 4 : 0u;
        if (__ballot(nc != 0u)) {
          u32x4 v[4];
#pragma unroll
          for (uint32_t j = 0; j < 4u; ++j)
            v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(j < nc ? tb + 16u * j : kNoRead), 0, 0);
#pragma unroll
          for (uint32_t j = 0; j < 4u; ++j) l0_sum = sum4(v[j], l0_sum);  // zeros where not loaded
          l0_adv = 16u * (nc < 4u ? nc : 4u);
        }
      }
    } else if (V4U) {
      // no frame of the wave reaches byte 64: in the IPv4/UDP variant these
      // words are only read by the checksum sums, which skip or mask them
#pragma unroll
      for (int j = 16; j < kWin; ++j) P[j] = __builtin_nondeterministic_value(0u);
    } else {
#pragma unroll
      for (int j = 16; j < kWin; ++j) P[j] = 0u;
    }
  }
  if constexpr (RECON && ROWS) {
    // the window's first 64 B, for the coalesced store at the end (the
    // wave's LDS is free once the prologue has handed the windows over)
    static_assert(kPathLds >= 64u * 16u, "a 64-B window per lane");
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    uint32_t *pl = &rlds[threadIdx.x >> 6][16u * (threadIdx.x & 63u)];
#pragma unroll
    for (int m = 0; m < 4; ++m)
      *reinterpret_cast<u32x4 *>(pl + 4 * m) = u32x4{P[4 * m], P[4 * m + 1], P[4 * m + 2], P[4 * m + 3]};
  }

  // --- Ethernet: VLAN marker at bytes 12-13 (ethernet.rs:164-181) ---------
  const uint32_t marker = be16_lo(P[3]);
  const uint32_t k = RECON ? m_k : (marker == 0x8100u ? 1u : (marker == 0x88a8u ? 2u : 0u));
  const uint32_t eth_len = 14u + 4u * k;  // header_len (ethernet.rs:253-261)
  // Q: the window with the VLAN tags squeezed out (ether_type in Q[3] low
  // half, L3 at normalized byte 14).
  uint32_t Q[kWin - 2];
  Q[0] = P[0];
  Q[1] = P[1];
  Q[2] = P[2];
  if (__ballot(k != 0u)) {
#pragma unroll
    for (int j = 3; j < kWin - 2; ++j) Q[j] = sel3(k, P[j], P[j + 1], P[j + 2]);
  } else {
#pragma unroll
    for (int j = 3; j < kWin - 2; ++j) Q[j] = P[j];
  }
  const uint32_t ether_type = be16_lo(Q[3]);

  // --- status: the first failing step of the reference chain --------------
  // RECON: the meta's layers, each only if the accept set has it (else the
  // packet is not one of the pipeline's: NOT_IP / NOT_L4, i.e. skipped)
  const bool v4 = (RECON ? m_l3 == CGPU_L3_IPV4 : ether_type == 0x0800u) && (a.accept & CGPU_F_ACCEPT_V4);
  const bool v6 = !V4U && (RECON ? m_l3 == CGPU_L3_IPV6 : ether_type == 0x86ddu) &&
                  (a.accept & CGPU_F_ACCEPT_V6);
  const uint32_t l3_len = v6 ? 40u : 20u;
  const uint32_t proto0 =
      !RECON ? (v6 ? (Q[5] & 0xffu) : (Q[5] >> 24))
      : (EXT && m_x == CGPU_EXT_SRH)      ? 43u
      : (EXT && m_x == CGPU_EXT_FRAGMENT) ? 44u
      : m_x != CGPU_EXT_NONE              ? 0x100u  // an extension the accept set lacks
      : m_l4 == CGPU_L4_UDP               ? 17u
      : m_l4 == CGPU_L4_TCP               ? 6u
      : m_l4 == CGPU_L4_ICMP              ? (v6 ? 58u : 1u)
                                          : 0x100u;
  // --- IPv6 extension header (CGPU_F_V6_EXT): SegmentRouting (43) or
  // Fragment (44) behind IPv6, read per lane from memory (rare: the L4
  // header behind it can lie past the register window) -------------------
  const bool xcand = EXT && (!RECON || L4C) && v6 && len > eth_len && eth_len + 40u <= len &&
                     (proto0 == 43u || proto0 == 44u);
  uint32_t proto = proto0, l4_off = eth_len + l3_len;
  uint32_t xkind = 0u, xst = 0u, xhl = 0u, X0 = 0u, X1 = 0u;
  uint32_t S0[4] = {0u, 0u, 0u, 0u};  // segments[0], LE dwords of its wire bytes
  uint32_t XU[5] = {0u, 0u, 0u, 0u, 0u};
  bool xok = false;  // the extension parsed: L4 sits at l4_off behind it
  if (EXT && __ballot(xcand)) {
    if (xcand) {
      const uint32_t xo = eth_len + 40u;  // the IPv6 payload offset
      xkind = proto0 == 43u ? CGPU_EXT_SRH : CGPU_EXT_FRAGMENT;
      if (xo >= len) {
        xst = CGPU_PKT_EXT_BAD_OFFSET;  // read_data(offset) (mbuf.rs:313-327)
      } else if (xo + 8u > len) {
        xst = CGPU_PKT_EXT_OUT_OF_BUFFER;
      } else {
        X0 = load4_any(rs, off + xo, a.arena_len);
        X1 = load4_any(rs, off + xo + 4u, a.arena_len);
        if (xkind == CGPU_EXT_SRH) {
          const uint32_t hel = (X0 >> 8) & 0xffu, nseg = (X1 & 0xffu) + 1u;
          if (!(hel != 0u && 2u * nseg == hel)) {
            xst = CGPU_PKT_SRH_INCONSISTENT;
          } else if (xo + 8u >= len) {  // read_data_slice(offset + 8, segments) (mbuf.rs:365-380)
            xst = CGPU_PKT_EXT_BAD_OFFSET;
          } else if (xo + 8u + 16u * nseg > len) {
            xst = CGPU_PKT_EXT_OUT_OF_BUFFER;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) S0[j] = load4_any(rs, off + xo + 8u + 4u * j, a.arena_len);
            xhl = 8u + 16u * nseg;
          }
        } else {
          xhl = 8u;
        }
        if (xst == 0u) {
          xok = true;
          proto = X0 & 0xffu;  // next_header of the extension
          l4_off = xo + xhl;
#pragma unroll
          for (int j = 0; j < 5; ++j) XU[j] = load4_any(rs, off + l4_off + 4u * j, a.arena_len);
        }
      }
    }
  }
  // RECON: the L4 type the meta records (behind an extension header too),
  // not the next-header byte the frame holds now
  const uint32_t lp = RECON ? ((mi & 0xffu) != CGPU_PKT_OK || (m_x != CGPU_EXT_NONE && !xok) ? 0x100u
                               : m_l4 == CGPU_L4_UDP        ? 17u
                               : m_l4 == CGPU_L4_TCP        ? 6u
                               : m_l4 == CGPU_L4_ICMP       ? (v6 ? 58u : 1u)
                                                            : 0x100u)
                            : proto;
  const bool udp = lp == 17u && (a.accept & CGPU_F_ACCEPT_UDP);
  const bool tcp = !V4U && lp == 6u && (a.accept & CGPU_F_ACCEPT_TCP);
  // ProtocolNumbers::Icmpv4 (1) under IPv4, Icmpv6 (58) under IPv6 (ip/mod.rs:41-75)
  const bool icmp = !V4U && lp == (v6 ? 58u : 1u) && (a.accept & CGPU_F_ACCEPT_ICMP);
  const uint32_t l4_len = udp ? 8u : (icmp ? 4u : 20u);
  uint32_t st = CGPU_PKT_OK;
  bool eth_ok = false, l3_ok = false;
  if (len == 0u) {
    st = CGPU_PKT_ETH_BAD_OFFSET;
  } else if (len < eth_len) {  // covers len < 14 and len < header_len (:294-297)
    st = CGPU_PKT_ETH_OUT_OF_BUFFER;
  } else {
    eth_ok = true;
    if (!v4 && !v6) {
      const bool acc4 = a.accept & CGPU_F_ACCEPT_V4, acc6 = a.accept & CGPU_F_ACCEPT_V6;
      st = (acc4 && acc6) ? CGPU_PKT_NOT_IP : (acc4 ? CGPU_PKT_NOT_IPV4 : CGPU_PKT_NOT_IPV6);
    } else if (eth_len >= len) {
      st = CGPU_PKT_L3_BAD_OFFSET;
    } else if (eth_len + l3_len > len) {
      st = CGPU_PKT_L3_OUT_OF_BUFFER;
    } else {
      l3_ok = true;
      if (xst != 0u) {
        st = xst;
      } else if (!udp && !tcp && !icmp) {
        // exactly one accepted L4 type: its own error; several: NOT_L4
        const uint32_t acc = a.accept & (CGPU_F_ACCEPT_UDP | CGPU_F_ACCEPT_TCP | CGPU_F_ACCEPT_ICMP);
        st = acc == CGPU_F_ACCEPT_UDP    ? CGPU_PKT_NOT_UDP
             : acc == CGPU_F_ACCEPT_TCP  ? CGPU_PKT_NOT_TCP
             : acc == CGPU_F_ACCEPT_ICMP ? (v6 ? CGPU_PKT_NOT_ICMPV6 : CGPU_PKT_NOT_ICMPV4)
                                         : CGPU_PKT_NOT_L4;
      } else if (l4_off >= len) {
        st = CGPU_PKT_L4_BAD_OFFSET;
      } else if (l4_off + l4_len > len) {
        st = CGPU_PKT_L4_OUT_OF_BUFFER;
      }
    }
  }
  const bool l4_ok = st == CGPU_PKT_OK;
  const uint32_t span16 = (len - l4_off) & 0xffffu;  // Udp/Tcp::len(), the checksum span

  uint32_t meta = st;
  if (eth_ok) {
    meta |= eth_len << 8;
    if (k == 1u) meta |= CGPU_META_DOT1Q;
    if (k == 2u) meta |= CGPU_META_QINQ;
  }
  if (l3_ok) meta |= (v6 ? CGPU_L3_IPV6 : CGPU_L3_IPV4) << 16;
  if (l4_ok) meta |= (udp ? CGPU_L4_UDP : (icmp ? CGPU_L4_ICMP : CGPU_L4_TCP)) << 18;
  if (xok) meta |= xkind << 24;

  // L4 header dwords (L4 starts at normalized byte 34 for v4, 54 for v6)
  uint32_t U[5];
#pragma unroll
  for (int j = 0; j < 5; ++j)
    U[j] = xok ? XU[j] : __builtin_amdgcn_alignbyte(v6 ? Q[14 + j] : Q[9 + j], v6 ? Q[13 + j] : Q[8 + j], 2);

  uint32_t ip_c = 0, l4_c = 0;
  if (IPC && l3_ok && !v6) {
    // compute(0, 20-B header with the checksum zeroed) (v4.rs:322-333);
    // RECON: on the header with total_length := len (v4.rs:486-489)
    const uint32_t q4 = RECON ? ((Q[4] & 0xffff0000u) | swap16((len - eth_len) & 0xffffu)) : Q[4];
    uint32_t s = sad16(Q[3] & 0xffff0000u, 0u);
    s = sad16(q4, s);
    s = sad16(Q[5], s);
    s = sad16(Q[6] & 0xffff0000u, s);
    s = sad16(Q[7], s);
    s = sad16(Q[8] & 0xffffu, s);
    ip_c = (~swap16(fold32(s))) & 0xffffu;
    if (ip_c == swap16(Q[6] & 0xffffu)) meta |= CGPU_META_IP_CSUM_OK;
  }
  uint32_t s = 0, stored_le = 0, t_b = 0;
  bool has_tail = false;
  if (ROWS && L4C && l4_ok && (rows || stream)) {
    // the rows / stream paths: the same byte range's sum is the frame's word
    // sum minus the words before it (start = 22 or 26, + 4 per VLAN tag; even)
    const uint32_t start = (v6 ? 22u : 26u) + 4u * k;
    uint32_t pre = 0;
#pragma unroll
    for (int j = 0; j < 11; ++j) {
      const uint32_t lo = 4u * (uint32_t)j;
      pre = sad16(lo + 4u <= start ? P[j] : (lo < start ? (P[j] & 0xffffu) : 0u), pre);
    }
    s = s_all - pre;
    stored_le = udp    ? (v6 ? (Q[15] & 0xffffu) : (Q[10] & 0xffffu))
                : icmp ? (v6 ? (Q[14] & 0xffffu) : (Q[9] & 0xffffu))
                       : (v6 ? (Q[17] >> 16) : (Q[12] >> 16));
    s -= stored_le;
    if (icmp && !v6) s -= (Q[6] >> 16) + (Q[7] & 0xffffu) + (Q[7] >> 16) + (Q[8] & 0xffffu);
    // RECON: Udp::reconcile sets length := span before the checksum (udp.rs:350-354)
    if (RECON && udp) s += swap16(span16) - (v6 ? (Q[14] >> 16) : (Q[9] >> 16));
    has_tail = rows && len > kRowMaxLen;  // the rows summed bytes [0, kRowMaxLen)
    t_b = off + kRowMaxLen;               // 16-B aligned: rows frames are
  }
  if (L4C && l4_ok && (!(ROWS && (rows || stream)) || xok)) {
    // pseudo-header addresses + span [l4, len) (udp.rs:204-219, tcp.rs:
    // 462-477, checksum.rs:56-128) are one contiguous byte range: [26, len)
    // for v4, [22, len) for v6; the stored checksum field is subtracted.
    s = V4U ? 0u : sad16(v6 ? (Q[5] & 0xffff0000u) : 0u, 0u);
    s = sad16(v6 ? Q[6] : (Q[6] & 0xffff0000u), s);
    const uint32_t endn = len - 4u * k;  // normalized end of frame
    // A span longer than the window is split at a 16-B aligned arena offset:
    // the window sums up to it, the tail loop below sums whole chunks from it.
    const uint32_t wq = wlim - 4u * k < kQEnd ? wlim - 4u * k : kQEnd;  // normalized window limit
    const uint32_t wend = endn <= wq ? endn : wq - ((off + wq + 4u * k) & 15u);
    if (!__ballot(wend != __builtin_amdgcn_readfirstlane(wend))) {
      s = sum_to_end_s<7>(Q, __builtin_amdgcn_readfirstlane(wend), s);  // scalar masks
    } else {
      s = sum_to_end<7>(Q, wend, s);
    }
    stored_le = udp    ? (v6 ? (Q[15] & 0xffffu) : (Q[10] & 0xffffu))
                : icmp ? (v6 ? (Q[14] & 0xffffu) : (Q[9] & 0xffffu))
                       : (v6 ? (Q[17] >> 16) : (Q[12] >> 16));
    s -= stored_le;
    // ICMPv4 has no pseudo-header (icmp/v4/mod.rs:118-129): take the
    // addresses (bytes 26..33) back out of the exact sum
    if (icmp && !v6) s -= (Q[6] >> 16) + (Q[7] & 0xffffu) + (Q[7] >> 16) + (Q[8] & 0xffffu);
    if (RECON && udp) s += swap16(span16) - (v6 ? (Q[14] >> 16) : (Q[9] >> 16));
    has_tail = endn > wq;  // span continues past the window
    t_b = off + 4u * k + wend;  // where it continues (16-B aligned)
    if (xok) {
      // Behind an extension header: src + (segments[0] behind a routing
      // header, else dst) + the span [l4_off, len) read from memory.  Sums mod
      // 0xFFFF suffice here: the pseudo-header's length and protocol terms
      // added at the end are positive (always IPv6).
      uint32_t x = sad16(Q[5] & 0xffff0000u, 0u);  // src: normalized bytes 22..37
      x = sad16(Q[6], x);
      x = sad16(Q[7], x);
      x = sad16(Q[8], x);
      x = sad16(Q[9] & 0xffffu, x);
      if (xkind == CGPU_EXT_SRH) {
#pragma unroll
        for (int j = 0; j < 4; ++j) x = sad16(S0[j], x);
      } else {  // dst: normalized bytes 38..53
        x = sad16(Q[9] & 0xffff0000u, x);
        x = sad16(Q[10], x);
        x = sad16(Q[11], x);
        x = sad16(Q[12], x);
        x = sad16(Q[13] & 0xffffu, x);
      }
      uint32_t r = fold64(sum_abs(rs, a.arena_len, off + l4_off, off + len));
      if (off & 1u) r = swap16(r);  // absolute parity -> packet parity (l4_off is even)
      stored_le = udp ? (XU[1] >> 16) : (icmp ? (XU[0] >> 16) : (XU[4] & 0xffffu));
      s = x + r + (0xffffu - stored_le);
      if (RECON && udp) s += (0xffffu - (XU[1] & 0xffffu)) + swap16(span16);
      has_tail = false;
    }
  }
  // Hash and header record first: only the checksum state stays live across
  // the cooperative tail loop below (register pressure).
  // addresses as LE dwords of their wire bytes
  uint32_t src[4], dst[4];
  if (HASH || FIELDS) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      src[j] = __builtin_amdgcn_alignbyte(Q[6 + j], Q[5 + j], 2);   // v6: bytes 22..37
      dst[j] = __builtin_amdgcn_alignbyte(Q[10 + j], Q[9 + j], 2);  // v6: bytes 38..53
    }
    if (!v6) {
      src[0] = __builtin_amdgcn_alignbyte(Q[7], Q[6], 2);  // v4: bytes 26..29
      dst[0] = __builtin_amdgcn_alignbyte(Q[8], Q[7], 2);  // v4: bytes 30..33
    }
  }

  if (HASH) {
    uint64_t h = 0;
    if (l4_ok && !icmp) {  // Udp::flow / Tcp::flow (udp.rs:151-159, tcp.rs:409-417); ICMP has none
      // behind a routing header the flow's dst is SegmentRouting::dst() = segments[0]
      const bool sdst = xok && xkind == CGPU_EXT_SRH;
      const uint32_t fdst[4] = {sdst ? S0[0] : dst[0], sdst ? S0[1] : dst[1], sdst ? S0[2] : dst[2],
                                sdst ? S0[3] : dst[3]};
      h = flow_hash(v6, src, fdst, be16_lo(U[0]), be16_hi(U[0]), udp ? 17u : 6u);
    }
    if (valid) a.hash[i] = h;
  }

  if (FIELDS && valid) {
    uint32_t R[24];
#pragma unroll
    for (int j = 0; j < 24; ++j) R[j] = 0u;
    if (eth_ok) {
      R[0] = P[0];
      R[1] = P[1];
      R[2] = P[2];
      R[3] = ether_type | (eth_len << 16) | (k << 24);
    }
    if (l3_ok && !v6) {  // accessors ip/v4.rs:164-357
      const uint32_t vihl = (Q[3] >> 16) & 0xffu, de = Q[3] >> 24;
      R[4] = (vihl >> 4) | ((vihl & 0xfu) << 8) | ((de >> 2) << 16) | ((de & 3u) << 24);
      R[5] = be16_lo(Q[4]) | (be16_hi(Q[4]) << 16);
      const uint32_t ff = be16_lo(Q[5]);
      const uint32_t fl = ((ff & 0x4000u) ? 1u : 0u) | ((ff & 0x2000u) ? 2u : 0u);
      R[6] = fl | (((Q[5] >> 16) & 0xffu) << 8) | ((ff & 0x1fffu) << 16);
      R[7] = (Q[5] >> 24) | (be16_lo(Q[6]) << 16);
      R[10] = src[0];
      R[14] = dst[0];
    }
    if (l3_ok && v6) {  // accessors ip/v6/mod.rs:116-209
      const uint32_t w = be32(__builtin_amdgcn_alignbyte(Q[4], Q[3], 2));
      R[4] = (w >> 28) | (((w & 0x0fc00000u) >> 22) << 16) | (((w & 0x00300000u) >> 20) << 24);
      R[5] = be16_hi(Q[4]);
      R[6] = ((Q[5] >> 8) & 0xffu) << 8;
      R[7] = Q[5] & 0xffu;
      R[8] = w & 0xfffffu;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        R[10 + j] = src[j];
        R[14 + j] = dst[j];
      }
    }
    if (l4_ok && icmp) {  // msg_type, code, checksum (icmp/v4/mod.rs:88-112, v6 :93-117)
      R[18] = (U[0] & 0xffu) | (((U[0] >> 8) & 0xffu) << 16);
      R[19] = be16_hi(U[0]) << 16;
    } else if (l4_ok) {  // udp.rs:90-128, tcp.rs:139-405
      R[18] = be16_lo(U[0]) | (be16_hi(U[0]) << 16);
      if (udp) {
        R[19] = be16_lo(U[1]) | (be16_hi(U[1]) << 16);
      } else {
        R[19] = be16_hi(U[3]) | (be16_lo(U[4]) << 16);
        R[20] = be32(U[1]);
        R[21] = be32(U[2]);
        const uint32_t ons = U[3] & 0xffu, fl = (U[3] >> 8) & 0xffu;
        R[22] = (ons >> 4) | (fl << 8) | ((ons & 1u) << 16);
        R[23] = be16_hi(U[4]);
      }
    }
    u32x4 *out = reinterpret_cast<u32x4 *>(a.fields + i);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      u32x4 v = {R[4 * q], R[4 * q + 1], R[4 * q + 2], R[4 * q + 3]};
      out[q] = v;
    }
  }
  if (a.ext != nullptr && valid) {  // the extension record (cgpu_ext_record, 48 B)
    u32x4 e0 = {0u, 0u, 0u, 0u}, e1 = {0u, 0u, 0u, 0u}, e2 = {0u, 0u, 0u, 0u};
    if (xok) {
      const uint32_t nh = X0 & 0xffu;
      if (xkind == CGPU_EXT_SRH) {  // srh.rs:499-507
        e0[0] = xkind | (nh << 8) | (xhl << 16);
        e0[1] = X0 >> 8 | ((X1 & 0xffu) << 24);  // hdr_ext_len, routing_type, segments_left, last_entry
        e0[2] = ((X1 >> 8) & 0xffu) | (be16_hi(X1) << 16);  // flags, tag
        e1[2] = S0[0];
        e1[3] = S0[1];
        e2[0] = S0[2];
        e2[1] = S0[3];
      } else {  // fragment.rs:322-327: frag_res_m = offset << 3 | M
        const uint32_t frm = be16_hi(X0);
        e0[0] = xkind | (nh << 8) | (xhl << 16);
        e0[2] = (frm & 1u) << 8;
        e0[3] = frm >> 3;
        e1[0] = be32(X1);
      }
    }
    u32x4 *out = reinterpret_cast<u32x4 *>(a.ext + i);
    out[0] = e0;
    out[1] = e1;
    out[2] = e2;
  }
  if (L4C && __ballot(has_tail)) {
    // Tails: the span past the window, from the 16-B aligned offset t_b to
    // the frame end, summed in 16-B chunks by 16-lane rows (a row reads 256
    // contiguous bytes per load) and reduced per frame.
    const uint32_t t_to = off + len;
    const uint32_t lane = threadIdx.x & 63u, grp = lane >> 4, l16 = lane & 15u;
    uint32_t tail = 0;
    // the window line's rest (see the window loads): summed early, or now
    // (waves that took the general window loader)
    if (l0_adv != 0u && has_tail) {
      tail = l0_sum;
      t_b += l0_adv;
    }
    {
      const uint32_t lb = (t_b + 127u) & ~127u;
      const uint32_t nc = has_tail && l0_adv == 0u && len >= kLine0Min && lb < t_to ? (lb - t_b) >> 4 : 0u;
      if (__ballot(nc != 0u)) {
        u32x4 v[4];
#pragma unroll
        for (uint32_t j = 0; j < 4u; ++j)
          v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(j < nc ? t_b + 16u * j : kNoRead), 0, 0);
#pragma unroll
        for (uint32_t j = 0; j < 4u; ++j) tail = sum4(v[j], tail);  // zeros where not loaded
        t_b += 16u * (nc < 4u ? nc : 4u);
      }
    }
    const uint32_t pieces = has_tail ? (t_to - t_b + 255u) >> 8 : 0u;  // 256-B pieces
    const bool slot_tail = has_tail && pieces <= kSlotPieces;
    // every chunk any tail needs lies inside the arena: branch-free loads
    const bool fast = !__ballot(has_tail && (uint64_t)((t_to + 15u) & ~15u) > (uint64_t)a.arena_len);
    // Short tails (one or two 256-B pieces): pass p sums piece p of every
    // frame that has one.  The frames of a pass are compacted (ds_permute of
    // their piece offset and end to lane rank), and a round takes 16 of
    // them: row g sums slots g, 4 + g, 8 + g, 12 + g, one 16-B chunk per lane
    // and slot, so a lane has four loads in flight and a row reads 256
    // contiguous bytes.  A slot's row sum is formed with DPP row shifts and
    // added by its frame's lane; a frame's last chunk is masked at its end.
#pragma unroll
    for (uint32_t pass = 0; pass < kSlotPieces; ++pass) {
      const bool in = slot_tail && pieces > pass;
      const uint64_t mp = __ballot(in);
      if (!mp) break;
      const uint32_t n_f = (uint32_t)__builtin_popcountll(mp);
      const uint32_t rank =
          __builtin_amdgcn_mbcnt_hi((uint32_t)(mp >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mp, 0u));
      const int to_addr = (int)(4u * (in ? rank : 63u));  // frames to their rank; others to lane 63
      const uint32_t c_own = (uint32_t)__builtin_amdgcn_ds_permute(to_addr, (int)lane);
      const uint32_t c_b = (uint32_t)__builtin_amdgcn_ds_permute(to_addr, (int)(t_b + 256u * pass));
      const uint32_t c_e = (uint32_t)__builtin_amdgcn_ds_permute(to_addr, (int)t_to);
      for (uint32_t base = 0; base < n_f; base += 4u * kSlotIt) {
        uint32_t acc[kSlotIt];
#pragma unroll
        for (uint32_t it = 0; it < kSlotIt; ++it) {
          const uint32_t q = base + 4u * it + grp;
          const bool live = q < n_f;
          const uint32_t fb = __shfl(c_b, live ? q : 0u), ft = __shfl(c_e, live ? q : 0u);
          const uint32_t o = fb + 16u * l16;
          const bool need = live && o < ft;
          u32x4 v;
          if (fast) {
            v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(need ? o : kNoRead), 0, kNT);
          } else {
            v = u32x4{0u, 0u, 0u, 0u};
            if (need) v = load16(rs, o, a.arena_len);
          }
          const uint32_t rem = need ? ft - o : 16u;  // bytes of the chunk inside the frame
          if (__ballot(rem < 16u)) {
#pragma unroll
            for (uint32_t t = 0; t < 4u; ++t) {
              const uint32_t lo = 4u * t;
              v[t] &= rem >= lo + 4u ? 0xffffffffu : (rem <= lo ? 0u : 0xffffffffu >> (8u * (lo + 4u - rem)));
            }
          }
          uint32_t x = sum4(v, 0u);
          x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, true);  // row_shr:1
          x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, true);  // row_shr:2
          x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, true);  // row_shr:4
          x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, true);  // row_shr:8
          acc[it] = x;  // lane 16 g + 15 holds slot base + 4 it + g
        }
#pragma unroll
        for (uint32_t it = 0; it < kSlotIt; ++it)
#pragma unroll
          for (uint32_t g = 0; g < 4u; ++g) {
            const uint32_t q = base + 4u * it + g;
            if (q < n_f) {
              const uint32_t x = __builtin_amdgcn_readlane(acc[it], 16 * g + 15);
              if (lane == __builtin_amdgcn_readlane(c_own, q)) tail += x;
            }
          }
      }
    }
    // Long tails: 16-lane group j takes the (4r + j)-th long frame of the
    // wave in round r and walks it 1 KiB at a time, four loads 256 B apart in
    // flight; the row reduces and the owner lane picks its sum up with a
    // bpermute.
    const bool long_tail = has_tail && !slot_tail;
    const uint64_t mall = __ballot(long_tail);
    const uint32_t my_rank =
        __builtin_amdgcn_mbcnt_hi((uint32_t)(mall >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mall, 0u));
    uint64_t m = mall;
    for (uint32_t r = 0; m; ++r) {
      uint32_t own[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        own[u] = 64u;
        if (m) {
          own[u] = (uint32_t)__builtin_ctzll(m);
          m &= m - 1;
        }
      }
      const uint32_t mine = grp == 0u ? own[0] : (grp == 1u ? own[1] : (grp == 2u ? own[2] : own[3]));
      const bool active = mine < 64u;
      const uint32_t src = active ? mine : 0u;
      const uint32_t fr = __shfl(t_b, src), to = __shfl(t_to, src);
      uint32_t acc = 0;
      if (active) {
        const uint32_t ct = (to - 1u) & ~15u;
        for (uint32_t base = fr; base < to; base += 1024u) {
          u32x4 v[4];
#pragma unroll
          for (uint32_t it = 0; it < 4u; ++it) {
            const uint32_t o = base + 256u * it + 16u * l16;
            const bool need = o < to;
            if (fast) {
              v[it] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(need ? o : kNoRead), 0, kNT);
            } else {
              v[it] = u32x4{0u, 0u, 0u, 0u};
              if (need) v[it] = load16(rs, o, a.arena_len);
            }
          }
#pragma unroll
          for (uint32_t it = 0; it < 4u; ++it) acc = sum4(v[it], acc);
#pragma unroll
          for (uint32_t it = 0; it < 4u; ++it) {
            const uint32_t o = base + 256u * it + 16u * l16;
            if (o == ct) acc -= chunk_excess(v[it], o, fr, to);  // fr is chunk-aligned
          }
        }
      }
#pragma unroll
      for (uint32_t d = 8; d > 0; d >>= 1) acc += __shfl_xor(acc, d, 16);
      const bool mine_now = long_tail && my_rank >= 4u * r && my_rank < 4u * r + 4u;
      const uint32_t got = __shfl(acc, mine_now ? (my_rank - 4u * r) * 16u : 0u);
      if (mine_now) tail += got;
    }
    if (has_tail) {
      uint32_t rt = fold32(tail);
      if (off & 1u) rt = swap16(rt);  // absolute parity -> packet parity
      s += rt;
    }
  }
  if (L4C && l4_ok) {
    const uint32_t span = (len - l4_off) & 0xffffu;
    if (icmp && !v6) l4_c = (~swap16(fold32(s))) & 0xffffu;  // compute(0, span)
    else l4_c = (~fold32(swap16(fold32(s)) + span + (udp ? 17u : (icmp ? 58u : 6u)))) & 0xffffu;
    if (udp && l4_c == 0u) l4_c = 0xffffu;  // udp.rs:137-140
    if (l4_c == swap16(stored_le)) meta |= CGPU_META_L4_CSUM_OK;
  }

  if constexpr (RECON) {
    // reconcile_all from the held layer outward: L4 (udp.rs:350-354,
    // tcp.rs:619-621, icmp/v4/mod.rs:246, icmp/v6/mod.rs:260), the
    // extension header (nothing), then L3 (v4.rs:486-489, v6/mod.rs:331-334)
    // a frame not wholly inside the arena (a descriptor against the ABI's
    // precondition, or stale meta) is skipped, never written past the end
    const bool rec = valid && (uint64_t)off + len <= (uint64_t)a.arena_len &&
                     (L4C ? l4_ok
                                   : (a.depth >= CGPU_LAYER_L3 ? l3_ok : eth_ok && ((mi >> 8) & 0xffu) != 0u));
    // the fields reconcile writes: frame position and big-endian value, in
    // fixed slots (L4 first / second, L3 first / second; kNoField: none) so
    // that every index is a compile-time constant and the arrays stay in
    // registers
    constexpr uint32_t kNoField = 0xffffu;
    uint32_t fp[4] = {kNoField, kNoField, kNoField, kNoField}, fv[4] = {0u, 0u, 0u, 0u};
    if (rec) {
      if (L4C) {
        if (udp) {
          fp[0] = l4_off + 4u;
          fv[0] = span16;
          fp[1] = l4_off + 6u;
          fv[1] = l4_c;
        } else {
          fp[0] = l4_off + (tcp ? 16u : 2u);
          fv[0] = l4_c;
        }
      }
      if (a.depth >= CGPU_LAYER_L3) {
        if (v6) {
          fp[2] = eth_len + 4u;
          fv[2] = (len - eth_len - 40u) & 0xffffu;
        } else {
          fp[2] = eth_len + 2u;
          fv[2] = (len - eth_len) & 0xffffu;
          fp[3] = eth_len + 10u;
          fv[3] = ip_c;
        }
      }
    }
    uint8_t *f = a.wr_arena + off;
    bool stored = false;  // the fields below byte 64 went out with the whole 64 B
    // Whole waves only (every lane holds a packet: each lane stores chunks of
    // other lanes' frames).  A frame goes out this way if it is reconciled,
    // 16-B aligned and at least 64 B long; its first 64 B are the window P
    // with the fields patched in.
    const bool whole = rec && (off & 15u) == 0u && len >= 64u && (uint64_t)off + 64u <= a.arena_len;
    if (__builtin_amdgcn_read_exec() == ~0ull && __ballot(whole)) {
      // four rounds of 16 frames: lane l takes chunk l & 3 of the round's
      // frame l >> 2, patches the fields that fall into it (positions and
      // values from the frame's lane by shuffles) and stores it: one
      // instruction writes the first 64 B of 16 frames, whole sectors in
      // 64-B slots.  The chunk comes from the copy of the window the rows
      // variant staged in LDS (below the loads); the window variant re-reads
      // it (an L2 hit there: the window loaded that line a moment ago, while
      // a long frame's first line has left the L2 by the time its tail is
      // summed; keeping the window in registers through the sums spilled)
      const uint32_t lane = threadIdx.x & 63u;
      const uint64_t wm = __ballot(whole);
      uint32_t pf[4];  // field: position << 16 | big-endian value (none: 0xffff0000)
#pragma unroll
      for (uint32_t q = 0; q < 4u; ++q) pf[q] = whole && fp[q] < 64u ? (fp[q] << 16) | fv[q] : 0xffff0000u;
      const rsrc_t ws = make_rsrc(a.wr_arena, a.arena_len);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
      for (uint32_t r = 0; r < 4u; ++r) {
        const uint32_t fr = 16u * r + (lane >> 2), c = lane & 3u;  // the wave's frame, its chunk
        const uint32_t foff = (uint32_t)__shfl((int)off, (int)fr);
        const bool fw = (wm >> fr) & 1ull;
        u32x4 v;
        if (ROWS)
          v = *reinterpret_cast<const u32x4 *>(&rlds[threadIdx.x >> 6][16u * fr + 4u * c]);
        else
          v = __builtin_amdgcn_raw_buffer_load_b128(ws, (int)(fw ? foff + 16u * c : kNoRead), 0, 0);
#pragma unroll
        for (uint32_t q = 0; q < 4u; ++q) {
          const uint32_t f = (uint32_t)__shfl((int)pf[q], (int)fr), pos = f >> 16, val = swap16(f & 0xffffu);
#pragma unroll
          for (uint32_t j = 0; j < 4u; ++j)
            if (pos == 16u * c + 4u * j || pos == 16u * c + 4u * j + 2u)
              v[j] = (pos & 2u) ? ((v[j] & 0xffffu) | (val << 16)) : ((v[j] & 0xffff0000u) | val);
        }
        if (fw) __builtin_amdgcn_raw_buffer_store_b128(v, ws, (int)(foff + 16u * c), 0, 0);
      }
      stored = whole;
    }
    if (rec) {
      // the fields not yet stored (all of them, or those past byte 64: IPv6
      // behind tags, its TCP checksum)
#pragma unroll
      for (uint32_t q = 0; q < 4u; ++q)
        if (fp[q] != kNoField && (!stored || fp[q] >= 64u)) st16be(f + fp[q], fv[q]);
    }
    if (valid && a.rstatus != nullptr) a.rstatus[i] = rec ? CGPU_RECON_OK : CGPU_RECON_SKIPPED;
    return;
  }
  if (!valid) return;
  a.meta[i] = meta;
  if ((IPC || L4C) && a.csum != nullptr) a.csum[i] = ip_c | (l4_c << 16);

}

// The header-record (FIELDS) and extension (EXT) variants of the rows kernel,
// and the window kernel with both, hold more state than 64 VGPRs at 8 waves
// per SIMD and spilled 12-52 B per lane to scratch; they run at 6 (no spill).
template <bool IPC, bool L4C, bool HASH, bool FIELDS, bool EXT, bool V4U, bool ROWS, bool RECON = false>
__global__ __launch_bounds__(kBlock, ((ROWS && (FIELDS || EXT)) || (FIELDS && EXT)) ? 6 : 8) void parse_kernel(
    ParseArgs a) {
  parse_body<IPC, L4C, HASH, FIELDS, EXT, V4U, ROWS, RECON>(a);
}

// ---- reconcile_all of short frames without a re-parse ----------------------
// The general RECON body above runs the whole parse machinery again (window
// paths, classification, status chain) although the meta word already holds
// every layer and offset.  A wave whose reconciled frames are all 16-B
// aligned, at most 64 B long and of one layout (VLAN depth, IPv4/IPv6,
// UDP/TCP/ICMP) takes this path instead.  The layout is a compile-time
// constant, so every field position and sum range is fixed.  A quad of lanes
// holds a frame: in round r (four per wave) lane l loads 16-B chunk l & 3 of
// the wave's frame 16 r + l / 4, so one load instruction reads 1 KiB of
// consecutive 64-B slots in whole lines.  The quad writes the new length
// fields and zeroed checksum fields into its registers first (reconcile's
// order: udp.rs:350-354 sets the length before the checksum, v4.rs:486-489
// the total_length before the header checksum), sums the L4 span with the
// pseudo-header addresses and the IPv4 header over its four chunks (byte
// masks fixed per lane, a two-step DPP quad reduction), patches the checksums
// in, and stores the frame back whole, again 1 KiB per instruction.
// Measured (round 5, 1 Mi x 64 B, A/B on one box): 29.6 us, against 31.1 us
// storing only the chunks that hold a field, and 32.6 us with a lane per
// frame (four strided 16-B loads, the two field chunks stored); the in-place
// read-modify-write floor of the same bytes is 26.5 us (tools/launch_gap.hip).
// Frames in any other shape take the general body.

// Bytes of dword j that lie in [A, B) (compile-time bounds).
constexpr uint32_t range_mask(uint32_t j, uint32_t A, uint32_t B) {
  uint32_t m = 0;
  for (uint32_t b = 0; b < 4u; ++b)
    if (4u * j + b >= A && 4u * j + b < B) m |= 0xffu << (8u * b);
  return m;
}

__device__ __forceinline__ uint32_t sel_c(uint32_t c, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
  return c == 0u ? c0 : (c == 1u ? c1 : (c == 2u ? c2 : c3));
}

// dword j of the lane's chunk c: halfword at frame byte POS set to the wire
// bytes of v where that halfword falls in it
template <uint32_t POS>
__device__ __forceinline__ void quad_set_be16(u32x4 &x, uint32_t c, uint32_t v) {
  constexpr uint32_t j = (POS & 15u) / 4u;
  const uint32_t le = swap16(v & 0xffffu);
  const uint32_t y = (POS & 2u) ? ((x[j] & 0xffffu) | (le << 16)) : ((x[j] & 0xffff0000u) | le);
  x[j] = c == POS / 16u ? y : x[j];
}

__device__ __forceinline__ uint32_t quad_sum(uint32_t s) {
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0xb1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x4e, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
  return s;
}

template <uint32_t K, bool V6, uint32_t L4T>
__device__ __forceinline__ void recon_quad_frames(rsrc_t rs, rsrc_t ws, uint64_t rm, uint32_t off, uint32_t len) {
  constexpr uint32_t E = 14u + 4u * K;
  constexpr uint32_t L4 = E + (V6 ? 40u : 20u);
  constexpr bool UDP = L4T == CGPU_L4_UDP, TCP = L4T == CGPU_L4_TCP, ICMP4 = !V6 && L4T == CGPU_L4_ICMP;
  constexpr uint32_t CS = L4 + (UDP ? 6u : (TCP ? 16u : 2u));
  constexpr uint32_t A = ICMP4 ? L4 : (V6 ? E + 8u : E + 12u);
  constexpr uint32_t PROTO = UDP ? 17u : (TCP ? 6u : 58u);
  if constexpr (L4 + (UDP ? 8u : (TCP ? 20u : 4u)) > 64u) {
    return;
  } else {
  constexpr uint32_t IPCS = E + 10u;
  constexpr uint32_t F0 = V6 ? E + 4u : E + 2u, F1 = V6 ? E + 4u : IPCS, F2 = UDP ? L4 + 4u : CS, F3 = CS;
  const uint32_t lane = threadIdx.x & 63u, c = lane & 3u, q = lane >> 2;
  // the lane's byte masks of the two sums (its chunk is the same every round)
  uint32_t ml4[4], mip[4];
#pragma unroll
  for (uint32_t j = 0; j < 4u; ++j) {
    ml4[j] = sel_c(c, range_mask(j, A, 64u), range_mask(4u + j, A, 64u), range_mask(8u + j, A, 64u),
                   range_mask(12u + j, A, 64u));
    mip[j] = sel_c(c, range_mask(j, E, E + 20u), range_mask(4u + j, E, E + 20u), range_mask(8u + j, E, E + 20u),
                   range_mask(12u + j, E, E + 20u));
  }
  uint32_t foff[4], flen[4];
  bool frec[4];
  u32x4 v[4];
#pragma unroll
  for (uint32_t r = 0; r < 4u; ++r) {
    const uint32_t fr = 16u * r + q;
    foff[r] = (uint32_t)__shfl((int)off, (int)fr);
    flen[r] = (uint32_t)__shfl((int)len, (int)fr);
    frec[r] = (rm >> fr) & 1ull;
    v[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(frec[r] && 16u * c < flen[r] ? foff[r] + 16u * c : kNoRead),
                                                 0, kNT);
  }
#pragma unroll
  for (uint32_t r = 0; r < 4u; ++r) {
    u32x4 x = v[r];
    const uint32_t fl = flen[r], span = fl - L4;
    if constexpr (UDP) quad_set_be16<L4 + 4u>(x, c, span);
    quad_set_be16<CS>(x, c, 0u);
    if constexpr (V6) {
      quad_set_be16<E + 4u>(x, c, fl - E - 40u);
    } else {
      quad_set_be16<E + 2u>(x, c, fl - E);
      quad_set_be16<IPCS>(x, c, 0u);
    }
    uint32_t s = 0, si = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4u; ++j) {
      s = sad16(x[j] & ml4[j] & end_mask((int)(4u * c + j), fl), s);
      if constexpr (!V6) si = sad16(x[j] & mip[j], si);
    }
    s = quad_sum(s);
    uint32_t l4_c = ICMP4 ? (~swap16(fold32(s))) & 0xffffu : (~fold32(swap16(fold32(s)) + span + PROTO)) & 0xffffu;
    if (UDP && l4_c == 0u) l4_c = 0xffffu;  // udp.rs:137-140
    quad_set_be16<CS>(x, c, l4_c);
    if constexpr (!V6) {
      si = quad_sum(si);
      quad_set_be16<IPCS>(x, c, (~swap16(fold32(si))) & 0xffffu);
    }
    // the frame back whole: every chunk inside it as one 16-B store (a
    // chunk that runs past the frame's end stores only its fields, 2 B each)
    if (frec[r]) {
      if (16u * c + 16u <= fl) {
        __builtin_amdgcn_raw_buffer_store_b128(x, ws, (int)(foff[r] + 16u * c), 0, 0);
      } else {
        constexpr uint32_t F[4] = {F0, F1, F2, F3};
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k) {
          if (k > 0u && F[k] == F[k - 1u]) continue;
          if (c == F[k] / 16u) {
            const uint32_t w = x[(F[k] & 15u) / 4u];
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)((F[k] & 2u) ? w >> 16 : w), ws, (int)(foff[r] + F[k]),
                                                  0, 0);
          }
        }
      }
    }
  }
  }
}

template <uint32_t K, bool V4U>
__device__ __forceinline__ void recon_short_k(uint32_t lay, rsrc_t rs, rsrc_t ws, uint64_t rm, uint32_t off,
                                              uint32_t len) {
  if (V4U || lay == CGPU_L4_UDP) return recon_quad_frames<K, false, CGPU_L4_UDP>(rs, ws, rm, off, len);
  if constexpr (!V4U) {
    switch (lay) {
      case CGPU_L4_TCP: return recon_quad_frames<K, false, CGPU_L4_TCP>(rs, ws, rm, off, len);
      case CGPU_L4_ICMP: return recon_quad_frames<K, false, CGPU_L4_ICMP>(rs, ws, rm, off, len);
      case 4u | CGPU_L4_UDP: return recon_quad_frames<K, true, CGPU_L4_UDP>(rs, ws, rm, off, len);
      case 4u | CGPU_L4_TCP: return recon_quad_frames<K, true, CGPU_L4_TCP>(rs, ws, rm, off, len);
      default: return recon_quad_frames<K, true, CGPU_L4_ICMP>(rs, ws, rm, off, len);
    }
  }
}

// The short path at depth L4 (wave-uniform decision).  Returns false when
// the wave has to take the general body; otherwise its frames are done.
template <bool EXT, bool V4U>
__device__ __forceinline__ bool recon_short(const ParseArgs &a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const bool valid = i < a.n;
  const uint64_t nb = (uint64_t)a.n;
  const rsrc_t r_off = make_rsrc(a.off, (uint32_t)(4u * nb < 0xffffffffull ? 4u * nb : 0xffffffffull));
  const rsrc_t r_len = make_rsrc(a.len, (uint32_t)(2u * nb < 0xffffffffull ? 2u * nb : 0xffffffffull));
  const rsrc_t r_meta = make_rsrc(a.meta_in, (uint32_t)(4u * nb < 0xffffffffull ? 4u * nb : 0xffffffffull));
  const uint32_t off = __builtin_amdgcn_raw_buffer_load_b32(r_off, (int)(4u * i), 0, 0);
  const uint32_t len = __builtin_amdgcn_raw_buffer_load_b16(r_len, (int)(2u * i), 0, 0);
  const uint32_t mi = __builtin_amdgcn_raw_buffer_load_b32(r_meta, (int)(4u * i), 0, 0);
  const uint32_t k = (mi & CGPU_META_QINQ) ? 2u : ((mi & CGPU_META_DOT1Q) ? 1u : 0u);
  const uint32_t m_l3 = (mi >> 16) & 3u, m_l4 = (mi >> 18) & 3u, m_x = (mi >> 24) & 3u;
  const bool okst = (mi & 0xffu) == CGPU_PKT_OK;
  // frames behind an IPv6 extension header: the general body (EXT), or not
  // a packet of the pipeline (no CGPU_F_V6_EXT: no L4 behind the extension)
  if (EXT && __ballot(valid && okst && m_x != CGPU_EXT_NONE)) return false;
  // parse_body's reconcile predicate at depth L4: the meta's layers, each in
  // the accept set, and read_data's bounds (mbuf.rs:313-327) on this length
  const bool v4 = m_l3 == CGPU_L3_IPV4 && (a.accept & CGPU_F_ACCEPT_V4);
  const bool v6 = !V4U && m_l3 == CGPU_L3_IPV6 && (a.accept & CGPU_F_ACCEPT_V6);
  const bool l4in = okst && m_x == CGPU_EXT_NONE;
  const bool udp = l4in && m_l4 == CGPU_L4_UDP && (a.accept & CGPU_F_ACCEPT_UDP);
  const bool tcp = !V4U && l4in && m_l4 == CGPU_L4_TCP && (a.accept & CGPU_F_ACCEPT_TCP);
  const bool icmp = !V4U && l4in && m_l4 == CGPU_L4_ICMP && (a.accept & CGPU_F_ACCEPT_ICMP);
  const uint32_t l4_end = 14u + 4u * k + (v6 ? 40u : 20u) + (udp ? 8u : (icmp ? 4u : 20u));
  const bool rec = valid && (v4 || v6) && (udp || tcp || icmp) && l4_end <= len &&
                   (uint64_t)off + len <= (uint64_t)a.arena_len;
  const bool fit = (off & 15u) == 0u && len <= 64u && (uint64_t)off + 64u <= (uint64_t)a.arena_len;
  if (__ballot(rec && !fit)) return false;
  const uint64_t rm = __ballot(rec);
  const uint32_t lay = (k << 3) | (v6 ? 4u : 0u) | m_l4;
  const uint32_t rl = rm ? (uint32_t)__builtin_ctzll(rm) : 0u;
  const uint32_t lay0 = __builtin_amdgcn_readlane(lay, (int)rl);
  if (__ballot(rec && lay != lay0)) return false;
  if (rm) {
    const rsrc_t rs = make_rsrc(a.arena, a.arena_len);
    const rsrc_t ws = make_rsrc(a.wr_arena, a.arena_len);
    switch (lay0 >> 3) {
      case 0u: recon_short_k<0u, V4U>(lay0 & 7u, rs, ws, rm, off, len); break;
      case 1u: recon_short_k<1u, V4U>(lay0 & 7u, rs, ws, rm, off, len); break;
      default: recon_short_k<2u, V4U>(lay0 & 7u, rs, ws, rm, off, len); break;
    }
  }
  if (valid && a.rstatus != nullptr) a.rstatus[i] = rec ? CGPU_RECON_OK : CGPU_RECON_SKIPPED;
  return true;
}

// The reconcile kernels: the same body with their own occupancy targets
// (workgroups of 256 per CU).  The window variant (short frames: every
// frame's sector is read and written back in place) runs at 6; a round-4
// A/B against 8 (45.95 against 50.5 us at 1 Mi x 64 B) was within that
// launch's run-to-run spread (44.9-50.0 us for 6 on one box), and with the
// short path 6 and 8 time the same (32.6 us, round 5).  The rows variant
// (IMIX) ran at 8 (126.2 us against 128.5 us at 6, round 4, one box) but
// spilled 12-24 B per lane to scratch there; it runs at 7, where it does not
// (no kernel of the library uses scratch memory: a launch whose scratch
// need differs from the one before it makes the runtime re-size the queue's
// scratch).
template <bool L4C, bool EXT, bool V4U>
__global__ __launch_bounds__(kBlock, 6) void recon_kernel(ParseArgs a) {
  if constexpr (L4C) {
    if (recon_short<EXT, V4U>(a)) return;
  }
  parse_body<true, L4C, false, false, EXT, V4U, false, true>(a);
}
template <bool L4C, bool EXT, bool V4U>
__global__ __launch_bounds__(kBlock, 7) void recon_rows_kernel(ParseArgs a) {
  parse_body<true, L4C, false, false, EXT, V4U, true, true>(a);
}

// The rows path is compiled into a variant that the checksum configs get when
// the batch's mean slot (arena bytes per packet) is 128..2200 B: long frames,
// but not jumbo ones; each wave still decides by its own frames.
bool rows_variant(const ParseArgs &a) {
  const uint64_t mean = (uint64_t)a.arena_len / a.n;
  return mean >= 128u && mean <= kRowsMeanMax;
}

// The launch of a rows kernel: sched_n / 256 workgroups more (they order the
// waves) when the host gave it a schedule buffer.
uint32_t rows_grid(const ParseArgs &a) {
  return (a.n + kBlock - 1) / kBlock + (a.sched != nullptr ? a.sched_n / kBlock : 0u);
}

template <bool IPC, bool L4C, bool HASH, bool FIELDS, bool EXT, bool V4U>
hipError_t launch_t(const ParseArgs &a, hipStream_t s) {
  if (L4C && rows_variant(a)) {
    hipLaunchKernelGGL((parse_kernel<IPC, L4C, HASH, FIELDS, EXT, V4U, true>), dim3(rows_grid(a)), dim3(kBlock), 0,
                       s, a);
  } else {
    ParseArgs b = a;
    b.sched = nullptr;
    hipLaunchKernelGGL((parse_kernel<IPC, L4C, HASH, FIELDS, EXT, V4U, false>), dim3((a.n + kBlock - 1) / kBlock),
                       dim3(kBlock), 0, s, b);
  }
  return hipGetLastError();
}

template <bool IPC, bool L4C, bool HASH, bool FIELDS>
hipError_t launch_e(const ParseArgs &a, bool ext, hipStream_t s) {
  if (ext) return launch_t<IPC, L4C, HASH, FIELDS, true, false>(a, s);
  // IPv4/UDP only (no header record): the monomorphised variant
  constexpr uint32_t kNotV4U = CGPU_F_ACCEPT_V6 | CGPU_F_ACCEPT_TCP | CGPU_F_ACCEPT_ICMP;
  if (!FIELDS && !(a.accept & kNotV4U)) return launch_t<IPC, L4C, HASH, FIELDS, false, !FIELDS>(a, s);
  return launch_t<IPC, L4C, HASH, FIELDS, false, false>(a, s);
}

template <bool IPC, bool L4C, bool HASH>
hipError_t launch_f(const ParseArgs &a, bool fields, bool ext, hipStream_t s) {
  return fields ? launch_e<IPC, L4C, HASH, true>(a, ext, s) : launch_e<IPC, L4C, HASH, false>(a, ext, s);
}

template <bool IPC, bool L4C>
hipError_t launch_h(const ParseArgs &a, bool hash, bool fields, bool ext, hipStream_t s) {
  return hash ? launch_f<IPC, L4C, true>(a, fields, ext, s) : launch_f<IPC, L4C, false>(a, fields, ext, s);
}

template <bool L4C, bool EXT, bool V4U>
hipError_t launch_recon_t(const ParseArgs &a, hipStream_t s) {
  if (L4C && rows_variant(a)) {
    hipLaunchKernelGGL((recon_rows_kernel<L4C, EXT, V4U>), dim3(rows_grid(a)), dim3(kBlock), 0, s, a);
  } else {
    ParseArgs b = a;
    b.sched = nullptr;
    hipLaunchKernelGGL((recon_kernel<L4C, EXT, V4U>), dim3((a.n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, b);
  }
  return hipGetLastError();
}

template <bool L4C>
hipError_t launch_recon_l(const ParseArgs &a, hipStream_t s) {
  if (a.accept & CGPU_F_V6_EXT) return launch_recon_t<L4C, true, false>(a, s);
  constexpr uint32_t kNotV4U = CGPU_F_ACCEPT_V6 | CGPU_F_ACCEPT_TCP | CGPU_F_ACCEPT_ICMP;
  if (!(a.accept & kNotV4U)) return launch_recon_t<L4C, false, true>(a, s);
  return launch_recon_t<L4C, false, false>(a, s);
}

}  // namespace

hipError_t launch_reconcile(const ParseArgs &a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  return a.depth >= CGPU_LAYER_L4 ? launch_recon_l<true>(a, s) : launch_recon_l<false>(a, s);
}

hipError_t launch_parse(const ParseArgs &a, uint32_t flags, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  const bool ipc = flags & CGPU_F_CSUM_IP, l4c = flags & CGPU_F_CSUM_L4;
  const bool hash = flags & CGPU_F_FLOW_HASH, fields = a.fields != nullptr;
  const bool ext = flags & CGPU_F_V6_EXT;  // the extension path is compiled out otherwise
  if (ipc) {
    return l4c ? launch_h<true, true>(a, hash, fields, ext, s) : launch_h<true, false>(a, hash, fields, ext, s);
  }
  return l4c ? launch_h<false, true>(a, hash, fields, ext, s) : launch_h<false, false>(a, hash, fields, ext, s);
}

}  // namespace cgpu
