// parse.hip — batched Ethernet -> IPv4/IPv6 -> UDP/TCP parse, Internet
// checksums and 5-tuple flow hash on gfx950.
//
// One packet per lane.  Each lane pulls a 96-byte packet-relative window
// into VGPRs (buffer_load_dwordx4 + v_alignbyte, so any arena offset works),
// parses every header from registers, sums the L4 span from the same
// registers and streams only the bytes beyond the window.  Outputs are SoA:
// a u32 meta word, a u32 (ip_csum | l4_csum << 16), a u64 flow hash and an
// optional 96-byte header record.
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
#include "capsule_gpu.h"
#include "device_common.hpp"
#include "kernels.hpp"

namespace cgpu {

namespace {

constexpr int kWinDw = 24;  // 96-byte register window
constexpr uint32_t kBlock = 256;

__device__ __forceinline__ uint32_t sel3(uint32_t k, uint32_t a, uint32_t b, uint32_t c) {
  return k == 0u ? a : (k == 1u ? b : c);
}

template <bool IPC, bool L4C, bool HASH, bool FIELDS>
__global__ __launch_bounds__(kBlock) void parse_kernel(ParseArgs a) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.n) return;
  const rsrc_t rs = make_rsrc(a.arena, a.arena_len);
  const uint32_t off = a.off[i];
  const uint32_t len = a.len[i];

  uint32_t P[kWinDw];
  load_window<kWinDw>(rs, a.arena_len, off, len < 96u ? len : 96u, P);

  // --- Ethernet: VLAN marker at bytes 12-13 (ethernet.rs:164-181) ---------
  const uint32_t marker = be16_lo(P[3]);
  const uint32_t k = marker == 0x8100u ? 1u : (marker == 0x88a8u ? 2u : 0u);
  const uint32_t eth_len = 14u + 4u * k;  // header_len (ethernet.rs:253-261)
  const uint32_t ether_type = be16_lo(sel3(k, P[3], P[4], P[5]));

  // L[j] = L3-relative dword j (packet bytes eth_len + 4j ...): realign by
  // 2 bytes, then shift by k dwords for the VLAN tags.
  uint32_t A[20];
#pragma unroll
  for (int j = 0; j < 20; ++j) A[j] = __builtin_amdgcn_alignbyte(P[4 + j], P[3 + j], 2);
  uint32_t L[18];
#pragma unroll
  for (int j = 0; j < 18; ++j) L[j] = sel3(k, A[j], A[j + 1], A[j + 2]);

  // --- status: the first failing step of the reference chain --------------
  uint32_t st = CGPU_PKT_OK;
  uint32_t l3 = CGPU_L3_NONE, l4 = CGPU_L4_NONE;
  bool eth_ok = false, l3_ok = false;
  const bool v4 = ether_type == 0x0800u && (a.accept & CGPU_F_ACCEPT_V4);
  const bool v6 = ether_type == 0x86ddu && (a.accept & CGPU_F_ACCEPT_V6);
  const uint32_t l3_len = v6 ? 40u : 20u;
  const uint32_t proto = v6 ? ((L[1] >> 16) & 0xffu) : ((L[2] >> 8) & 0xffu);
  const bool udp = proto == 17u && (a.accept & CGPU_F_ACCEPT_UDP);
  const bool tcp = proto == 6u && (a.accept & CGPU_F_ACCEPT_TCP);
  const uint32_t l4_off = eth_len + l3_len;
  const uint32_t l4_len = udp ? 8u : 20u;
  if (len == 0u) {
    st = CGPU_PKT_ETH_BAD_OFFSET;
  } else if (len < eth_len) {  // covers len < 14 and len < header_len
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
      l3 = v6 ? CGPU_L3_IPV6 : CGPU_L3_IPV4;
      if (!udp && !tcp) {
        const bool au = a.accept & CGPU_F_ACCEPT_UDP, at = a.accept & CGPU_F_ACCEPT_TCP;
        st = (au && at) ? CGPU_PKT_NOT_L4 : (au ? CGPU_PKT_NOT_UDP : CGPU_PKT_NOT_TCP);
      } else if (l4_off >= len) {
        st = CGPU_PKT_L4_BAD_OFFSET;
      } else if (l4_off + l4_len > len) {
        st = CGPU_PKT_L4_OUT_OF_BUFFER;
      } else {
        l4 = udp ? CGPU_L4_UDP : CGPU_L4_TCP;
      }
    }
  }
  const bool l4_ok = st == CGPU_PKT_OK;

  // U[j] = L4-relative dword j.
  uint32_t U[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) U[j] = v6 ? L[10 + j] : L[5 + j];

  uint32_t meta = st;
  if (eth_ok) {
    meta |= eth_len << 8;
    if (k == 1u) meta |= CGPU_META_DOT1Q;
    if (k == 2u) meta |= CGPU_META_QINQ;
  }
  meta |= l3 << 16;
  meta |= l4 << 18;

  uint32_t ip_c = 0, l4_c = 0;
  if (IPC && l3_ok && !v6) {
    // compute(0, header with checksum zeroed): LE residue, swap to BE order.
    const uint64_t s = (uint64_t)L[0] + L[1] + (L[2] & 0xffffu) + L[3] + L[4];
    ip_c = (~swap16(fold64(s))) & 0xffffu;
    if (ip_c == be16_hi(L[2])) meta |= CGPU_META_IP_CSUM_OK;
  }
  if (L4C && l4_ok) {
    const uint32_t l4dw = v6 ? 10u : 5u;
    const uint32_t end = len - eth_len;  // L3-relative end of the span
    const uint32_t cs_dw = udp ? l4dw + 1u : l4dw + 4u;
    const uint32_t cs_keep = udp ? 0x0000ffffu : 0xffff0000u;
    uint64_t acc = 0;
#pragma unroll
    for (int j = 5; j < 18; ++j) {
      uint32_t m = ((uint32_t)j >= l4dw) ? end_mask(j, end) : 0u;
      if ((uint32_t)j == cs_dw) m &= cs_keep;
      acc += (uint64_t)(L[j] & m);
    }
    if (len > eth_len + 72u) {  // span continues past the register window
      uint32_t rt = fold64(sum_abs(rs, a.arena_len, off + eth_len + 72u, off + len));
      if (off & 1u) rt = swap16(rt);  // absolute parity -> packet parity
      acc += rt;
    }
    const uint32_t sum_be = swap16(fold64(acc));
    const uint32_t span = (len - l4_off) & 0xffffu;
    const uint32_t pr = udp ? 17u : 6u;
    uint32_t ph;
    if (v6) {
      const uint64_t as = (uint64_t)L[2] + L[3] + L[4] + L[5] + L[6] + L[7] + L[8] + L[9];
      ph = fold32(swap16(fold64(as)) + span + pr);
    } else {
      const uint32_t src = be32(L[3]), dst = be32(L[4]);
      ph = fold32((src >> 16) + (src & 0xffffu) + (dst >> 16) + (dst & 0xffffu) + pr + span);
    }
    l4_c = (~fold32(ph + sum_be)) & 0xffffu;
    if (udp && l4_c == 0u) l4_c = 0xffffu;  // udp.rs:137-140
    const uint32_t stored = udp ? be16_hi(U[1]) : be16_lo(U[4]);
    if (l4_c == stored) meta |= CGPU_META_L4_CSUM_OK;
  }

  a.meta[i] = meta;
  if (IPC || L4C) a.csum[i] = ip_c | (l4_c << 16);

  if (HASH) {
    uint64_t h = 0;
    if (l4_ok) {
      const uint32_t sport = be16_lo(U[0]), dport = be16_hi(U[0]);
      const uint32_t pr = udp ? 17u : 6u;  // layer constant (udp.rs:157, tcp.rs:415)
      if (v6) {
        const uint32_t s6[4] = {L[2], L[3], L[4], L[5]};
        const uint32_t d6[4] = {L[6], L[7], L[8], L[9]};
        h = flow_hash_v6(s6, d6, sport, dport, pr);
      } else {
        h = flow_hash_v4(L[3], L[4], sport, dport, pr);
      }
    }
    a.hash[i] = h;
  }

  if (FIELDS) {
    uint32_t R[24];
#pragma unroll
    for (int j = 0; j < 24; ++j) R[j] = 0u;
    if (eth_ok) {
      R[0] = P[0];
      R[1] = P[1];
      R[2] = P[2];
      R[3] = ether_type | (eth_len << 16) | (k << 24);
    }
    if (l3_ok && !v6) {
      const uint32_t vihl = L[0] & 0xffu, de = (L[0] >> 8) & 0xffu;
      R[4] = (vihl >> 4) | ((vihl & 0xfu) << 8) | ((de >> 2) << 16) | ((de & 3u) << 24);
      R[5] = be16_hi(L[0]) | (be16_lo(L[1]) << 16);
      const uint32_t ff = be16_hi(L[1]);
      const uint32_t fl = ((ff & 0x4000u) ? 1u : 0u) | ((ff & 0x2000u) ? 2u : 0u);
      R[6] = fl | ((L[2] & 0xffu) << 8) | ((ff & 0x1fffu) << 16);
      R[7] = ((L[2] >> 8) & 0xffu) | (be16_hi(L[2]) << 16);
      R[10] = L[3];
      R[14] = L[4];
    }
    if (l3_ok && v6) {
      const uint32_t w = be32(L[0]);
      R[4] = (w >> 28) | (((w & 0x0fc00000u) >> 22) << 16) | (((w & 0x00300000u) >> 20) << 24);
      R[5] = be16_lo(L[1]);
      R[6] = (L[1] >> 24) << 8;
      R[7] = (L[1] >> 16) & 0xffu;
      R[8] = w & 0xfffffu;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        R[10 + j] = L[2 + j];
        R[14 + j] = L[6 + j];
      }
    }
    if (l4_ok) {
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
    u32x4 *dst = reinterpret_cast<u32x4 *>(a.fields + i);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      u32x4 v = {R[4 * q], R[4 * q + 1], R[4 * q + 2], R[4 * q + 3]};
      dst[q] = v;
    }
  }
}

template <bool IPC, bool L4C, bool HASH, bool FIELDS>
hipError_t launch_t(const ParseArgs &a, hipStream_t s) {
  const uint32_t grid = (a.n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL((parse_kernel<IPC, L4C, HASH, FIELDS>), dim3(grid), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

template <bool IPC, bool L4C, bool HASH>
hipError_t launch_f(const ParseArgs &a, bool fields, hipStream_t s) {
  return fields ? launch_t<IPC, L4C, HASH, true>(a, s) : launch_t<IPC, L4C, HASH, false>(a, s);
}

template <bool IPC, bool L4C>
hipError_t launch_h(const ParseArgs &a, bool hash, bool fields, hipStream_t s) {
  return hash ? launch_f<IPC, L4C, true>(a, fields, s) : launch_f<IPC, L4C, false>(a, fields, s);
}

}  // namespace

hipError_t launch_parse(const ParseArgs &a, uint32_t flags, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  const bool ipc = flags & CGPU_F_CSUM_IP, l4c = flags & CGPU_F_CSUM_L4;
  const bool hash = flags & CGPU_F_FLOW_HASH, fields = a.fields != nullptr;
  if (ipc) {
    return l4c ? launch_h<true, true>(a, hash, fields, s) : launch_h<true, false>(a, hash, fields, s);
  }
  return l4c ? launch_h<false, true>(a, hash, fields, s) : launch_h<false, false>(a, hash, fields, s);
}

}  // namespace cgpu
