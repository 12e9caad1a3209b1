/*
 * oracle.c — scalar CPU restatement of Capsule's packet hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  It is the parity checker for the
 * HIP kernels and the "port" CPU baseline of bench.py; nothing under
 * capsule_amd/ links or calls it.
 *
 * Every routine restates the reference Rust step by step, deliberately in the
 * reference's own shape (one u16 word per loop iteration, memmove-based
 * shrink/extend on a simulated rte_mbuf), NOT in the GPU kernels' shape
 * (dword residues in registers), so that agreement between the two is
 * evidence rather than a tautology.  File:line citations are relative to
 * /root/reference.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

/* ---- core/src/packets/types.rs:40-50,124-134 (u16be / u32be) ------------ */
static uint16_t rd16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
static uint32_t rd32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static void wr16(uint8_t *p, uint16_t v) {
  p[0] = (uint8_t)(v >> 8);
  p[1] = (uint8_t)v;
}

/* ---- core/src/packets/checksum.rs:145-168 `compute` ---------------------- */
uint16_t or_compute(uint16_t pseudo_header_sum, const uint8_t *payload, size_t len) {
  uint32_t checksum = pseudo_header_sum;
  size_t n = len;
  if (len % 2 > 0) { /* odd # of bytes: last byte padded (:152-155) */
    checksum += (uint32_t)payload[len - 1] << 8;
    n = len - 1;
  }
  for (size_t i = 0; i < n; i += 2) /* u16::from_be per word (:157-162) */
    checksum += rd16(payload + i);
  while (checksum >> 16 != 0) checksum = (checksum >> 16) + (checksum & 0xFFFF);
  return (uint16_t)~(uint16_t)checksum;
}

/* ---- checksum.rs:182-195 `compute_inc` (RFC 1624) ------------------------ */
uint16_t or_compute_inc(uint16_t old_checksum, const uint16_t *old_value,
                        const uint16_t *new_value, size_t n) {
  uint32_t checksum = (uint16_t)~old_checksum;
  for (size_t i = 0; i < n; ++i)
    checksum += (uint32_t)(uint16_t)~old_value[i] + (uint32_t)new_value[i];
  while (checksum >> 16 != 0) checksum = (checksum >> 16) + (checksum & 0xFFFF);
  return (uint16_t)~(uint16_t)checksum;
}

/* ---- checksum.rs:56-77 PseudoHeader::sum + v4_csum :93-103 --------------- */
uint16_t or_pseudo_v4(uint32_t src, uint32_t dst, uint16_t packet_len, uint8_t protocol) {
  uint32_t sum = (src >> 16) + (src & 0xFFFF) + (dst >> 16) + (dst & 0xFFFF) + protocol +
                 packet_len;
  while (sum >> 16 != 0) sum = (sum >> 16) + (sum & 0xFFFF);
  return (uint16_t)sum;
}

/* ---- checksum.rs:56-77 + v6_csum :123-128 (Ipv6Addr::segments) ----------- */
uint16_t or_pseudo_v6(const uint8_t src[16], const uint8_t dst[16], uint16_t packet_len,
                      uint8_t protocol) {
  uint32_t sum = 0;
  for (int s = 0; s < 8; ++s) sum += rd16(src + 2 * s);
  for (int s = 0; s < 8; ++s) sum += rd16(dst + 2 * s);
  sum += packet_len;
  sum += protocol;
  while (sum >> 16 != 0) sum = (sum >> 16) + (sum & 0xFFFF);
  return (uint16_t)sum;
}

/* ---- SipHash-c-d (Aumasson & Bernstein 2012), Rust std sip.rs layout ----- */
#define ROTL(x, b) (uint64_t)(((x) << (b)) | ((x) >> (64 - (b))))
static void sipround(uint64_t *v0, uint64_t *v1, uint64_t *v2, uint64_t *v3) {
  *v0 += *v1; *v1 = ROTL(*v1, 13); *v1 ^= *v0; *v0 = ROTL(*v0, 32);
  *v2 += *v3; *v3 = ROTL(*v3, 16); *v3 ^= *v2;
  *v0 += *v3; *v3 = ROTL(*v3, 21); *v3 ^= *v0;
  *v2 += *v1; *v1 = ROTL(*v1, 17); *v1 ^= *v2; *v2 = ROTL(*v2, 32);
}

uint64_t or_siphash(int c_rounds, int d_rounds, uint64_t k0, uint64_t k1, const uint8_t *msg,
                    size_t len) {
  uint64_t v0 = k0 ^ 0x736f6d6570736575ull, v1 = k1 ^ 0x646f72616e646f6dull;
  uint64_t v2 = k0 ^ 0x6c7967656e657261ull, v3 = k1 ^ 0x7465646279746573ull;
  size_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint64_t m = 0;
    for (int b = 0; b < 8; ++b) m |= (uint64_t)msg[i + b] << (8 * b);
    v3 ^= m;
    for (int r = 0; r < c_rounds; ++r) sipround(&v0, &v1, &v2, &v3);
    v0 ^= m;
  }
  uint64_t b = ((uint64_t)len & 0xff) << 56;
  for (size_t t = 0; i + t < len; ++t) b |= (uint64_t)msg[i + t] << (8 * t);
  v3 ^= b;
  for (int r = 0; r < c_rounds; ++r) sipround(&v0, &v1, &v2, &v3);
  v0 ^= b;
  v2 ^= 0xff;
  for (int r = 0; r < d_rounds; ++r) sipround(&v0, &v1, &v2, &v3);
  return v0 ^ v1 ^ v2 ^ v3;
}

/* Byte stream of `#[derive(Hash)] struct Flow` (core/src/packets/ip/mod.rs:
 * 142-150) as Rust 1.50 std feeds a Hasher on x86-64:
 *   IpAddr: discriminant as isize (8 B LE; V4 = 0, V6 = 1), then
 *     Ipv4Addr -> s_addr.hash() = write_u32 of the in-memory (wire-order) bytes,
 *     Ipv6Addr -> s6_addr.hash() = [u8;16] slice: write_usize(16) + 16 bytes;
 *   src_port, dst_port: write_u16 (2 B LE); protocol: ProtocolNumber(u8).  */
static size_t put_le(uint8_t *o, uint64_t v, int n) {
  for (int i = 0; i < n; ++i) o[i] = (uint8_t)(v >> (8 * i));
  return (size_t)n;
}

size_t or_flow_bytes(int v6, const uint8_t *src, const uint8_t *dst, uint16_t src_port,
                     uint16_t dst_port, uint8_t protocol, uint8_t out[69]) {
  size_t k = 0;
  const uint8_t *addr[2] = {src, dst};
  for (int a = 0; a < 2; ++a) {
    k += put_le(out + k, v6 ? 1 : 0, 8);
    if (v6) {
      k += put_le(out + k, 16, 8);
      memcpy(out + k, addr[a], 16);
      k += 16;
    } else {
      memcpy(out + k, addr[a], 4);
      k += 4;
    }
  }
  k += put_le(out + k, src_port, 2);
  k += put_le(out + k, dst_port, 2);
  out[k++] = protocol;
  return k;
}

uint64_t or_flow_hash(int v6, const uint8_t *src, const uint8_t *dst, uint16_t src_port,
                      uint16_t dst_port, uint8_t protocol) {
  uint8_t buf[69];
  size_t n = or_flow_bytes(v6, src, dst, src_port, dst_port, protocol, buf);
  /* std::collections::hash_map::DefaultHasher::new() = SipHasher13, key 0 */
  return or_siphash(1, 3, 0, 0, buf, n);
}

/* ---- a simulated single-segment rte_mbuf (core/src/dpdk/mbuf.rs) --------- */
#define MBUF_HEADROOM 128u  /* RTE_PKTMBUF_HEADROOM */
/* buf_len of the simulated mbufs: 2048 data room + headroom
 * (bindings_rustdoc.rs:561) unless a test models a custom mempool
 * (or_set_mbuf_data_room) */
static uint32_t g_buf_len = 2176u;

void or_set_mbuf_data_room(uint32_t room) { g_buf_len = MBUF_HEADROOM + room; }

typedef struct {
  uint8_t *buf; /* g_buf_len bytes */
  uint32_t data_off, data_len;
} mbuf_t;

static mbuf_t *mb_new(void) {
  mbuf_t *m = (mbuf_t *)malloc(sizeof(mbuf_t));
  m->buf = (uint8_t *)malloc(g_buf_len);
  return m;
}

static void mb_free(mbuf_t *m) {
  free(m->buf);
  free(m);
}

static uint8_t *mb_data(mbuf_t *m, uint32_t off) { return m->buf + m->data_off + off; }

/* mbuf.rs:313-327 read_data::<T>(offset): 0 ok, else the status for `layer`. */
static int read_data(uint32_t data_len, uint32_t offset, uint32_t size_of, int bad_off,
                     int oob) {
  if (!(offset < data_len)) return bad_off;
  if (!(offset + size_of <= data_len)) return oob;
  return 0;
}

/* mbuf.rs:225-245 extend */
static int mb_extend(mbuf_t *m, uint32_t offset, uint32_t len) {
  uint32_t tailroom = g_buf_len - m->data_off - m->data_len;
  if (!(len > 0)) return -1;
  if (!(offset <= m->data_len)) return -1;
  if (!(len < tailroom)) return -1;
  uint32_t to_copy = m->data_len - offset;
  if (to_copy > 0) memmove(mb_data(m, offset + len), mb_data(m, offset), to_copy);
  m->data_len += len;
  return 0;
}

/* mbuf.rs:256-275 shrink */
static int mb_shrink(mbuf_t *m, uint32_t offset, uint32_t len) {
  if (!(len > 0)) return -1;
  if (!(offset + len <= m->data_len)) return -1;
  uint32_t to_copy = m->data_len - offset - len;
  if (to_copy > 0) memmove(mb_data(m, offset), mb_data(m, offset + len), to_copy);
  m->data_len -= len;
  return 0;
}

/* ---- Ethernet (core/src/packets/ethernet.rs) ----------------------------- */
typedef struct {
  uint32_t header_len; /* :253-261 */
  uint16_t ether_type; /* :170-181 */
  uint32_t vlan;       /* 0, 1 dot1q (:197), 2 qinq (:203) */
  uint32_t et_off;     /* where ether_type lives (set_ether_type :185-192) */
} eth_t;

/* :279-300 try_parse */
static int eth_parse(const uint8_t *p, uint32_t data_len, eth_t *e) {
  int st = read_data(data_len, 0, 14, CGPU_PKT_ETH_BAD_OFFSET, CGPU_PKT_ETH_OUT_OF_BUFFER);
  if (st) return st;
  uint16_t marker = rd16(p + 12); /* vlan_marker :164-167 */
  if (marker == 0x8100) {
    e->vlan = 1;
    e->header_len = 18;
    e->et_off = 16;
  } else if (marker == 0x88a8) {
    e->vlan = 2;
    e->header_len = 22;
    e->et_off = 20;
  } else {
    e->vlan = 0;
    e->header_len = 14;
    e->et_off = 12;
  }
  if (!(data_len >= e->header_len)) return CGPU_PKT_ETH_OUT_OF_BUFFER; /* :294-297 */
  e->ether_type = rd16(p + e->et_off);
  return 0;
}

/* ---- one packet through Ethernet -> Ipv4|Ipv6 -> Udp|Tcp ---------------- */
static void parse_one(const uint8_t *p, uint32_t len, uint32_t flags, uint32_t *meta_out,
                      uint32_t *csum_out, uint64_t *hash_out, cgpu_hdr_record *rec,
                      cgpu_ext_record *ext) {
  const int acc4 = (flags & CGPU_F_ACCEPT_V4) != 0, acc6 = (flags & CGPU_F_ACCEPT_V6) != 0;
  const int accu = (flags & CGPU_F_ACCEPT_UDP) != 0, acct = (flags & CGPU_F_ACCEPT_TCP) != 0;
  const int acci = (flags & CGPU_F_ACCEPT_ICMP) != 0;
  uint32_t meta = 0, ip_c = 0, l4_c = 0;
  uint64_t hash = 0;
  cgpu_hdr_record r;
  memset(&r, 0, sizeof r);
  cgpu_ext_record x;
  memset(&x, 0, sizeof x);
  const uint8_t *seg0 = NULL; /* SegmentRouting::dst() when behind a routing header */

  eth_t e;
  int st = eth_parse(p, len, &e);
  int l3 = 0, l4 = 0; /* CGPU_L3_*, CGPU_L4_* */
  uint32_t l3_off = 0, l3_len = 0, l4_off = 0;
  if (!st) {
    meta |= e.header_len << 8;
    if (e.vlan == 1) meta |= CGPU_META_DOT1Q;
    if (e.vlan == 2) meta |= CGPU_META_QINQ;
    memcpy(r.dst_mac, p, 6);
    memcpy(r.src_mac, p + 6, 6);
    r.ether_type = e.ether_type;
    r.eth_len = (uint8_t)e.header_len;
    r.vlan = (uint8_t)e.vlan;
    l3_off = e.header_len; /* payload_offset = offset + header_len */
    /* Ipv4::try_parse (ip/v4.rs:427-442) / Ipv6::try_parse (ip/v6/mod.rs:274-289) */
    if (acc4 && e.ether_type == 0x0800) {
      l3 = CGPU_L3_IPV4;
      l3_len = 20; /* Ipv4Header::size_of, :403-405 */
    } else if (acc6 && e.ether_type == 0x86DD) {
      l3 = CGPU_L3_IPV6;
      l3_len = 40;
    } else {
      st = (acc4 && acc6) ? CGPU_PKT_NOT_IP : (acc4 ? CGPU_PKT_NOT_IPV4 : CGPU_PKT_NOT_IPV6);
    }
    if (!st)
      st = read_data(len, l3_off, l3_len, CGPU_PKT_L3_BAD_OFFSET, CGPU_PKT_L3_OUT_OF_BUFFER);
    if (st) l3 = 0;
  }
  uint8_t proto = 0;
  if (l3) {
    const uint8_t *h = p + l3_off;
    if (l3 == CGPU_L3_IPV4) { /* accessors ip/v4.rs:164-357 */
      r.version = (h[0] & 0xf0) >> 4;
      r.ihl = h[0] & 0x0f;
      r.dscp = h[1] >> 2;
      r.ecn = h[1] & 0x03;
      r.ip_length = rd16(h + 2);
      r.identification = rd16(h + 4);
      uint16_t ff = rd16(h + 6);
      r.ip_flags = (uint8_t)(((ff & 0x4000) ? 1 : 0) | ((ff & 0x2000) ? 2 : 0));
      r.fragment_offset = ff & 0x1fff;
      r.ttl = h[8];
      r.protocol = h[9];
      r.ip_checksum = rd16(h + 10);
      memcpy(r.src_ip, h + 12, 4);
      memcpy(r.dst_ip, h + 16, 4);
      proto = h[9];
      if (flags & CGPU_F_CSUM_IP) { /* compute_checksum :322-333 */
        uint8_t hdr[20];
        memcpy(hdr, h, 20);
        wr16(hdr + 10, 0);
        ip_c = or_compute(0, hdr, 20);
        if (ip_c == r.ip_checksum) meta |= CGPU_META_IP_CSUM_OK;
      }
    } else { /* accessors ip/v6/mod.rs:116-209 */
      uint32_t w = rd32(h);
      r.version = (uint8_t)(w >> 28);
      r.dscp = (uint8_t)((w & 0x0fc00000) >> 22);
      r.ecn = (uint8_t)((w & 0x00300000) >> 20);
      r.flow_label = w & 0x000fffff;
      r.ip_length = rd16(h + 4);
      r.protocol = h[6];
      r.ttl = h[7];
      memcpy(r.src_ip, h + 8, 16);
      memcpy(r.dst_ip, h + 24, 16);
      proto = h[6];
    }
    meta |= (uint32_t)l3 << 16;
    l4_off = l3_off + l3_len;
    /* CGPU_F_V6_EXT: SegmentRouting<Ipv6>::try_parse (ip/v6/srh.rs:299-327) or
     * Fragment<Ipv6>::try_parse (ip/v6/fragment.rs:187-202), then L4 behind it */
    if (l3 == CGPU_L3_IPV6 && (flags & CGPU_F_V6_EXT) && (proto == 43 || proto == 44)) {
      const uint32_t xo = l4_off; /* envelope.payload_offset() */
      uint32_t xhl = 0;
      st = read_data(len, xo, 8, CGPU_PKT_EXT_BAD_OFFSET, CGPU_PKT_EXT_OUT_OF_BUFFER);
      if (!st && proto == 43) {
        const uint8_t *h = p + xo; /* SegmentRoutingHeader (srh.rs:499-507) */
        const uint32_t hel = h[1], nseg = (uint32_t)h[4] + 1;
        if (!(hel != 0 && 2 * nseg == hel)) {
          st = CGPU_PKT_SRH_INCONSISTENT; /* "Packet has inconsistent segment list length." */
        } else {
          /* read_data_slice::<Ipv6Addr>(offset + 8, segments) (mbuf.rs:365-380) */
          st = read_data(len, xo + 8, 16 * nseg, CGPU_PKT_EXT_BAD_OFFSET,
                         CGPU_PKT_EXT_OUT_OF_BUFFER);
        }
        if (!st) {
          xhl = 8 + 16 * nseg; /* header_len (srh.rs:274-276) */
          seg0 = h + 8;
          x.kind = CGPU_EXT_SRH;
          x.hdr_ext_len = h[1];
          x.routing_type = h[2];
          x.segments_left = h[3];
          x.last_entry = h[4];
          x.srh_flags = h[5];
          x.tag = rd16(h + 6);
          memcpy(x.segment0, seg0, 16);
        }
      } else if (!st) {
        const uint8_t *h = p + xo; /* FragmentHeader (fragment.rs:322-327) */
        xhl = 8;
        x.kind = CGPU_EXT_FRAGMENT;
        x.fragment_offset = rd16(h + 2) >> 3; /* & FRAG_OS, >> 3 (:93-96) */
        x.more_fragments = rd16(h + 2) & 1;   /* FLAG_MORE (:105-107) */
        x.identification = rd32(h + 4);
      }
      if (!st) {
        x.next_header = p[xo];
        x.header_len = (uint16_t)xhl;
        proto = p[xo]; /* next_protocol() of the extension */
        l4_off = xo + xhl;
        meta |= (uint32_t)x.kind << 24;
      } else {
        memset(&x, 0, sizeof x);
        seg0 = NULL;
      }
    }
    /* Udp::try_parse (udp.rs:287-302) / Tcp::try_parse (tcp.rs:558-573) /
     * Icmpv4::try_parse (icmp/v4/mod.rs:205-220: protocol() == Icmpv4) /
     * Icmpv6::try_parse (icmp/v6/mod.rs:217-232: next_protocol() == Icmpv6) */
    uint32_t l4_len = 0;
    const uint8_t icmp_proto = l3 == CGPU_L3_IPV4 ? 0x01 : 0x3A; /* ip/mod.rs:41-75 */
    if (st) {
      /* the extension header failed */
    } else if (accu && proto == 17) {
      l4 = CGPU_L4_UDP;
      l4_len = 8;
    } else if (acct && proto == 6) {
      l4 = CGPU_L4_TCP;
      l4_len = 20; /* TcpHeader::size_of, tcp.rs:531-533 */
    } else if (acci && proto == icmp_proto) {
      l4 = CGPU_L4_ICMP;
      l4_len = 4; /* Icmpv4Header / Icmpv6Header::size_of (icmp/v4/mod.rs:455) */
    } else if (accu + acct + acci > 1) {
      st = CGPU_PKT_NOT_L4;
    } else {
      st = accu ? CGPU_PKT_NOT_UDP
                : acct ? CGPU_PKT_NOT_TCP
                       : (l3 == CGPU_L3_IPV4 ? CGPU_PKT_NOT_ICMPV4 : CGPU_PKT_NOT_ICMPV6);
    }
    if (!st)
      st = read_data(len, l4_off, l4_len, CGPU_PKT_L4_BAD_OFFSET, CGPU_PKT_L4_OUT_OF_BUFFER);
    if (st) l4 = 0;
  }
  if (l4) {
    const uint8_t *u = p + l4_off;
    r.src_port = rd16(u);
    r.dst_port = rd16(u + 2);
    uint32_t cs_at;
    if (l4 == CGPU_L4_UDP) { /* udp.rs:90-128 */
      r.udp_length_or_window = rd16(u + 4);
      r.l4_checksum = rd16(u + 6);
      cs_at = 6;
    } else if (l4 == CGPU_L4_ICMP) { /* msg_type, code, checksum (icmp/v4/mod.rs:88-112) */
      r.src_port = u[0];
      r.dst_port = u[1];
      r.l4_checksum = rd16(u + 2);
      cs_at = 2;
    } else { /* tcp.rs:139-405 */
      r.seq_no = rd32(u + 4);
      r.ack_no = rd32(u + 8);
      r.data_offset = (u[12] & 0xf0) >> 4;
      r.ns = u[12] & 0x01;
      r.tcp_flags = u[13];
      r.udp_length_or_window = rd16(u + 14);
      r.l4_checksum = rd16(u + 16);
      r.urgent_pointer = rd16(u + 18);
      cs_at = 16;
    }
    meta |= (uint32_t)l4 << 18;
    const uint8_t pr = l4 == CGPU_L4_UDP ? 17 : (l4 == CGPU_L4_ICMP ? 0x3A : 6); /* ip/mod.rs:41-75 */
    if (flags & CGPU_F_CSUM_L4) {
      /* Udp::compute_checksum (udp.rs:204-219) / Tcp (tcp.rs:462-477): the
       * span is [offset, data_len), checksum field zeroed first. */
      uint32_t span = len - l4_off;
      uint8_t *data = (uint8_t *)malloc(span);
      memcpy(data, u, span);
      wr16(data + cs_at, 0);
      uint16_t ph;
      if (l4 == CGPU_L4_ICMP && l3 == CGPU_L3_IPV4)
        ph = 0; /* Icmpv4::compute_checksum: compute(0, data) (icmp/v4/mod.rs:118-129) */
      else if (l3 == CGPU_L3_IPV4)
        ph = or_pseudo_v4(rd32(p + l3_off + 12), rd32(p + l3_off + 16), (uint16_t)span, pr);
      else /* behind a routing header: dst = segments[0] (srh.rs:456-470) */
        ph = or_pseudo_v6(p + l3_off + 8, seg0 ? seg0 : p + l3_off + 24, (uint16_t)span, pr);
      l4_c = or_compute(ph, data, span);
      free(data);
      if (l4 == CGPU_L4_UDP && l4_c == 0) l4_c = 0xFFFF; /* set_checksum udp.rs:137-140 */
      if (l4_c == r.l4_checksum) meta |= CGPU_META_L4_CSUM_OK;
    }
    /* Udp::flow udp.rs:151-159, Tcp::flow tcp.rs:409-417; ICMP has no flow */
    if ((flags & CGPU_F_FLOW_HASH) && l4 != CGPU_L4_ICMP)
      hash = or_flow_hash(l3 == CGPU_L3_IPV6, r.src_ip, seg0 ? seg0 : r.dst_ip, r.src_port,
                          r.dst_port, pr);
  }
  meta |= (uint32_t)st;
  *meta_out = meta;
  if (csum_out) *csum_out = ip_c | (l4_c << 16);
  if (hash_out) *hash_out = hash;
  if (rec) *rec = r;
  if (ext) *ext = x;
}

void or_parse_batch_ext(const uint8_t *arena, const uint32_t *off, const uint16_t *len,
                        uint32_t n, uint32_t flags, uint32_t *meta, uint32_t *csum,
                        uint64_t *flow_hash, cgpu_hdr_record *fields, cgpu_ext_record *ext) {
  /* no L3 (L4) type named: every IP version (UDP and TCP) accepted */
  if ((flags & (CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_V6)) == 0) flags |= CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_V6;
  if ((flags & (CGPU_F_ACCEPT_UDP | CGPU_F_ACCEPT_TCP | CGPU_F_ACCEPT_ICMP)) == 0)
    flags |= CGPU_F_ACCEPT_UDP | CGPU_F_ACCEPT_TCP;
  for (uint32_t i = 0; i < n; ++i)
    parse_one(arena + off[i], len[i], flags, meta + i,
              (flags & (CGPU_F_CSUM_IP | CGPU_F_CSUM_L4)) && csum ? csum + i : NULL,
              (flags & CGPU_F_FLOW_HASH) && flow_hash ? flow_hash + i : NULL,
              fields ? fields + i : NULL, ext ? ext + i : NULL);
}

void or_parse_batch(const uint8_t *arena, const uint32_t *off, const uint16_t *len, uint32_t n,
                    uint32_t flags, uint32_t *meta, uint32_t *csum, uint64_t *flow_hash,
                    cgpu_hdr_record *fields) {
  or_parse_batch_ext(arena, off, len, n, flags, meta, csum, flow_hash, fields, NULL);
}

/* bench/packets.rs:65-69 multi_parse_udp: parse::<Ethernet>() ->
 * parse::<Ipv4>() -> parse::<Udp4>(), nothing else.  Written as the bare
 * chain of checks (no field extraction) so it times what the reference
 * bench times.                                                             */
uint32_t or_multi_parse_udp(const uint8_t *arena, const uint32_t *off, const uint16_t *len,
                            uint32_t n) {
  uint32_t ok = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t *p = arena + off[i];
    eth_t e;
    if (eth_parse(p, len[i], &e)) continue;
    if (e.ether_type != 0x0800) continue;
    if (read_data(len[i], e.header_len, 20, 1, 1)) continue;
    if (p[e.header_len + 9] != 17) continue;
    if (read_data(len[i], e.header_len + 20, 8, 1, 1)) continue;
    ++ok;
  }
  return ok;
}

/* ---- examples/nat64: PORT_MAP + NEXT_PORT (main.rs:37-53) ---------------- */
typedef struct {
  uint8_t key[18]; /* (Ipv6Addr, u16) */
  uint16_t port;
  uint8_t used;
} pm_slot;

struct or_portmap {
  pm_slot *slots;
  uint32_t cap, size;
  uint16_t next_port; /* AtomicU16 NEXT_PORT (main.rs:42), initial 1025 */
  /* ADDR_MAP (main.rs:38): gateway port -> (v6 addr, port), insert_new */
  uint8_t addr_key[65536][18];
  uint8_t addr_used[65536];
};

or_portmap *or_portmap_new(uint16_t first_port) {
  or_portmap *pm = (or_portmap *)calloc(1, sizeof *pm);
  pm->cap = 1024;
  pm->slots = (pm_slot *)calloc(pm->cap, sizeof(pm_slot));
  pm->next_port = first_port;
  return pm;
}

void or_portmap_free(or_portmap *pm) {
  if (!pm) return;
  free(pm->slots);
  free(pm);
}

uint16_t or_portmap_next_port(const or_portmap *pm) { return pm->next_port; }
uint32_t or_portmap_size(const or_portmap *pm) { return pm->size; }

static uint32_t key_hash(const uint8_t *k) {
  uint32_t h = 2166136261u; /* FNV-1a: any hash will do for a host map */
  for (int i = 0; i < 18; ++i) h = (h ^ k[i]) * 16777619u;
  return h;
}

static pm_slot *pm_find(or_portmap *pm, const uint8_t *k) {
  uint32_t h = key_hash(k) & (pm->cap - 1);
  while (pm->slots[h].used) {
    if (!memcmp(pm->slots[h].key, k, 18)) return &pm->slots[h];
    h = (h + 1) & (pm->cap - 1);
  }
  return &pm->slots[h];
}

static void pm_grow(or_portmap *pm) {
  pm_slot *old = pm->slots;
  uint32_t oc = pm->cap;
  pm->cap *= 2;
  pm->slots = (pm_slot *)calloc(pm->cap, sizeof(pm_slot));
  for (uint32_t i = 0; i < oc; ++i)
    if (old[i].used) *pm_find(pm, old[i].key) = old[i];
  free(old);
}

/* main.rs:41-53 assigned_port */
static uint16_t assigned_port(or_portmap *pm, const uint8_t addr[16], uint16_t port) {
  uint8_t k[18];
  memcpy(k, addr, 16);
  k[16] = (uint8_t)(port >> 8);
  k[17] = (uint8_t)port;
  pm_slot *s = pm_find(pm, k);
  if (s->used) return s->port;
  uint16_t p = pm->next_port; /* fetch_add(1): wraps mod 2^16 */
  pm->next_port = (uint16_t)(pm->next_port + 1);
  memcpy(s->key, k, 18);
  s->port = p;
  s->used = 1;
  pm->size++;
  if (!pm->addr_used[p]) { /* ADDR_MAP.insert_new(port, key): first one stays */
    memcpy(pm->addr_key[p], k, 18);
    pm->addr_used[p] = 1;
  }
  if (pm->size * 2 > pm->cap) pm_grow(pm);
  return p;
}

/* main.rs:121-150 nat_6to4 on one mbuf; returns disposition, sets *status. */
static int nat_6to4(or_portmap *pm, mbuf_t *m, uint8_t *status) {
  uint8_t *p = mb_data(m, 0);
  /* let ethernet = packet.parse::<Ethernet>()?; */
  eth_t e;
  int st = eth_parse(p, m->data_len, &e);
  if (st) { *status = (uint8_t)st; return CGPU_ABORT; }
  /* let v6 = ethernet.parse::<Ipv6>()?; */
  if (e.ether_type != 0x86DD) { *status = CGPU_PKT_NOT_IPV6; return CGPU_ABORT; }
  const uint32_t v6_off = e.header_len;
  st = read_data(m->data_len, v6_off, 40, CGPU_PKT_L3_BAD_OFFSET, CGPU_PKT_L3_OUT_OF_BUFFER);
  if (st) { *status = (uint8_t)st; return CGPU_ABORT; }
  const uint8_t *h6 = p + v6_off;
  *status = CGPU_PKT_OK;
  /* if v6.next_header() == ProtocolNumbers::Tcp { ... } else Drop */
  if (h6[6] != 6) return CGPU_DROP;
  uint32_t w = rd32(h6);
  uint8_t dscp = (uint8_t)((w & 0x0fc00000) >> 22);
  uint8_t ecn = (uint8_t)((w & 0x00300000) >> 20);
  uint8_t ttl = (uint8_t)(h6[7] - 1); /* hop_limit - 1 (wrapping, release build) */
  uint8_t protocol = h6[6];
  uint8_t src[16];
  memcpy(src, h6 + 8, 16);
  uint8_t dst4[4]; /* map6to4 :79-83: segments[6..8] */
  memcpy(dst4, h6 + 36, 4);
  /* let ethernet = v6.remove()?;  (packets/mod.rs:242 -> shrink(offset, 40)) */
  if (mb_shrink(m, v6_off, 40)) { *status = CGPU_PKT_NOT_RESIZED; return CGPU_ABORT; }
  /* let mut v4 = ethernet.push::<Ipv4>()?;  (ip/v4.rs:455-469) */
  if (mb_extend(m, v6_off, 20)) { *status = CGPU_PKT_NOT_RESIZED; return CGPU_ABORT; }
  p = mb_data(m, 0);
  uint8_t *h4 = p + v6_off;
  static const uint8_t dflt[20] = {0x45, 0, 0, 0, 0, 0, 0, 0, 64, 0,
                                   0,    0, 0, 0, 0, 0, 0, 0, 0,  0}; /* :594-609 */
  memcpy(h4, dflt, 20);
  wr16(p + e.et_off, 0x0800); /* envelope.set_ether_type(Ipv4), ethernet.rs:185-192 */
  /* setters ip/v4.rs:189-203, 293-357 */
  h4[1] = (uint8_t)((h4[1] & 0x03) | (uint8_t)(dscp << 2));
  h4[1] = (uint8_t)((h4[1] & 0xfc) | (ecn & 0x03));
  h4[8] = ttl;
  h4[9] = protocol;
  h4[12] = 203; h4[13] = 0; h4[14] = 113; h4[15] = 1; /* V4_ADDR main.rs:35 */
  memcpy(h4 + 16, dst4, 4);
  /* let mut tcp = v4.parse::<Tcp4>()?; */
  const uint32_t tcp_off = v6_off + 20;
  if (h4[9] != 6) { *status = CGPU_PKT_NOT_TCP; return CGPU_ABORT; }
  st = read_data(m->data_len, tcp_off, 20, CGPU_PKT_L4_BAD_OFFSET, CGPU_PKT_L4_OUT_OF_BUFFER);
  if (st) { *status = (uint8_t)st; return CGPU_ABORT; }
  uint8_t *t = p + tcp_off;
  /* tcp.set_src_port(assigned_port(src, tcp.src_port())); */
  wr16(t, assigned_port(pm, src, rd16(t)));
  /* tcp.reconcile_all(): Tcp::reconcile -> compute_checksum (tcp.rs:462-477) */
  uint32_t span = m->data_len - tcp_off;
  wr16(t + 16, 0);
  uint16_t ph = or_pseudo_v4(rd32(h4 + 12), rd32(h4 + 16), (uint16_t)span, 6);
  wr16(t + 16, or_compute(ph, t, span));
  /* then Ipv4::reconcile (ip/v4.rs:486-489): total_length, header checksum */
  wr16(h4 + 2, (uint16_t)(m->data_len - v6_off));
  wr16(h4 + 10, 0);
  wr16(h4 + 10, or_compute(0, h4, 20));
  return CGPU_ACT;
}

/* main.rs:86-118 nat_4to6 on one mbuf; returns disposition, sets *status. */
static int nat_4to6(or_portmap *pm, mbuf_t *m, uint8_t *status) {
  uint8_t *p = mb_data(m, 0);
  /* let ethernet = packet.parse::<Ethernet>()?; */
  eth_t e;
  int st = eth_parse(p, m->data_len, &e);
  if (st) { *status = (uint8_t)st; return CGPU_ABORT; }
  /* let v4 = ethernet.parse::<Ipv4>()?; */
  if (e.ether_type != 0x0800) { *status = CGPU_PKT_NOT_IPV4; return CGPU_ABORT; }
  const uint32_t v4_off = e.header_len;
  st = read_data(m->data_len, v4_off, 20, CGPU_PKT_L3_BAD_OFFSET, CGPU_PKT_L3_OUT_OF_BUFFER);
  if (st) { *status = (uint8_t)st; return CGPU_ABORT; }
  const uint8_t *h4 = p + v4_off;
  *status = CGPU_PKT_OK;
  /* if protocol == Tcp && fragment_offset() == 0 && !more_fragments() */
  const uint16_t ff = rd16(h4 + 6);
  if (!(h4[9] == 6 && (ff & 0x1fff) == 0 && !(ff & 0x2000))) return CGPU_DROP;
  /* let tcp = v4.peek::<Tcp4>()?; */
  const uint32_t tcp_off = v4_off + 20;
  st = read_data(m->data_len, tcp_off, 20, CGPU_PKT_L4_BAD_OFFSET, CGPU_PKT_L4_OUT_OF_BUFFER);
  if (st) { *status = (uint8_t)st; return CGPU_ABORT; }
  /* if let Some((dst, port)) = assigned_addr(tcp.dst_port()) (main.rs:56-58) */
  const uint16_t gw_port = rd16(p + tcp_off + 2);
  if (!pm->addr_used[gw_port]) return CGPU_DROP;
  uint8_t dst6[16];
  memcpy(dst6, pm->addr_key[gw_port], 16);
  const uint16_t orig_port = rd16(pm->addr_key[gw_port] + 16);
  const uint8_t dscp = h4[1] >> 2, ecn = h4[1] & 0x03; /* v4.rs:186-203 */
  const uint8_t next_header = h4[9];
  const uint8_t hop_limit = (uint8_t)(h4[8] - 1); /* ttl - 1 (wrapping, release build) */
  /* map4to6(v4.src()) = 64:ff9b::a.b.c.d (main.rs:62-74) */
  uint8_t src6[16] = {0x00, 0x64, 0xff, 0x9b, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  memcpy(src6 + 12, h4 + 12, 4);
  /* let ethernet = v4.remove()?;  (shrink(offset, 20)) */
  if (mb_shrink(m, v4_off, 20)) { *status = CGPU_PKT_NOT_RESIZED; return CGPU_ABORT; }
  /* let mut v6 = ethernet.push::<Ipv6>()?;  (ip/v6/mod.rs:302-316) */
  if (mb_extend(m, v4_off, 40)) { *status = CGPU_PKT_NOT_RESIZED; return CGPU_ABORT; }
  p = mb_data(m, 0);
  uint8_t *h6 = p + v4_off;
  memset(h6, 0, 40); /* Ipv6Header::default (:453-464) */
  h6[0] = 0x60;
  h6[7] = 64;
  wr16(p + e.et_off, 0x86DD); /* envelope.set_ether_type(Ipv6) */
  /* setters (ip/v6/mod.rs:130-209) */
  uint32_t w = rd32(h6);
  w = (w & ~0x0fc00000u) | (((uint32_t)dscp << 22) & 0x0fc00000u);
  w = (w & ~0x00300000u) | (((uint32_t)ecn << 20) & 0x00300000u);
  h6[0] = (uint8_t)(w >> 24); h6[1] = (uint8_t)(w >> 16); h6[2] = (uint8_t)(w >> 8); h6[3] = (uint8_t)w;
  h6[6] = next_header;
  h6[7] = hop_limit;
  memcpy(h6 + 8, src6, 16);
  memcpy(h6 + 24, dst6, 16);
  /* let mut tcp = v6.parse::<Tcp6>()?; */
  const uint32_t tcp6_off = v4_off + 40;
  if (h6[6] != 6) { *status = CGPU_PKT_NOT_TCP; return CGPU_ABORT; }
  st = read_data(m->data_len, tcp6_off, 20, CGPU_PKT_L4_BAD_OFFSET, CGPU_PKT_L4_OUT_OF_BUFFER);
  if (st) { *status = (uint8_t)st; return CGPU_ABORT; }
  uint8_t *t = p + tcp6_off;
  wr16(t + 2, orig_port); /* tcp.set_dst_port(port) */
  /* tcp.reconcile_all(): Tcp::compute_checksum with the v6 pseudo-header */
  const uint32_t span = m->data_len - tcp6_off;
  wr16(t + 16, 0);
  const uint16_t ph = or_pseudo_v6(h6 + 8, h6 + 24, (uint16_t)span, 6);
  wr16(t + 16, or_compute(ph, t, span));
  /* Ipv6::reconcile (ip/v6/mod.rs:331-334): payload_length */
  wr16(h6 + 4, (uint16_t)(m->data_len - v4_off - 40));
  return CGPU_ACT;
}

void or_nat64_4to6(or_portmap *pm, const uint8_t *arena, const uint32_t *off, const uint16_t *len,
                   uint32_t n, uint8_t *out_arena, const uint32_t *out_off, uint16_t *out_len,
                   uint8_t *disposition, uint8_t *status) {
  mbuf_t *m = mb_new();
  for (uint32_t i = 0; i < n; ++i) {
    m->data_off = MBUF_HEADROOM;
    m->data_len = len[i];
    if (m->data_len > g_buf_len - MBUF_HEADROOM) m->data_len = g_buf_len - MBUF_HEADROOM;
    memcpy(mb_data(m, 0), arena + off[i], m->data_len);
    int d = nat_4to6(pm, m, status + i);
    disposition[i] = (uint8_t)d;
    if (d == CGPU_ACT) {
      memcpy(out_arena + out_off[i], mb_data(m, 0), m->data_len);
      out_len[i] = (uint16_t)m->data_len;
    } else {
      out_len[i] = 0;
    }
  }
  mb_free(m);
}

void or_nat64_6to4(or_portmap *pm, const uint8_t *arena, const uint32_t *off, const uint16_t *len,
                   uint32_t n, uint8_t *out_arena, const uint32_t *out_off, uint16_t *out_len,
                   uint8_t *disposition, uint8_t *status) {
  mbuf_t *m = mb_new();
  for (uint32_t i = 0; i < n; ++i) {
    m->data_off = MBUF_HEADROOM;
    m->data_len = len[i];
    if (m->data_len > g_buf_len - MBUF_HEADROOM) m->data_len = g_buf_len - MBUF_HEADROOM;
    memcpy(mb_data(m, 0), arena + off[i], m->data_len);
    int d = nat_6to4(pm, m, status + i);
    disposition[i] = (uint8_t)d;
    if (d == CGPU_ACT) {
      memcpy(out_arena + out_off[i], mb_data(m, 0), m->data_len);
      out_len[i] = (uint16_t)m->data_len;
    } else {
      out_len[i] = 0;
    }
  }
  mb_free(m);
}

/* ---- group_by (core/src/batch/group_by.rs) ------------------------------ */

/* The selector of the CGPU_KEY_META_CLASS arms: a match on the typed parse
 * result a pipeline would write as its group_by closure. */
static uint32_t meta_class(uint32_t m) {
  if ((m & 0xffu) != CGPU_PKT_OK) return 4;
  const uint32_t l3 = (m >> 16) & 3u, l4 = (m >> 18) & 3u;
  if (l4 != CGPU_L4_UDP && l4 != CGPU_L4_TCP) return 4; /* ICMP: neither Udp nor Tcp */
  if (l3 == CGPU_L3_IPV4) return l4 == CGPU_L4_TCP ? 1 : 0;
  return l4 == CGPU_L4_TCP ? 3 : 2;
}

/* GroupBy::next (group_by.rs:143-172): for each packet in arrival order,
 * `groups.get_mut(&key)` or the catch-all, then the arm runs the packet.
 * Each arm's packets are collected in a growable list, like the fanout
 * queue, and concatenated arm by arm. */
void or_group_by(const void *key, uint32_t key_kind, uint32_t n, uint32_t n_groups, uint32_t *idx,
                 uint32_t *group_off) {
  uint32_t **arm = (uint32_t **)calloc(n_groups, sizeof(uint32_t *));
  uint32_t *cnt = (uint32_t *)calloc(n_groups, sizeof(uint32_t));
  uint32_t *cap = (uint32_t *)calloc(n_groups, sizeof(uint32_t));
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t k = key_kind == CGPU_KEY_META_CLASS ? meta_class(((const uint32_t *)key)[i])
                                                  : ((const uint8_t *)key)[i];
    if (k >= n_groups - 1) k = n_groups - 1; /* None => catchall */
    if (cnt[k] == cap[k]) {
      cap[k] = cap[k] ? 2 * cap[k] : 16;
      arm[k] = (uint32_t *)realloc(arm[k], cap[k] * sizeof(uint32_t));
    }
    arm[k][cnt[k]++] = i;
  }
  uint32_t at = 0;
  for (uint32_t k = 0; k < n_groups; ++k) {
    group_off[k] = at;
    if (cnt[k]) memcpy(idx + at, arm[k], cnt[k] * sizeof(uint32_t));
    at += cnt[k];
    free(arm[k]);
  }
  group_off[n_groups] = at;
  free(arm);
  free(cnt);
  free(cap);
}

/* ---- checksum.rs:202-220 `compute_with_ipaddr` --------------------------
 * Returns 0 and the new checksum, or -1 for "cannot mix IPv4 and IPv6
 * addresses." (:218).  Address words are Ipv4Addr -> u32 split hi/lo
 * (:209-213) or Ipv6Addr::segments() (:215-216).                          */
static int or_compute_with_ipaddr(uint16_t old_checksum, int old_v6, const uint8_t *old_addr,
                                  const cgpu_ip_addr *new_addr, uint16_t *out) {
  uint16_t ow[8], nw[8];
  const size_t words = old_v6 ? 8 : 2;
  if (new_addr->family != (old_v6 ? 6u : 4u)) return -1;
  for (size_t i = 0; i < words; ++i) {
    ow[i] = rd16(old_addr + 2 * i);
    nw[i] = rd16(new_addr->octets + 2 * i);
  }
  *out = or_compute_inc(old_checksum, ow, nw, words);
  return 0;
}

/* udp.rs:174-201 / tcp.rs:432-459 `set_src_ip` / `set_dst_ip`: checksum from
 * the envelope's current address, then envelope_mut().set_src/set_dst
 * (v4.rs:343-357 / v6/mod.rs:195-209: the field store only), then
 * set_checksum (UDP: 0 stored as 0xFFFF, udp.rs:132-141; TCP as is).     */
static int or_set_addr(uint8_t *frame, uint32_t l4_off, int udp, int v6, uint32_t addr_off,
                       const cgpu_ip_addr *a) {
  uint8_t *ck = frame + l4_off + (udp ? 6 : 16);
  uint16_t c;
  if (or_compute_with_ipaddr(rd16(ck), v6, frame + addr_off, a, &c) != 0) return -1;
  memcpy(frame + addr_off, a->octets, v6 ? 16 : 4);
  wr16(ck, (udp && c == 0) ? 0xFFFF : c);
  return 0;
}

/* ---- Packet::reconcile_all (core/src/packets/mod.rs:297-300) --------------
 * `self.reconcile(); self.envelope_mut().reconcile_all()`: the held layer
 * first, then every envelope outward.  The layers and their offsets are the
 * ones the parse recorded in `meta` (a typed packet keeps its offset; the
 * L4 layer's pseudo-header protocol is its type's constant, udp.rs:212,
 * tcp.rs:470, icmp/v6/mod.rs:130), the bytes are the frame's current ones. */

/* L4 offset of a packet whose meta records an L4 layer: behind the IPv6
 * extension header the parse found (SegmentRouting::header_len srh.rs:
 * 274-276 from the frame's current last_entry, or Fragment's 8 B), with the
 * parse's checks (srh.rs:299-327); -1 when they fail on the current bytes. */
static int64_t recon_l4_off(const uint8_t *p, uint32_t len, uint32_t meta, const uint8_t **seg0) {
  const uint32_t eth = CGPU_META_ETH_LEN(meta), l3 = CGPU_META_L3(meta);
  uint32_t l4_off = eth + (l3 == CGPU_L3_IPV6 ? 40 : 20);
  *seg0 = NULL;
  const uint32_t xk = CGPU_META_EXT(meta);
  if (xk != CGPU_EXT_NONE) {
    if (read_data(len, l4_off, 8, 1, 1)) return -1;
    if (xk == CGPU_EXT_SRH) {
      const uint8_t *h = p + l4_off;
      const uint32_t hel = h[1], nseg = (uint32_t)h[4] + 1;
      if (!(hel != 0 && 2 * nseg == hel)) return -1;
      if (read_data(len, l4_off + 8, 16 * nseg, 1, 1)) return -1;
      *seg0 = h + 8;
      l4_off += 8 + 16 * nseg;
    } else {
      l4_off += 8;
    }
  }
  const uint32_t l4 = CGPU_META_L4(meta);
  const uint32_t l4_len = l4 == CGPU_L4_UDP ? 8 : (l4 == CGPU_L4_TCP ? 20 : 4);
  if (read_data(len, l4_off, l4_len, 1, 1)) return -1;
  return l4_off;
}

/* Udp::reconcile (udp.rs:350-354) / Tcp::reconcile (tcp.rs:619-621) /
 * Icmpv4::reconcile (icmp/v4/mod.rs:246-248) / Icmpv6 (icmp/v6/mod.rs:260-262) */
static void l4_reconcile(uint8_t *p, uint32_t len, uint32_t meta, uint32_t l4_off,
                         const uint8_t *seg0) {
  const uint32_t eth = CGPU_META_ETH_LEN(meta), l3 = CGPU_META_L3(meta), l4 = CGPU_META_L4(meta);
  uint8_t *u = p + l4_off;
  const uint32_t span = len - l4_off; /* self.len(): data_len - offset */
  if (l4 == CGPU_L4_UDP) wr16(u + 4, (uint16_t)span); /* set_length(len as u16) */
  const uint32_t cs_at = l4 == CGPU_L4_UDP ? 6 : (l4 == CGPU_L4_TCP ? 16 : 2);
  wr16(u + cs_at, 0); /* no_checksum / header_mut().checksum = default */
  const uint8_t pr = l4 == CGPU_L4_UDP ? 17 : (l4 == CGPU_L4_TCP ? 6 : 0x3A);
  uint16_t ph;
  if (l4 == CGPU_L4_ICMP && l3 == CGPU_L3_IPV4)
    ph = 0; /* compute(0, data) (icmp/v4/mod.rs:118-129) */
  else if (l3 == CGPU_L3_IPV4)
    ph = or_pseudo_v4(rd32(p + eth + 12), rd32(p + eth + 16), (uint16_t)span, pr);
  else /* behind a routing header: dst = segments[0] (srh.rs:456-470) */
    ph = or_pseudo_v6(p + eth + 8, seg0 ? seg0 : p + eth + 24, (uint16_t)span, pr);
  uint16_t c = or_compute(ph, u, span);
  if (l4 == CGPU_L4_UDP && c == 0) c = 0xFFFF; /* set_checksum (udp.rs:132-141) */
  wr16(u + cs_at, c);
}

/* Ipv4::reconcile (ip/v4.rs:486-489) / Ipv6::reconcile (ip/v6/mod.rs:331-334) */
static void l3_reconcile(uint8_t *p, uint32_t len, uint32_t meta) {
  const uint32_t eth = CGPU_META_ETH_LEN(meta);
  uint8_t *h = p + eth;
  if (CGPU_META_L3(meta) == CGPU_L3_IPV4) {
    wr16(h + 2, (uint16_t)(len - eth)); /* set_total_length(self.len() as u16) */
    wr16(h + 10, 0);                    /* compute_checksum (:322-333) */
    wr16(h + 10, or_compute(0, h, 20));
  } else {
    wr16(h + 4, (uint16_t)(len - eth - 40)); /* set_payload_length(payload_len) */
  }
}

/* Whether the accept set (defaults applied as in or_parse_batch_ext) has
 * every layer meta records up to `depth`. */
static int recon_accepts(uint32_t flags, uint32_t m, uint32_t depth) {
  if ((flags & (CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_V6)) == 0) flags |= CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_V6;
  if ((flags & (CGPU_F_ACCEPT_UDP | CGPU_F_ACCEPT_TCP | CGPU_F_ACCEPT_ICMP)) == 0)
    flags |= CGPU_F_ACCEPT_UDP | CGPU_F_ACCEPT_TCP;
  if (depth >= CGPU_LAYER_L3) {
    if (CGPU_META_L3(m) == CGPU_L3_IPV4 && !(flags & CGPU_F_ACCEPT_V4)) return 0;
    if (CGPU_META_L3(m) == CGPU_L3_IPV6 && !(flags & CGPU_F_ACCEPT_V6)) return 0;
  }
  if (depth >= CGPU_LAYER_L4) {
    const uint32_t l4 = CGPU_META_L4(m);
    if (l4 == CGPU_L4_UDP && !(flags & CGPU_F_ACCEPT_UDP)) return 0;
    if (l4 == CGPU_L4_TCP && !(flags & CGPU_F_ACCEPT_TCP)) return 0;
    if (l4 == CGPU_L4_ICMP && !(flags & CGPU_F_ACCEPT_ICMP)) return 0;
    if (CGPU_META_EXT(m) != CGPU_EXT_NONE && !(flags & CGPU_F_V6_EXT)) return 0;
  }
  return 1;
}

/* A frame not wholly inside the arena (off + len > arena_len: against the
 * ABI's precondition, or meta left from other descriptors) is skipped, not
 * written; the reference's Mbuf always holds its data_len bytes. */
void or_reconcile(uint8_t *arena, uint64_t arena_len, const uint32_t *off, const uint16_t *len,
                  const uint32_t *meta, uint32_t n, uint32_t flags, uint32_t depth, uint8_t *status) {
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t m = meta[i];
    uint8_t *p = arena + off[i];
    const uint32_t eth = CGPU_META_ETH_LEN(m);
    int done = 0;
    if ((uint64_t)off[i] + len[i] > arena_len || !recon_accepts(flags, m, depth)) {
      /* outside the arena, or a layer outside the parse's accept set: not a
       * packet of this pipeline */
    } else if (depth == CGPU_LAYER_L4) {
      const uint8_t *seg0;
      int64_t l4_off = -1;
      if (CGPU_META_STATUS(m) == CGPU_PKT_OK && CGPU_META_L4(m) != CGPU_L4_NONE &&
          CGPU_META_L3(m) != CGPU_L3_NONE)
        l4_off = recon_l4_off(p, len[i], m, &seg0);
      if (l4_off >= 0) {
        l4_reconcile(p, len[i], m, (uint32_t)l4_off, seg0);
        /* SegmentRouting / Fragment: the default reconcile (packets/mod.rs:288) */
        l3_reconcile(p, len[i], m);
        done = 1;
      }
    } else if (depth == CGPU_LAYER_L3) {
      if (CGPU_META_L3(m) != CGPU_L3_NONE &&
          !read_data(len[i], eth, CGPU_META_L3(m) == CGPU_L3_IPV6 ? 40 : 20, 1, 1)) {
        l3_reconcile(p, len[i], m);
        done = 1;
      }
    } else { /* Ethernet: the default reconcile, nothing */
      done = eth != 0 && len[i] >= eth;
    }
    if (status) status[i] = done ? CGPU_RECON_OK : CGPU_RECON_SKIPPED;
  }
}

void or_set_ip(uint8_t *arena, const uint32_t *off, const uint16_t *len, const uint32_t *meta,
               uint32_t n, const cgpu_ip_addr *src, uint32_t src_stride, const cgpu_ip_addr *dst,
               uint32_t dst_stride, uint8_t *status) {
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t m = meta[i];
    const uint32_t l3 = CGPU_META_L3(m), l4 = CGPU_META_L4(m), eth = CGPU_META_ETH_LEN(m);
    const int udp = l4 == CGPU_L4_UDP, v6 = l3 == CGPU_L3_IPV6;
    const uint32_t l4_off = eth + (v6 ? 40 : 20);
    uint8_t st = CGPU_SETIP_OK;
    if (CGPU_META_STATUS(m) != CGPU_PKT_OK || CGPU_META_EXT(m) != 0 || l3 == CGPU_L3_NONE ||
        (l4 != CGPU_L4_UDP && l4 != CGPU_L4_TCP) || l4_off + (udp ? 8u : 20u) > len[i]) {
      st = CGPU_SETIP_SKIPPED;
    } else {
      uint8_t *f = arena + off[i];
      if (src && or_set_addr(f, l4_off, udp, v6, eth + (v6 ? 8 : 12),
                             &src[(size_t)i * src_stride]) != 0)
        st = CGPU_SETIP_SRC_MISMATCH;
      else if (dst && or_set_addr(f, l4_off, udp, v6, eth + (v6 ? 24 : 16),
                                  &dst[(size_t)i * dst_stride]) != 0)
        st = CGPU_SETIP_DST_MISMATCH;
    }
    if (status) status[i] = st;
  }
}
