/*
 * capsule_gpu.h — C ABI of the MI355X-native packet hot path.
 *
 * This header is the drop-in boundary: it is a sibling of Capsule's DPDK
 * binding header (reference ffi/src/bindings.h:42-89, shim.c:19-64) and is
 * meant to be bound the same way (bindgen with an allow-list `cgpu_.*`, see
 * INTEGRATION.md).  Every entry point takes plain pointers and sizes; no HIP
 * or torch type appears in a signature (streams are passed as `void*`, i.e.
 * a hipStream_t, NULL = the legacy default stream).
 *
 * Error convention (mirrors reference core/src/ffi.rs:86-141 `ToResult` and
 * core/src/dpdk/mod.rs:62-70): functions return 0 on success and a negative
 * errno-style code on failure; the same code is kept in a thread-local that
 * `cgpu_last_error()` returns (the `_rte_errno()` analogue, ffi/src/shim.c:24).
 * Per-packet failures are never a call failure: they are reported in the
 * per-packet status byte (CGPU_PKT_*), which mirrors the reference's
 * `BufferError::{BadOffset,OutOfBuffer}` (core/src/dpdk/mbuf.rs:85-98) and the
 * "not an IPv4/IPv6/UDP/TCP packet." errors (ip/v4.rs:430, ip/v6/mod.rs:277,
 * udp.rs:290, tcp.rs:561).
 *
 * Ownership (reference core/src/dpdk/mbuf.rs:467-479, 420-424): the library
 * only BORROWS packet bytes for the duration of a call and never frees or
 * retains caller memory.
 */
#ifndef CAPSULE_GPU_H
#define CAPSULE_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history:
 *   2  round-2 layout.
 *   3  cgpu_portmap_reset; CGPU_MAX_BATCH is 2^30 - 1; group_by's
 *      CGPU_KEY_META_CLASS sends ICMP to the catch-all arm (4); mbufs with
 *      data_off + data_len > buf_len are rejected (CGPU_EINVAL); the mbuf
 *      and frame-pair entry points also check that every byte a frame may
 *      be rewritten into lies in a registered region.
 *   4  cgpu_reconcile (Packet::reconcile_all over a parsed batch).
 *   5  cgpu_reconcile_frames (the same over frames in registered host
 *      memory, in place: the mbuf seam of a reconcile combinator).
 *   6  cgpu_ctx_check (the context's device error word); cgpu_host_register
 *      takes whole pages only and refuses ranges it cannot prove are the
 *      caller's; calls captured into a graph run without the wave order;
 *      cgpu_parse_frames_submit / _wait (two bursts in flight).            */
#define CGPU_ABI_VERSION 6

/* ---- call-level return codes (negative errno style) -------------------- */
#define CGPU_OK 0
#define CGPU_EINVAL (-22)  /* bad argument (null pointer, size overflow) */
#define CGPU_ENOMEM (-12)  /* device or pinned host allocation failed      */
#define CGPU_ENODEV (-19)  /* no such HIP device                           */
#define CGPU_EIO (-5)      /* a HIP runtime call failed                    */
#define CGPU_ENOSPC (-28)  /* nat64 port table is full                     */
#define CGPU_EBUSY (-16)   /* cgpu_parse_frames_submit: two bursts in flight */

/* ---- per-packet parse status (low byte of `meta`) -----------------------
 * The first layer of the reference chain Ethernet -> Ipv4|Ipv6 -> Udp|Tcp
 * that fails decides the code; OK means all three layers parsed.          */
enum cgpu_pkt_status {
  CGPU_PKT_OK = 0,
  /* Ethernet::try_parse (ethernet.rs:279-300) */
  CGPU_PKT_ETH_BAD_OFFSET = 1,   /* read_data(0): BadOffset(0, data_len)     */
  CGPU_PKT_ETH_OUT_OF_BUFFER = 2, /* OutOfBuffer(14 or header_len, data_len) */
  /* Ipv4/Ipv6::try_parse (ip/v4.rs:427-442, ip/v6/mod.rs:274-289) */
  CGPU_PKT_NOT_IPV4 = 3,         /* "not an IPv4 packet."                    */
  CGPU_PKT_NOT_IPV6 = 4,         /* "not an IPv6 packet."                    */
  CGPU_PKT_NOT_IP = 5,           /* neither, when both were accepted        */
  CGPU_PKT_L3_BAD_OFFSET = 6,
  CGPU_PKT_L3_OUT_OF_BUFFER = 7,
  /* Udp/Tcp::try_parse (udp.rs:287-302, tcp.rs:558-573) */
  CGPU_PKT_NOT_UDP = 8,          /* "not a UDP packet."                      */
  CGPU_PKT_NOT_TCP = 9,          /* "not a TCP packet."                      */
  CGPU_PKT_NOT_L4 = 10,          /* none, when several L4 types were accepted */
  CGPU_PKT_L4_BAD_OFFSET = 11,
  CGPU_PKT_L4_OUT_OF_BUFFER = 12,
  /* nat64 only */
  CGPU_PKT_NOT_RESIZED = 13,     /* Mbuf::extend NotResized (mbuf.rs:225-233) */
  CGPU_PKT_TABLE_FULL = 14,      /* port table capacity exhausted            */
  /* Icmpv4/Icmpv6::try_parse (icmp/v4/mod.rs:205-220, icmp/v6/mod.rs:217-232) */
  CGPU_PKT_NOT_ICMPV4 = 15,      /* "not an ICMPv4 packet."                  */
  CGPU_PKT_NOT_ICMPV6 = 16,      /* "not an ICMPv6 packet."                  */
  /* SegmentRouting / Fragment::try_parse (ip/v6/srh.rs:299-327,
   * ip/v6/fragment.rs:187-202), with CGPU_F_V6_EXT */
  CGPU_PKT_EXT_BAD_OFFSET = 17,
  CGPU_PKT_EXT_OUT_OF_BUFFER = 18,
  CGPU_PKT_SRH_INCONSISTENT = 19, /* "Packet has inconsistent segment list length." */
  CGPU_PKT_STATUS_COUNT = 20
};

/* ---- `meta` word layout (one u32 per packet) ---------------------------- */
#define CGPU_META_STATUS(m) ((m) & 0xffu)        /* enum cgpu_pkt_status     */
#define CGPU_META_ETH_LEN(m) (((m) >> 8) & 0xffu) /* 14 / 18 / 22, 0 if none  */
#define CGPU_META_L3(m) (((m) >> 16) & 0x3u)      /* 0 none, 1 IPv4, 2 IPv6   */
#define CGPU_META_L4(m) (((m) >> 18) & 0x3u)      /* 0 none, 1 UDP, 2 TCP, 3 ICMP */
#define CGPU_META_IP_CSUM_OK (1u << 20)           /* stored == computed       */
#define CGPU_META_L4_CSUM_OK (1u << 21)           /* stored == computed       */
#define CGPU_META_DOT1Q (1u << 22)                /* Ethernet::is_dot1q       */
#define CGPU_META_QINQ (1u << 23)                 /* Ethernet::is_qinq        */
#define CGPU_META_EXT(m) (((m) >> 24) & 0x3u)     /* 0 none, 1 SRH, 2 Fragment */
#define CGPU_EXT_NONE 0u
#define CGPU_EXT_SRH 1u
#define CGPU_EXT_FRAGMENT 2u
#define CGPU_L3_NONE 0u
#define CGPU_L3_IPV4 1u
#define CGPU_L3_IPV6 2u
#define CGPU_L4_NONE 0u
#define CGPU_L4_UDP 1u
#define CGPU_L4_TCP 2u
#define CGPU_L4_ICMP 3u /* ICMPv4 under IPv4, ICMPv6 under IPv6 */

/* ---- parse flags --------------------------------------------------------
 * ACCEPT_* select which typed parses the caller would have written
 * (`parse::<Ipv4>()`, `parse::<Udp4>()` ...).  With both L3 (or both L4)
 * types accepted the kernel dispatches on ether_type / protocol the way a
 * `group_by` over them would (batch/group_by.rs:143-172).                 */
#define CGPU_F_ACCEPT_V4 (1u << 0)
#define CGPU_F_ACCEPT_V6 (1u << 1)
#define CGPU_F_ACCEPT_UDP (1u << 2)
#define CGPU_F_ACCEPT_TCP (1u << 3)
#define CGPU_F_ACCEPT_ALL 0xfu
#define CGPU_F_CSUM_IP (1u << 4)   /* Ipv4::compute_checksum (v4.rs:322-333) */
#define CGPU_F_CSUM_L4 (1u << 5)   /* Udp/Tcp::compute_checksum              */
#define CGPU_F_FLOW_HASH (1u << 6) /* SipHash-1-3(0,0) of `Flow` */
/* Also accept ICMPv4 (protocol 1) / ICMPv6 (next header 58) as the L4
 * layer: Icmpv4/Icmpv6::try_parse, a 4-byte header; with CGPU_F_CSUM_L4 the
 * checksum of Icmpv4::compute_checksum (no pseudo-header) / Icmpv6 (v6
 * pseudo-header, protocol 58) over [l4 offset, data_len).  ICMP has no Flow:
 * flow_hash is 0.  In the header record src_port = msg_type, dst_port =
 * code, l4_checksum = the stored checksum.  Not part of CGPU_F_ACCEPT_ALL. */
#define CGPU_F_ACCEPT_ICMP (1u << 7)
/* IPv6 extension headers: an IPv6 next header of 43 (Ipv6Route) is parsed
 * as SegmentRouting<Ipv6> (srh.rs:299-327: fixed 8-B header, then
 * hdr_ext_len == 2 * (last_entry + 1) != 0, then the segment list), 44
 * (Ipv6Frag) as Fragment<Ipv6> (fragment.rs:187-202, 8 B); the L4 layer is
 * then parsed behind it, on its next_header -- the dispatch a group_by on
 * next_header would do.  One extension level.  Behind a routing header the
 * pseudo-header and the flow use dst = segments[0] (srh.rs:421-470);
 * behind a fragment header the IPv6 addresses.                            */
#define CGPU_F_V6_EXT (1u << 8)

/* ---- batch descriptor ---------------------------------------------------
 * A batch is an arena of packet bytes plus one (offset, data_len) pair per
 * packet: the device image of a burst of single-segment mbufs
 * (buf_addr + data_off, data_len; mbuf.rs:196-205).  All pointers are
 * device pointers for the *_batch entry points.  arena_len must be <= 0xFFFF0000
 * and n <= CGPU_MAX_BATCH.                                                   */
#define CGPU_MAX_BATCH ((1u << 30) - 1u) /* 4 * n bytes of off[] fit a 32-bit buffer range */
typedef struct cgpu_batch {
  const uint8_t *arena;
  uint64_t arena_len;
  const uint32_t *off; /* [n] byte offset of packet i in the arena */
  const uint16_t *len; /* [n] data_len of packet i                 */
  uint32_t n;
} cgpu_batch;

/* Parsed header fields of one packet, host byte order.  Filled only when
 * requested; fields of layers that did not parse are zero.  96 bytes.     */
typedef struct cgpu_hdr_record {
  uint8_t dst_mac[6];          /*  0 Ethernet::dst                         */
  uint8_t src_mac[6];          /*  6 Ethernet::src                         */
  uint16_t ether_type;         /* 12 Ethernet::ether_type (VLAN aware)     */
  uint8_t eth_len;             /* 14 Ethernet::header_len                  */
  uint8_t vlan;                /* 15 0 none, 1 802.1Q, 2 802.1ad           */
  uint8_t version;             /* 16 Ipv4/Ipv6::version                    */
  uint8_t ihl;                 /* 17 Ipv4::ihl                             */
  uint8_t dscp;                /* 18                                       */
  uint8_t ecn;                 /* 19                                       */
  uint16_t ip_length;          /* 20 Ipv4::total_length / Ipv6::payload_length */
  uint16_t identification;     /* 22 Ipv4::identification                  */
  uint8_t ip_flags;            /* 24 bit0 dont_fragment, bit1 more_fragments */
  uint8_t ttl;                 /* 25 Ipv4::ttl / Ipv6::hop_limit           */
  uint16_t fragment_offset;    /* 26 Ipv4::fragment_offset                 */
  uint8_t protocol;            /* 28 Ipv4::protocol / Ipv6::next_header    */
  uint8_t pad0;                /* 29                                       */
  uint16_t ip_checksum;        /* 30 Ipv4::checksum (stored)               */
  uint32_t flow_label;         /* 32 Ipv6::flow_label                      */
  uint32_t pad1;               /* 36                                       */
  uint8_t src_ip[16];          /* 40 v4 uses the first 4 bytes             */
  uint8_t dst_ip[16];          /* 56                                       */
  uint16_t src_port;           /* 72                                       */
  uint16_t dst_port;           /* 74                                       */
  uint16_t udp_length_or_window; /* 76 Udp::length / Tcp::window           */
  uint16_t l4_checksum;        /* 78 Udp::checksum / Tcp::checksum (stored) */
  uint32_t seq_no;             /* 80 Tcp::seq_no                           */
  uint32_t ack_no;             /* 84 Tcp::ack_no                           */
  uint8_t data_offset;         /* 88 Tcp::data_offset                      */
  uint8_t tcp_flags;           /* 89 CWR..FIN = 0x80..0x01                 */
  uint8_t ns;                  /* 90 Tcp::ns                               */
  uint8_t pad2;                /* 91                                       */
  uint16_t urgent_pointer;     /* 92                                       */
  uint16_t pad3;               /* 94                                       */
} cgpu_hdr_record;

/* The extension header of one packet (CGPU_F_V6_EXT), host byte order;
 * zero when there is none or it did not parse.  48 bytes.                 */
typedef struct cgpu_ext_record {
  uint8_t kind;              /*  0 CGPU_EXT_*                               */
  uint8_t next_header;       /*  1 SegmentRouting / Fragment::next_header   */
  uint16_t header_len;       /*  2 8 + 16 * segments / 8                    */
  uint8_t hdr_ext_len;       /*  4 SegmentRouting::hdr_ext_len             */
  uint8_t routing_type;      /*  5 ::routing_type                          */
  uint8_t segments_left;     /*  6 ::segments_left                         */
  uint8_t last_entry;        /*  7 ::last_entry                            */
  uint8_t srh_flags;         /*  8 ::flags                                 */
  uint8_t more_fragments;    /*  9 Fragment::more_fragments                */
  uint16_t tag;              /* 10 SegmentRouting::tag                     */
  uint16_t fragment_offset;  /* 12 Fragment::fragment_offset               */
  uint16_t pad0;             /* 14                                         */
  uint32_t identification;   /* 16 Fragment::identification                */
  uint32_t pad1;             /* 20                                         */
  uint8_t segment0[16];      /* 24 SegmentRouting::segments()[0] (= dst()) */
  uint8_t pad2[8];           /* 40                                         */
} cgpu_ext_record;

/* Outputs of cgpu_parse_batch, all device pointers with n entries.       */
typedef struct cgpu_parse_out {
  uint32_t *meta;       /* required                                          */
  uint32_t *csum;       /* ip_calc | l4_calc << 16, or NULL: verify only (the
                         * CSUM_OK bits of meta are set either way)          */
  uint64_t *flow_hash;  /* required with CGPU_F_FLOW_HASH                     */
  cgpu_hdr_record *fields; /* optional (NULL = skip field extraction)        */
  cgpu_ext_record *ext;    /* optional (NULL = skip); all-zero records unless
                           * CGPU_F_V6_EXT parsed an extension header       */
} cgpu_parse_out;

typedef struct cgpu_ctx cgpu_ctx;

/* ---- context ------------------------------------------------------------
 * One context per core thread / RX queue (reference runtime/core_map.rs:
 * 236-293: shared-nothing).  Contexts are independent; the library keeps
 * no global locks on the launch path.                                     */
int cgpu_ctx_create(int hip_device, cgpu_ctx **out);
/* Waits for the context's own stream, then frees everything the context
 * holds and unregisters its host regions.                                 */
void cgpu_ctx_destroy(cgpu_ctx *ctx);

/* The context's device error word: kernels that cannot complete their part
 * of a call set it instead of failing silently (today: a wave of the
 * longest-span-first order that gave up waiting for its group, which leaves
 * that group's 64 outputs unwritten).  Synchronises `stream`, then returns
 * CGPU_EIO if the word was set by any call of this context since it was
 * last read (and clears it), else 0.  The synchronous entry points read it
 * themselves and fail with CGPU_EIO; asynchronous callers (cgpu_parse_batch,
 * cgpu_reconcile) call this where they synchronise, as a CUDA caller checks
 * a sticky error.                                                          */
int cgpu_ctx_check(cgpu_ctx *ctx, void *stream);

/* Batched Ethernet -> IPv4/IPv6 -> UDP/TCP parse + checksum + flow hash.
 * Replaces the per-packet chain Mbuf::parse::<Ethernet>() (ethernet.rs:279)
 * -> parse::<Ipv4|Ipv6>() (v4.rs:427 / v6/mod.rs:274) -> parse::<Udp|Tcp>()
 * (udp.rs:287 / tcp.rs:558), plus Ipv4::compute_checksum (v4.rs:322),
 * Udp/Tcp::compute_checksum (udp.rs:204 / tcp.rs:462) evaluated on the bytes
 * as they are, and the hash of Udp/Tcp::flow() (udp.rs:151, tcp.rs:409).
 * Asynchronous on `stream`.  A batch of more than one round of waves (64
 * frames a wave, 32 waves resident per CU) with checksums over long frames
 * orders its later waves longest span first (from half a round on when the
 * stream's previous ordered batch had spans that vary, else from the second
 * round on) through a 128 KB buffer the
 * context keeps per stream (allocated by the first such call on a stream
 * and zeroed on that stream; no device-wide synchronisation).  A call made
 * while its stream is being captured into a graph runs without the order
 * (replays would share the buffer), as does one whose buffer cannot be
 * allocated.  The results do not depend on the order.                    */
int cgpu_parse_batch(cgpu_ctx *ctx, const cgpu_batch *batch, uint32_t flags,
                     const cgpu_parse_out *out, void *stream);

/* Host-memory variant for the DPDK seam: gathers `n` host packets (e.g.
 * rte_mbuf data addresses, mbuf.rs:202-205) into pinned staging, copies to
 * the device, parses, and copies the outputs back into HOST arrays (any of
 * csum / flow_hash / fields may be NULL).  Synchronous.                    */
int cgpu_parse_host(cgpu_ctx *ctx, const uint8_t *const *pkt, const uint16_t *len,
                    uint32_t n, uint32_t flags, uint32_t *meta, uint32_t *csum,
                    uint64_t *flow_hash, cgpu_hdr_record *fields);

/* ---- rte_mbuf bursts (the DPDK seam) -------------------------------------
 * A burst as PacketRx::receive returns it (Vec<Mbuf>, batch/mod.rs:110-119,
 * port.rs:149-205): an array of rte_mbuf pointers.  The library reads three
 * fields of each rte_mbuf, at the DPDK 19.11 offsets pinned by the bindgen
 * layout test (ffi/src/bindings_rustdoc.rs:6869-6898): buf_addr, data_off,
 * data_len.  Only the first segment is read, like Mbuf::data_len and
 * read_data (mbuf.rs:196, 313-327).  The mbufs are borrowed for the call
 * (never freed or kept, mbuf.rs:467-479).                                   */
#define CGPU_MBUF_BUF_ADDR_OFF 0
#define CGPU_MBUF_DATA_OFF_OFF 16
#define CGPU_MBUF_DATA_LEN_OFF 40
#define CGPU_MBUF_SIZE 128

/* Ingress modes.
 *   STAGE:     the calling core gathers each frame into pinned staging
 *              (64-B slots) and one DMA copies the burst to the device.
 *   ZERO_COPY: the device reads the mbufs and their frames straight from
 *              host memory over PCIe into HBM; every mbuf and data buffer
 *              must lie in a region registered with cgpu_host_register (a
 *              mempool's memzone).  A pointer outside every registered
 *              region fails the call with CGPU_EINVAL (nothing is read
 *              through it).                                                */
#define CGPU_INGRESS_STAGE 0u
#define CGPU_INGRESS_ZERO_COPY 1u

/* Page-lock and map host memory [base, base + bytes) for the device (the
 * mempool of mempool.rs:64-106); up to 16 regions per context.
 * base and bytes must be multiples of the page size (a DPDK memzone always
 * is), and no two regions of a context may overlap; otherwise CGPU_EINVAL.
 * Pageable memory is registered (hipHostRegister) and unregistered again by
 * cgpu_host_unregister / cgpu_ctx_destroy.  Memory that is already
 * page-locked is only mapped, and only if the whole range lies inside one
 * pinned allocation (hipHostMalloc, torch pinned memory); a range that
 * straddles pinned and pageable pages, or several pinned allocations, is
 * refused.  Lifetime (the ownership rule of mbuf.rs:467-479): the caller
 * keeps the range mapped, and a pinned allocation allocated, until the
 * region is unregistered; the library never frees or unmaps it.
 * cgpu_host_unregister waits for the context's stream (every call that
 * touches registered memory runs there) before unpinning.               */
int cgpu_host_register(cgpu_ctx *ctx, void *base, size_t bytes);
int cgpu_host_unregister(cgpu_ctx *ctx, void *base);

/* Parse a burst of n rte_mbufs; outputs as cgpu_parse_host, into HOST
 * arrays (csum / flow_hash / fields may be NULL).  Synchronous: the burst's
 * results are in the host arrays when the call returns.                  */
int cgpu_parse_mbufs(cgpu_ctx *ctx, void *const *mbufs, uint32_t n, uint32_t flags,
                     uint32_t ingress, uint32_t *meta, uint32_t *csum, uint64_t *flow_hash,
                     cgpu_hdr_record *fields);

/* Parse a burst of n frames handed over as host (address, length) pairs --
 * each mbuf's data_address / data_len (mbuf.rs:196-205), which the RX core
 * has in cache right after rte_eth_rx_burst; outputs as cgpu_parse_host, in
 * HOST arrays.  STAGE: the calling core gathers (= cgpu_parse_host).
 * ZERO_COPY: the device reads the frames alone from regions registered with
 * cgpu_host_register -- no mbuf header line per packet, as
 * cgpu_parse_mbufs must read; a frame outside every registered region fails
 * the call with CGPU_EINVAL (nothing is read through it).  Synchronous.   */
int cgpu_parse_frames(cgpu_ctx *ctx, const uint8_t *const *pkt, const uint16_t *len, uint32_t n,
                      uint32_t flags, uint32_t ingress, uint32_t *meta, uint32_t *csum,
                      uint64_t *flow_hash, cgpu_hdr_record *fields);

/* The same as cgpu_parse_frames with CGPU_INGRESS_ZERO_COPY, split in two
 * so that the caller's core works on one burst while the device parses the
 * next (double buffering at the seam of a batch combinator): submit copies
 * the burst's descriptors, launches, and returns a ticket at once; the
 * results are in meta / csum / flow_hash (which must stay valid until then;
 * pkt / len need not) when cgpu_parse_frames_wait(ticket) returns 0.  At
 * most two bursts per context are in flight: a third submit fails with
 * CGPU_EBUSY.  Bursts are parsed in submission order.  A burst the one-launch
 * path cannot take (frames in several registered regions, more than 2^20
 * frames) is parsed synchronously inside submit, and its wait returns that
 * call's result.  No header records (use cgpu_parse_frames for those).    */
int cgpu_parse_frames_submit(cgpu_ctx *ctx, const uint8_t *const *pkt, const uint16_t *len,
                             uint32_t n, uint32_t flags, uint32_t *meta, uint32_t *csum,
                             uint64_t *flow_hash, uint32_t *ticket);
int cgpu_parse_frames_wait(cgpu_ctx *ctx, uint32_t ticket);

/* ---- examples/nat64 6to4 -------------------------------------------------
 * Stateful IPv6 -> IPv4 rewrite of examples/nat64/main.rs:121-150, with the
 * port map of :37-53 held on the device.  NEXT_PORT starts at `first_port`
 * (1025 in the reference) and wraps modulo 2^16 like AtomicU16::fetch_add. */
typedef struct cgpu_portmap cgpu_portmap;

/* capacity_log2: table slots = 2^capacity_log2 (keep load < 0.5).         */
int cgpu_portmap_create(cgpu_ctx *ctx, uint32_t capacity_log2, uint16_t first_port,
                        cgpu_portmap **out);
void cgpu_portmap_destroy(cgpu_portmap *pm);
/* Synchronous reads of the map state (test/debug helpers).  They wait for
 * the map's latest call by an event the library records on that call's
 * stream, so the caller may destroy the stream first.                     */
int cgpu_portmap_next_port(cgpu_portmap *pm, uint16_t *next_port);
int cgpu_portmap_size(cgpu_portmap *pm, uint32_t *entries);
/* Empty the map again (PORT_MAP, ADDR_MAP, NEXT_PORT = first_port), as a
 * fresh cgpu_portmap_create would leave it, asynchronously on `stream`
 * behind the map's earlier calls.  Calls on one map are ordered: a call on
 * another stream than the previous one waits for it.                      */
int cgpu_portmap_reset(cgpu_portmap *pm, uint16_t first_port, void *stream);

/* Disposition per packet (reference batch/mod.rs:54-107, filter_map.rs:73):
 * ACT = Either::Keep (emitted), DROP = Either::Drop, ABORT = Err.          */
enum cgpu_disposition { CGPU_ACT = 0, CGPU_DROP = 1, CGPU_ABORT = 2 };

/* in:  device batch of frames.  out_arena/out_off: where frame i is written
 * (out_off[i] must leave room for len[i] bytes; out_arena must not overlap
 * the input arena).  out_len[i] = new data_len for ACT packets.
 * disposition[i] = enum cgpu_disposition; status[i] = enum cgpu_pkt_status
 * explaining an ABORT.  All device pointers; asynchronous on `stream`.     */
int cgpu_nat64_6to4(cgpu_ctx *ctx, cgpu_portmap *pm, const cgpu_batch *in,
                    uint8_t *out_arena, uint64_t out_arena_len, const uint32_t *out_off,
                    uint16_t *out_len, uint8_t *disposition, uint8_t *status, void *stream);

/* ---- examples/nat64 4to6 -------------------------------------------------
 * IPv4 -> IPv6 rewrite of examples/nat64/main.rs:86-118: TCP frames that are
 * not fragments and whose destination port the 6to4 direction assigned
 * (ADDR_MAP, :38, :56-58 — the same cgpu_portmap) become IPv6 frames to the
 * original v6 source and port, from 64:ff9b::<v4 src>; everything else is
 * DROP (or ABORT on a parse error).  Output frames are 20 bytes longer than
 * the input (out_off[i] must leave room for len[i] + 20 bytes).  Same
 * argument conventions as cgpu_nat64_6to4.                                   */
int cgpu_nat64_4to6(cgpu_ctx *ctx, cgpu_portmap *pm, const cgpu_batch *in,
                    uint8_t *out_arena, uint64_t out_arena_len, const uint32_t *out_off,
                    uint16_t *out_len, uint8_t *disposition, uint8_t *status, void *stream);

/* ---- nat64 over an rte_mbuf burst (the DPDK seam, both directions) -------
 * install_6to4 / install_4to6 (examples/nat64/main.rs:152-165) applied to a
 * burst exactly as PacketRx::receive returns it (an array of rte_mbuf*): the
 * device reads the frames from the registered mempool (cgpu_host_register,
 * zero-copy), rewrites them as cgpu_nat64_6to4 / cgpu_nat64_4to6, and writes
 * every ACT frame back into its own mbuf over PCIe: the new frame at
 * buf_addr + data_off (Mbuf::shrink / extend move bytes, never data_off,
 * mbuf.rs:225-270), data_len and pkt_len changed by -20 (6to4) / +20 (4to6).
 * 4to6 checks extend's `20 < tailroom` (mbuf.rs:228) against the mbuf's own
 * buf_len (@54); without the room the packet is ABORT / NOT_RESIZED.  DROP
 * and ABORT mbufs are not touched: the caller frees or forwards them
 * (Send::run, batch/send.rs:95-118).  disposition / status: HOST arrays [n].
 * Synchronous.  Fails with CGPU_EINVAL if a pointer lies outside every
 * registered region (nothing is read or written through it).             */
#define CGPU_NAT64_6TO4 0u
#define CGPU_NAT64_4TO6 1u
#define CGPU_MBUF_PKT_LEN_OFF 36
#define CGPU_MBUF_BUF_LEN_OFF 54
int cgpu_nat64_mbufs(cgpu_ctx *ctx, cgpu_portmap *pm, uint32_t direction, void *const *mbufs,
                     uint32_t n, uint8_t *disposition, uint8_t *status);

/* The same over a burst handed over as frame pairs: frames[i] / len[i] =
 * data_address / data_len of mbuf i (mbuf.rs:196-205), tailroom[i] =
 * buf_len - data_off - data_len (Mbuf::tailroom, mbuf.rs:207-213; needed by
 * 4to6's extend check, may be NULL for 6to4).  The device reads and writes
 * only the frames (in registered memory, rewritten in place, every call all
 * or nothing as above); out_len[i] is the new data_len of each ACT frame (0
 * otherwise), which the caller stores into data_len / pkt_len.            */
int cgpu_nat64_frames(cgpu_ctx *ctx, cgpu_portmap *pm, uint32_t direction,
                      const uint8_t *const *frames, const uint16_t *len, const uint16_t *tailroom,
                      uint32_t n, uint16_t *out_len, uint8_t *disposition, uint8_t *status);

/* ---- group_by (core/src/batch/group_by.rs:143-172) -----------------------
 * Stable partition of a batch's packet indices by a per-packet arm key: the
 * device form of `batch.group_by(selector, compose!{...})`.  Arm k (k <
 * n_groups - 1) receives the packets whose key is k, in batch order; every
 * other key goes to the last arm, the catch-all (`_ =>` / the implicit
 * pass-through arm of compose!, group_by.rs:186-200).  The per-arm counts
 * double as the disposition counters of send.rs:104-110 when the key is a
 * cgpu_disposition array.
 *   key_kind CGPU_KEY_U8:         key = const uint8_t[n] (e.g. disposition)
 *   key_kind CGPU_KEY_META_CLASS: key = const uint32_t[n] parse meta words;
 *     arm = 0 v4/UDP, 1 v4/TCP, 2 v6/UDP, 3 v6/TCP, 4 everything else
 *     (status != OK, or an L4 layer other than UDP/TCP, i.e. ICMP)
 * idx[n]: packet indices grouped by arm; group_off[n_groups + 1]: arm k owns
 * idx[group_off[k] .. group_off[k+1]).  n_groups in 1..64, n <= 2^28.  All
 * device pointers; asynchronous on `stream`.  Uses per-context scratch: one
 * stream at a time per context (one context per core thread, as everywhere). */
#define CGPU_KEY_U8 0u
#define CGPU_KEY_META_CLASS 1u
int cgpu_group_by(cgpu_ctx *ctx, const void *key, uint32_t key_kind, uint32_t n,
                  uint32_t n_groups, uint32_t *idx, uint32_t *group_off, void *stream);

/* ---- Udp/Tcp::set_src_ip / set_dst_ip (udp.rs:174-201, tcp.rs:432-459) ----
 * Address rewrite with the incremental L4 checksum update, over a parsed
 * batch (the bytes cgpu_parse_batch saw, its meta words).  For each packet
 * whose meta is OK with a UDP or TCP layer (no extension header), in the
 * order the reference's test calls them: if `src` is given,
 * `set_src_ip(src[i * src_stride])`, then if `dst` is given,
 * `set_dst_ip(dst[...])`.  Each is checksum::compute_with_ipaddr
 * (checksum.rs:202-220: RFC 1624 `~(~HC + ~m + m')` over the 2 (v4) or 8
 * (v6) address words of checksum.rs:182-195) on the stored checksum, then
 * the address store, then Udp/Tcp::set_checksum (UDP stores 0 as 0xFFFF,
 * udp.rs:132-141).  The IPv4 header checksum is left as it is, like
 * Ipv4::set_src/set_dst (v4.rs:343-357).  An address of the other family
 * fails that call with "cannot mix IPv4 and IPv6 addresses." and changes
 * nothing (an earlier src update stays).  stride 0 broadcasts entry 0.
 * status (optional, u8 per packet) = enum cgpu_setip_status.  The arena is
 * updated in place; all device pointers; asynchronous on `stream`.         */
typedef struct cgpu_ip_addr {
  uint8_t octets[16]; /* wire order; IPv4 uses the first 4                  */
  uint32_t family;    /* 4 or 6                                             */
} cgpu_ip_addr;
enum cgpu_setip_status {
  CGPU_SETIP_OK = 0,
  CGPU_SETIP_SKIPPED = 1,      /* meta not OK, or no UDP/TCP layer: untouched */
  CGPU_SETIP_SRC_MISMATCH = 2, /* src family != packet's: untouched          */
  CGPU_SETIP_DST_MISMATCH = 3, /* dst family != packet's: src (if any) applied */
};
int cgpu_set_ip(cgpu_ctx *ctx, uint8_t *arena, uint64_t arena_len, const uint32_t *off,
                const uint16_t *len, const uint32_t *meta, uint32_t n, const cgpu_ip_addr *src,
                uint32_t src_stride, const cgpu_ip_addr *dst, uint32_t dst_stride,
                uint8_t *status, void *stream);

/* ---- Packet::reconcile_all (core/src/packets/mod.rs:297-300) -------------
 * The transmit-side fix-up of a header-modifying pipeline, in place, over a
 * parsed batch (the frames cgpu_parse_batch saw, possibly modified since,
 * and its meta words; data_len as in `len`).  Every packet is taken as the
 * typed packet held at layer `depth` -- the layers and offsets its meta
 * records, as a typed packet keeps the offsets of its parse -- and
 * reconciled from that layer outward, as reconcile_all walks the envelopes:
 *   CGPU_LAYER_L4  Udp::reconcile (udp.rs:350-354): length := data_len -
 *                  offset, then compute_checksum (:204-219) on the frame with
 *                  that length, 0 stored as 0xFFFF (set_checksum :132-141);
 *                  Tcp::reconcile (tcp.rs:619-621): compute_checksum;
 *                  Icmpv4 / Icmpv6::reconcile (icmp/v4/mod.rs:246-248,
 *                  icmp/v6/mod.rs:260-262): compute_checksum.  Behind an
 *                  IPv6 extension header (CGPU_F_V6_EXT meta) the
 *                  pseudo-header is the parse's (segments[0] behind a routing
 *                  header); SegmentRouting / Fragment reconcile nothing
 *                  (packets/mod.rs:288).  Then the L3 layer:
 *   CGPU_LAYER_L3  Ipv4::reconcile (ip/v4.rs:486-489): total_length :=
 *                  data_len - offset, then the header checksum;
 *                  Ipv6::reconcile (ip/v6/mod.rs:331-334): payload_length :=
 *                  data_len - offset - 40.
 *   CGPU_LAYER_L2  Ethernet: nothing (the default reconcile).
 * A packet whose parse did not reach `depth` (its meta has no such layer:
 * the typed parse failed and the reference would hold an Err), or whose
 * layers no longer fit in data_len, is not touched.  status (optional, u8
 * per packet) = enum cgpu_recon_status.  flags: the accept set the parse ran
 * with (CGPU_F_ACCEPT_*, CGPU_F_ACCEPT_ICMP, CGPU_F_V6_EXT, defaults as in
 * cgpu_parse_batch; other bits are ignored): a packet whose meta records a
 * layer up to `depth` outside it is SKIPPED, and the set selects the kernel
 * variant (IPv4/UDP only compiles the other branches out).  Frames must not
 * overlap.  All device pointers; asynchronous on `stream`.                 */
#define CGPU_LAYER_L2 2u
#define CGPU_LAYER_L3 3u
#define CGPU_LAYER_L4 4u
enum cgpu_recon_status { CGPU_RECON_OK = 0, CGPU_RECON_SKIPPED = 1 };
int cgpu_reconcile(cgpu_ctx *ctx, uint8_t *arena, uint64_t arena_len, const uint32_t *off,
                   const uint16_t *len, const uint32_t *meta, uint32_t n, uint32_t flags,
                   uint32_t depth, uint8_t *status, void *stream);

/* The same over a burst as the RX path hands it over: frames[i] =
 * Mbuf::data_address(0), len[i] = data_len (mbuf.rs:196-205), in memory
 * registered with cgpu_host_register (a mempool's memzone), reconciled in
 * place through the device's mapping of that memory: no staging copy, the
 * device reads each frame once and writes the rewritten fields back.
 * meta[i]: the words a parse of these bytes returned (host array, e.g. from
 * cgpu_parse_frames), flags / depth / status (host, optional) as
 * cgpu_reconcile.  Every frame must lie wholly inside one registered region,
 * and a region's frames of one call within 4 GiB - 64 KiB of each other;
 * otherwise CGPU_EINVAL and nothing is written.  Synchronous; uses the
 * context's stream (one call at a time per context).  Replaces
 * packet.reconcile_all() (packets/mod.rs:297-300) inside a pipeline closure
 * over a burst whose typed packets came from the device parse.              */
int cgpu_reconcile_frames(cgpu_ctx *ctx, uint8_t *const *frames, const uint16_t *len,
                          const uint32_t *meta, uint32_t n, uint32_t flags, uint32_t depth,
                          uint8_t *status);

/* ---- errors -------------------------------------------------------------- */
int cgpu_last_error(void);
const char *cgpu_strerror(int code);
const char *cgpu_pkt_status_str(int status);
int cgpu_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* CAPSULE_GPU_H */
