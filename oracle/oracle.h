/*
 * oracle.h — CPU restatement of Capsule's packet hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in capsule_amd/ links or calls this;
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg do,
 * as the checker / CPU baseline.  Every function follows the reference
 * source (/root/reference, file:line in oracle.c) scalar step by scalar step
 * and reports results in the same output contract as include/capsule_gpu.h.
 *
 * Pinned by the reference's own known-answer tests (tests/golden/, see
 * tests/test_oracle_golden.py).  The flow-hash convention has no reference
 * vector: that part is "parity unpinned" (DESIGN.md §4).
 */
#ifndef CAPSULE_ORACLE_H
#define CAPSULE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/capsule_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* checksum.rs */
uint16_t or_compute(uint16_t pseudo_header_sum, const uint8_t *payload, size_t len);
uint16_t or_compute_inc(uint16_t old_checksum, const uint16_t *old_value,
                        const uint16_t *new_value, size_t n);
uint16_t or_pseudo_v4(uint32_t src, uint32_t dst, uint16_t packet_len, uint8_t protocol);
uint16_t or_pseudo_v6(const uint8_t src[16], const uint8_t dst[16], uint16_t packet_len,
                      uint8_t protocol);

/* SipHash-c-d with 128-bit key (k0, k1); DefaultHasher::new() = c1 d3, k 0. */
uint64_t or_siphash(int c_rounds, int d_rounds, uint64_t k0, uint64_t k1, const uint8_t *msg,
                    size_t len);
/* Byte stream that Rust 1.50 #[derive(Hash)] on Flow writes (29 / 69 B). */
size_t or_flow_bytes(int v6, const uint8_t *src, const uint8_t *dst, uint16_t src_port,
                     uint16_t dst_port, uint8_t protocol, uint8_t out[69]);
uint64_t or_flow_hash(int v6, const uint8_t *src, const uint8_t *dst, uint16_t src_port,
                      uint16_t dst_port, uint8_t protocol);

/* Batched parse with the cgpu_parse_batch output contract (host memory). */
/* or_parse_batch plus the extension records (CGPU_F_V6_EXT); ext may be NULL */
void or_parse_batch_ext(const uint8_t *arena, const uint32_t *off, const uint16_t *len,
                        uint32_t n, uint32_t flags, uint32_t *meta, uint32_t *csum,
                        uint64_t *flow_hash, cgpu_hdr_record *fields, cgpu_ext_record *ext);
void or_parse_batch(const uint8_t *arena, const uint32_t *off, const uint16_t *len, uint32_t n,
                    uint32_t flags, uint32_t *meta, uint32_t *csum, uint64_t *flow_hash,
                    cgpu_hdr_record *fields);

/* bench/packets.rs multi_parse_udp (:65-69): Ethernet -> Ipv4 -> Udp4 parse
 * only; returns the number of packets whose parse succeeded.             */
uint32_t or_multi_parse_udp(const uint8_t *arena, const uint32_t *off, const uint16_t *len,
                            uint32_t n);

/* examples/nat64 6to4 with a host port map (examples/nat64/main.rs). */
typedef struct or_portmap or_portmap;
or_portmap *or_portmap_new(uint16_t first_port);
void or_portmap_free(or_portmap *pm);
uint16_t or_portmap_next_port(const or_portmap *pm);
uint32_t or_portmap_size(const or_portmap *pm);
/* Data room of the simulated mbufs nat64 runs in (default 2048, DPDK's
 * RTE_MBUF_DEFAULT_DATAROOM); a test of a custom mempool sets its own. */
void or_set_mbuf_data_room(uint32_t room);
void or_nat64_6to4(or_portmap *pm, const uint8_t *arena, const uint32_t *off, const uint16_t *len,
                   uint32_t n, uint8_t *out_arena, const uint32_t *out_off, uint16_t *out_len,
                   uint8_t *disposition, uint8_t *status);

/* examples/nat64 4to6 (main.rs:86-118) with the same port map's ADDR_MAP. */
void or_nat64_4to6(or_portmap *pm, const uint8_t *arena, const uint32_t *off, const uint16_t *len,
                   uint32_t n, uint8_t *out_arena, const uint32_t *out_off, uint16_t *out_len,
                   uint8_t *disposition, uint8_t *status);

/* core/src/batch/group_by.rs:143-172 over a burst: packets visited in
 * order, each appended to the arm its key selects (catch-all = last arm).
 * key_kind / arms as cgpu_group_by.                                      */
void or_group_by(const void *key, uint32_t key_kind, uint32_t n, uint32_t n_groups, uint32_t *idx,
                 uint32_t *group_off);

/* Udp/Tcp::set_src_ip then set_dst_ip (udp.rs:174-201, tcp.rs:432-459) on
 * the packets or_parse_batch accepted as UDP/TCP; contract of cgpu_set_ip. */
void or_set_ip(uint8_t *arena, const uint32_t *off, const uint16_t *len, const uint32_t *meta,
               uint32_t n, const cgpu_ip_addr *src, uint32_t src_stride, const cgpu_ip_addr *dst,
               uint32_t dst_stride, uint8_t *status);

/* Packet::reconcile_all (packets/mod.rs:297-300) at layer `depth` over the
 * packets of a parsed batch, in place; contract of cgpu_reconcile.        */
void or_reconcile(uint8_t *arena, uint64_t arena_len, const uint32_t *off, const uint16_t *len,
                  const uint32_t *meta, uint32_t n, uint32_t flags, uint32_t depth, uint8_t *status);

#ifdef __cplusplus
}
#endif

#endif
