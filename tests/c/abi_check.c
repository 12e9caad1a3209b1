/* Plain-C (C11, no HIP) consumer of include/capsule_gpu.h: the stand-in for
 * the bindgen step a Rust binding crate would run (reference ffi/build.rs:
 * 171-199), which cannot run here.  It compiles the header as C, pins the
 * record layouts the Rust side would mirror, and pins the rte_mbuf field
 * offsets the library reads against the reference's own bindgen layout test
 * for DPDK 19.11 (ffi/src/bindings_rustdoc.rs:6869-6898: buf_addr @0,
 * data_off @16, pkt_len @36, data_len @40, buf_len @54, 128-byte struct).
 * Built and run by tests/test_abi.py with gcc -std=c11 -Wall -Wextra
 * -Werror -pedantic. */
#include <stddef.h>
#include <stdio.h>

#include "capsule_gpu.h"

/* rte_mbuf offsets (ffi/src/bindings_rustdoc.rs:6869-6898) */
_Static_assert(CGPU_MBUF_BUF_ADDR_OFF == 0, "rte_mbuf.buf_addr");
_Static_assert(CGPU_MBUF_DATA_OFF_OFF == 16, "rte_mbuf.data_off");
_Static_assert(CGPU_MBUF_PKT_LEN_OFF == 36, "rte_mbuf.pkt_len");
_Static_assert(CGPU_MBUF_DATA_LEN_OFF == 40, "rte_mbuf.data_len");
_Static_assert(CGPU_MBUF_BUF_LEN_OFF == 54, "rte_mbuf.buf_len");
_Static_assert(CGPU_MBUF_SIZE == 128, "sizeof(rte_mbuf)");

/* records: sizes and the offsets the header comments promise */
_Static_assert(sizeof(cgpu_hdr_record) == 96, "cgpu_hdr_record size");
_Static_assert(offsetof(cgpu_hdr_record, ether_type) == 12, "ether_type");
_Static_assert(offsetof(cgpu_hdr_record, eth_len) == 14, "eth_len");
_Static_assert(offsetof(cgpu_hdr_record, ip_length) == 20, "ip_length");
_Static_assert(offsetof(cgpu_hdr_record, fragment_offset) == 26, "fragment_offset");
_Static_assert(offsetof(cgpu_hdr_record, ip_checksum) == 30, "ip_checksum");
_Static_assert(offsetof(cgpu_hdr_record, flow_label) == 32, "flow_label");
_Static_assert(offsetof(cgpu_hdr_record, src_ip) == 40, "src_ip");
_Static_assert(offsetof(cgpu_hdr_record, dst_ip) == 56, "dst_ip");
_Static_assert(offsetof(cgpu_hdr_record, src_port) == 72, "src_port");
_Static_assert(offsetof(cgpu_hdr_record, l4_checksum) == 78, "l4_checksum");
_Static_assert(offsetof(cgpu_hdr_record, seq_no) == 80, "seq_no");
_Static_assert(offsetof(cgpu_hdr_record, data_offset) == 88, "data_offset");
_Static_assert(offsetof(cgpu_hdr_record, urgent_pointer) == 92, "urgent_pointer");
_Static_assert(sizeof(cgpu_ext_record) == 48, "cgpu_ext_record size");
_Static_assert(offsetof(cgpu_ext_record, tag) == 10, "tag");
_Static_assert(offsetof(cgpu_ext_record, identification) == 16, "identification");
_Static_assert(offsetof(cgpu_ext_record, segment0) == 24, "segment0");
_Static_assert(sizeof(cgpu_ip_addr) == 20, "cgpu_ip_addr size");
_Static_assert(offsetof(cgpu_ip_addr, family) == 16, "cgpu_ip_addr.family");

/* descriptor structs as a 64-bit C compiler lays them out */
_Static_assert(sizeof(cgpu_batch) == 40, "cgpu_batch size");
_Static_assert(offsetof(cgpu_batch, n) == 32, "cgpu_batch.n");
_Static_assert(sizeof(cgpu_parse_out) == 40, "cgpu_parse_out size");

/* status codes and meta layout */
_Static_assert(CGPU_PKT_STATUS_COUNT == 20, "status count");
_Static_assert(CGPU_META_L4((unsigned)CGPU_L4_ICMP << 18) == CGPU_L4_ICMP, "meta L4 field");
_Static_assert(CGPU_MAX_BATCH * 4ull <= 0xffffffffull, "off[] fits a 32-bit range");

/* every entry point, bound through a pointer of exactly the C type a
 * binding generator would emit for it (a signature change fails to compile) */
typedef void (*any_fn)(void);
static int (*const p_ctx_create)(int, cgpu_ctx **) = cgpu_ctx_create;
static void (*const p_ctx_destroy)(cgpu_ctx *) = cgpu_ctx_destroy;
static int (*const p_ctx_check)(cgpu_ctx *, void *) = cgpu_ctx_check;
static int (*const p_frames_submit)(cgpu_ctx *, const uint8_t *const *, const uint16_t *, uint32_t,
                                    uint32_t, uint32_t *, uint32_t *, uint64_t *,
                                    uint32_t *) = cgpu_parse_frames_submit;
static int (*const p_frames_wait)(cgpu_ctx *, uint32_t) = cgpu_parse_frames_wait;
static int (*const p_parse_batch)(cgpu_ctx *, const cgpu_batch *, uint32_t,
                                  const cgpu_parse_out *, void *) = cgpu_parse_batch;
static int (*const p_parse_host)(cgpu_ctx *, const uint8_t *const *, const uint16_t *, uint32_t,
                                 uint32_t, uint32_t *, uint32_t *, uint64_t *,
                                 cgpu_hdr_record *) = cgpu_parse_host;
static int (*const p_host_register)(cgpu_ctx *, void *, size_t) = cgpu_host_register;
static int (*const p_host_unregister)(cgpu_ctx *, void *) = cgpu_host_unregister;
static int (*const p_parse_mbufs)(cgpu_ctx *, void *const *, uint32_t, uint32_t, uint32_t,
                                  uint32_t *, uint32_t *, uint64_t *,
                                  cgpu_hdr_record *) = cgpu_parse_mbufs;
static int (*const p_parse_frames)(cgpu_ctx *, const uint8_t *const *, const uint16_t *, uint32_t,
                                   uint32_t, uint32_t, uint32_t *, uint32_t *, uint64_t *,
                                   cgpu_hdr_record *) = cgpu_parse_frames;
static int (*const p_nat64_frames)(cgpu_ctx *, cgpu_portmap *, uint32_t, const uint8_t *const *,
                                   const uint16_t *, const uint16_t *, uint32_t, uint16_t *,
                                   uint8_t *, uint8_t *) = cgpu_nat64_frames;
static int (*const p_portmap_create)(cgpu_ctx *, uint32_t, uint16_t,
                                     cgpu_portmap **) = cgpu_portmap_create;
static void (*const p_portmap_destroy)(cgpu_portmap *) = cgpu_portmap_destroy;
static int (*const p_portmap_next_port)(cgpu_portmap *, uint16_t *) = cgpu_portmap_next_port;
static int (*const p_portmap_size)(cgpu_portmap *, uint32_t *) = cgpu_portmap_size;
static int (*const p_portmap_reset)(cgpu_portmap *, uint16_t, void *) = cgpu_portmap_reset;
static int (*const p_nat64_6to4)(cgpu_ctx *, cgpu_portmap *, const cgpu_batch *, uint8_t *,
                                 uint64_t, const uint32_t *, uint16_t *, uint8_t *, uint8_t *,
                                 void *) = cgpu_nat64_6to4;
static int (*const p_nat64_4to6)(cgpu_ctx *, cgpu_portmap *, const cgpu_batch *, uint8_t *,
                                 uint64_t, const uint32_t *, uint16_t *, uint8_t *, uint8_t *,
                                 void *) = cgpu_nat64_4to6;
static int (*const p_nat64_mbufs)(cgpu_ctx *, cgpu_portmap *, uint32_t, void *const *, uint32_t,
                                  uint8_t *, uint8_t *) = cgpu_nat64_mbufs;
static int (*const p_group_by)(cgpu_ctx *, const void *, uint32_t, uint32_t, uint32_t,
                               uint32_t *, uint32_t *, void *) = cgpu_group_by;
static int (*const p_set_ip)(cgpu_ctx *, uint8_t *, uint64_t, const uint32_t *,
                             const uint16_t *, const uint32_t *, uint32_t, const cgpu_ip_addr *,
                             uint32_t, const cgpu_ip_addr *, uint32_t, uint8_t *,
                             void *) = cgpu_set_ip;
static int (*const p_reconcile)(cgpu_ctx *, uint8_t *, uint64_t, const uint32_t *,
                                const uint16_t *, const uint32_t *, uint32_t, uint32_t, uint32_t,
                                uint8_t *, void *) = cgpu_reconcile;
static int (*const p_reconcile_frames)(cgpu_ctx *, uint8_t *const *, const uint16_t *,
                                       const uint32_t *, uint32_t, uint32_t, uint32_t,
                                       uint8_t *) = cgpu_reconcile_frames;
static int (*const p_last_error)(void) = cgpu_last_error;
static const char *(*const p_strerror)(int) = cgpu_strerror;
static const char *(*const p_pkt_status_str)(int) = cgpu_pkt_status_str;
static int (*const p_abi_version)(void) = cgpu_abi_version;

static const any_fn entry_points[] = {
    (any_fn)p_ctx_create,     (any_fn)p_ctx_destroy,      (any_fn)p_parse_batch,
    (any_fn)p_parse_host,     (any_fn)p_host_register,    (any_fn)p_host_unregister,
    (any_fn)p_parse_mbufs,    (any_fn)p_portmap_create,   (any_fn)p_portmap_destroy,
    (any_fn)p_portmap_next_port, (any_fn)p_portmap_size,  (any_fn)p_nat64_6to4,
    (any_fn)p_nat64_4to6,     (any_fn)p_nat64_mbufs,      (any_fn)p_group_by,
    (any_fn)p_set_ip,         (any_fn)p_last_error,       (any_fn)p_strerror,
    (any_fn)p_parse_frames,   (any_fn)p_nat64_frames,
    (any_fn)p_pkt_status_str, (any_fn)p_abi_version,    (any_fn)p_portmap_reset,
    (any_fn)p_reconcile,      (any_fn)p_reconcile_frames, (any_fn)p_ctx_check,
    (any_fn)p_frames_submit,  (any_fn)p_frames_wait,
};

int main(void) {
  /* host-only calls: no device is touched */
  size_t i;
  for (i = 0; i < sizeof entry_points / sizeof entry_points[0]; ++i)
    if (!entry_points[i]) return 4;
  if (p_abi_version() != CGPU_ABI_VERSION) return 1;
  if (p_parse_batch(NULL, NULL, 0, NULL, NULL) != CGPU_EINVAL) return 2;
  if (p_last_error() != CGPU_EINVAL) return 3;
  if (p_reconcile(NULL, NULL, 0, NULL, NULL, NULL, 0, 0, CGPU_LAYER_L4, NULL, NULL) != CGPU_EINVAL)
    return 5;
  if (p_ctx_check(NULL, NULL) != CGPU_EINVAL) return 6;
  if (p_frames_wait(NULL, 1) != CGPU_EINVAL) return 7;
  printf("abi ok: %zu entry points, %s\n", sizeof entry_points / sizeof entry_points[0],
         p_pkt_status_str(CGPU_PKT_NOT_UDP));
  return 0;
}
