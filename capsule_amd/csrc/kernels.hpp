// kernels.hpp — host-visible launch interface of the HIP kernels (internal,
// not part of the C ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "capsule_gpu.h"

namespace cgpu {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct ParseArgs {
  const uint8_t *arena;
  uint32_t arena_len;
  const uint32_t *off;
  const uint16_t *len;
  uint32_t n;
  uint32_t accept;  // CGPU_F_ACCEPT_* bits
  uint32_t *meta;
  uint32_t *csum;
  uint64_t *hash;
  cgpu_hdr_record *fields;
};

hipError_t launch_parse(const ParseArgs &a, uint32_t flags, hipStream_t s);

// ---- nat64 6to4 ------------------------------------------------------------
// Device port map (examples/nat64/main.rs:37-53): open addressing, linear
// probing.  slot_ref: 0 empty, kPersist = committed entry whose key lives in
// key_src/key_port, else (packet index + 1) of a representative packet of
// the batch in flight.
constexpr uint32_t kPersist = 0x80000000u;

struct PortMapDev {
  uint32_t *slot_ref;   // [cap]
  uint32_t *slot_min;   // [cap] min packet index of the batch (0xffffffff idle)
  uint32_t *key_src;    // [cap * 4] v6 source address, wire bytes as LE dwords
  uint32_t *key_port;   // [cap] v6-side TCP source port
  uint32_t *slot_port;  // [cap] assigned gateway port
  uint32_t *state;      // [4]: next_port, entries, batch_base, batch_new
  uint32_t cap_mask;
};

struct Nat64Args {
  const uint8_t *arena;
  uint32_t arena_len;
  const uint32_t *off;
  const uint16_t *len;
  uint32_t n;
  uint8_t *out_arena;
  uint32_t out_arena_len;
  const uint32_t *out_off;
  uint16_t *out_len;
  uint8_t *disposition;
  uint8_t *status;
  uint32_t *pkt_slot;    // scratch [n]: table slot (or 0xffffffff)
  uint32_t *block_sums;  // scratch [nblocks + 1]
  u32x4 *rec_h;          // scratch [n]: new IPv4 header dwords 0..3 (K1 -> K5)
  uint2 *rec_b;          // scratch [n]: header dword 4, eth_len | k << 8 | new_len << 16
  PortMapDev pm;
};

hipError_t launch_nat64_6to4(const Nat64Args &a, hipStream_t s);
hipError_t launch_portmap_init(const PortMapDev &pm, uint32_t first_port, hipStream_t s);
uint32_t nat64_num_blocks(uint32_t n);

}  // namespace cgpu
