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
  uint32_t accept;  // CGPU_F_ACCEPT_* bits and CGPU_F_V6_EXT
  uint32_t *meta;
  uint32_t *csum;
  uint64_t *hash;
  cgpu_hdr_record *fields;
  cgpu_ext_record *ext;  // optional, with CGPU_F_V6_EXT
  // cgpu_reconcile only (the parse kernel's RECON variant): the arena written
  // in place (= arena), the parse's meta words (read), the layer the packets
  // are held at and the optional per-packet status
  uint8_t *wr_arena = nullptr;
  const uint32_t *meta_in = nullptr;
  uint32_t depth = 0;
  uint8_t *rstatus = nullptr;
  // The rows kernels' wave order (parse.hip, "Longest span first"): a wave
  // takes a group of 64 frames; waves sched_from .. sched_from + sched_n - 1
  // take the groups the launch's first sched_n / 256 workgroups order for
  // them, longest span first, through 8-byte granules {tag, group} in
  // `sched`.  nullptr: every wave takes the group of its own index.
  unsigned long long *sched = nullptr;
  uint32_t sched_from = 0, sched_n = 0;
  uint32_t sched_tag = 0;  // this call's granule tag (never 0)
  // A wave that polled its granule sched_spins times without seeing the tag
  // gives up, takes no group and ORs kDevErrSched into *dev_err (the
  // context's device error word, which cgpu_ctx_check and the synchronous
  // entry points report as CGPU_EIO).
  uint32_t sched_spins = 0;
  uint32_t *dev_err = nullptr;
  // Optional (page-locked host word, device mapping): the first ordering
  // workgroup writes whether its groups' spans fall in more than one class,
  // which the host reads when it sizes the stream's next schedule.
  uint32_t *sched_spread = nullptr;
};

// Waves the rows kernels keep resident per CU (8 waves per SIMD), and the
// most waves one launch orders (the granules of one schedule buffer).
constexpr uint32_t kResidentWavesPerCU = 32;
constexpr uint32_t kSchedMax = 16384;
// Granule polls before a wave gives up (each poll sleeps ~0.5 us: seconds,
// against the microseconds the ordering workgroups take; DESIGN.md §3.1
// "Forward progress").
constexpr uint32_t kSchedSpins = 1u << 24;
// Bits of the context's device error word.
constexpr uint32_t kDevErrSched = 1u;

hipError_t launch_parse(const ParseArgs &a, uint32_t flags, hipStream_t s);
// Packet::reconcile_all at a.depth (accept set in a.accept).
hipError_t launch_reconcile(const ParseArgs &a, hipStream_t s);

// ---- nat64 6to4 ------------------------------------------------------------
// Device port map (examples/nat64/main.rs:37-53): open addressing, linear
// probing over 32-byte slots (PortSlot).  A slot's ref word is 0 (empty),
// kPersist (committed; its key words are valid) or (packet index + 1) of the
// packet of the batch in flight that claimed it.
constexpr uint32_t kPersist = 0x80000000u;

// One slot of the device port map, 32 bytes (two dwordx4, one cache line
// half): a lookup is a single line.
//   w[0] ref   0 empty | kPersist committed | (claiming packet + 1)
//   w[1]       claim tag (a second hash of the key; w[0..1] are one 64-bit CAS)
//   w[2..5]    key: v6 source address (wire bytes as LE dwords)
//   w[6]       key: v6-side TCP source port | assigned gateway port << 16
//   w[7]       first packet index of the key in the batch that claimed it
struct PortSlot {
  uint32_t w[8];
};

// ADDR_MAP (main.rs:38: CHashMap<u16, (Ipv6Addr, u16)>) as one dense array
// indexed by gateway port that holds the value itself: the v6 source address
// (16 B, wire bytes as LE dwords) and the v6-side TCP source port with a
// valid bit (4 B), 20 B per port, packed.  A 4to6 lookup is one read of 20
// B (a dwordx4 and a dword at the same place, 1.16 lines on average); 50,000
// mapped ports occupy 7,800 lines (1 MiB), as many as two split arrays, but
// with one request per lookup instead of two, and fewer than with 32-B
// entries (12,500), so more of them stay in the XCD's L2 against the frame
// stream.
constexpr uint32_t kRevValid = 0x10000u;

struct PortMapDev {
  PortSlot *slots;  // [cap]
  uint32_t *rev;      // [65536 * 5] ADDR_MAP: per gateway port, the address (4 dwords)
                      // and the port | kRevValid, 20 B per port, packed
  uint32_t *state;  // [64]: next_port, entries, -, -, then per call parity: deferred[2]
  uint32_t cap_mask;
  uint32_t tag_mask;  // claim-tag bits kept (all; a test build of the map keeps fewer:
                      // CGPU_TEST_NAT64_TAG_MASK, to exercise the tail's collision repair)
  uint32_t seed_hash, seed_tag;  // per-map random seeds of key_hash / key_tag
  // per-map random odd multipliers, one per key word, of key_hash / key_tag
  uint32_t mul_hash[5], mul_tag[5];
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
  uint32_t *pkt_slot;    // scratch [n]: table slot (| kLocalBit: a key new in this batch), or 0xffffffff
  uint8_t *wave_flag;    // scratch [n / 32 + 1]: 1 if the fused kernel's wave of 32 frames wrote
                         // their pkt_slot entries (it had a deferred frame), else 0: the
                         // entries are stale and read as 0xffffffff (the steady state
                         // writes no pkt_slot at all)
  uint32_t *chunks;      // scratch [10 nblocks + n (rounded up to 32) + 33 * 32]: the tail's
                         // chunk counts, bases, first-packet masks, its list of tag
                         // collisions, then its control lines (zero between calls)
  uint32_t *ctl;         // scratch: the tail's control lines (at a place fixed for the
                         // scratch's capacity, not the call's n: zeroed once)
  u32x4 *stash_key;      // scratch [n]: a tag-joined packet's key (v6 source address) ...
  uint16_t *stash_port;  // scratch [n]: ... and its TCP source port, verified by the tail
  uint32_t *stash_c0;    // scratch [n]: a deferred frame's TCP checksum (port 0) | VLAN depth << 16
  uint32_t par;          // call parity: selects the deferred flag state[4 + par]
  uint32_t room;         // data room of Mbuf::extend's tailroom model (mbuf.rs:225-233):
                         // 2048 for device batches; 65535 on the mbuf path, whose
                         // scatter checks each mbuf's real tailroom instead
  PortMapDev pm;
};

hipError_t launch_nat64_6to4(const Nat64Args &a, hipStream_t s, hipEvent_t done);
hipError_t launch_nat64_4to6(const Nat64Args &a, hipStream_t s, hipEvent_t done);
hipError_t launch_portmap_init(const PortMapDev &pm, uint32_t first_port, hipStream_t s);
uint32_t nat64_num_blocks(uint32_t n);
// bytes of Nat64Args::chunks for up to n packets, and the offset of the
// control lines in it (Nat64Args::ctl, zeroed once when allocated)
size_t nat64_chunk_bytes(uint32_t n);
size_t nat64_ctl_offset(uint32_t n);

// ---- zero-copy rte_mbuf ingress (ingress.hip) ------------------------------
struct HostRegion {
  uint64_t host_base, dev_base, bytes;
};
constexpr uint32_t kMaxRegions = 16;
struct GatherArgs {
  const uint64_t *mbufs;  // [n] host rte_mbuf addresses (device copy of the array)
  const uint64_t *frames; // or, when not null: [n] host frame addresses (data_address),
  const uint16_t *flen;   //   [n] their lengths (data_len); no mbuf header is read
  const uint16_t *ftail;  //   [n] their tailrooms (Mbuf::tailroom), for the egress records
  uint32_t n;
  uint32_t nreg;
  HostRegion reg[kMaxRegions];
  uint8_t *arena;         // device arena, 64-B slots; nullptr: validate only (no copy)
  uint64_t arena_cap;     // bytes of `arena`: no slot is written past it
  uint32_t *off;          // [n]
  uint16_t *len;          // [n]
  unsigned long long *cursor;  // slot allocation cursor (zero before the launch); after
                               // it, the bytes the chunk needs (> arena_cap: redo bigger)
  uint32_t *bad;          // mbufs / frames outside every registered region, or frames
                          // past their buffer (data_off + data_len > buf_len)
  uint32_t slot_extra;    // bytes of room past each frame in its slot (nat64 4to6: 20)
  // optional (nullptr: not written), for the egress scatter:
  uint64_t *mb_dev;       // [n] device address of the rte_mbuf header (0: bad)
  uint64_t *fr_dev;       // [n] device address of the frame (buf_addr + data_off)
  uint32_t *pkt_len;      // [n] rte_mbuf pkt_len (@36)
  uint32_t *tailroom;     // [n] buf_len - data_off - data_len (Mbuf::tailroom, mbuf.rs:207-213)
};
hipError_t launch_mbuf_gather(const GatherArgs &g, hipStream_t s);

// Egress: the rewritten ACT frames back into their own mbufs.
struct ScatterArgs {
  const uint8_t *out_arena;
  const uint32_t *out_off;
  const uint16_t *out_len;
  uint8_t *disposition;   // ACT frames are written; 4to6 without tailroom -> ABORT
  uint8_t *status;
  const uint64_t *mb_dev;
  const uint64_t *fr_dev;
  const uint32_t *pkt_len;
  const uint32_t *tailroom;
  const uint16_t *in_len;
  uint32_t n;
  int32_t delta;          // data_len change: -20 (6to4) or +20 (4to6)
};
hipError_t launch_mbuf_scatter(const ScatterArgs &a, hipStream_t s);

// ---- group_by --------------------------------------------------------------
struct GroupByArgs {
  const void *key;     // u8 arm keys or u32 meta words (kind)
  uint32_t kind;       // CGPU_KEY_*
  uint32_t n;
  uint32_t groups;     // arms, the last one is the catch-all (1..64)
  uint32_t tiles;      // group_by_tiles(n)
  uint32_t *counts;    // scratch [groups * tiles]
  uint32_t *idx;       // [n] packet indices grouped by arm
  uint32_t *group_off; // [groups + 1]
};

uint32_t group_by_tiles(uint32_t n);
hipError_t launch_group_by(const GroupByArgs &a, hipStream_t s);

// ---- set_src_ip / set_dst_ip (setip.hip) -----------------------------------
struct SetIpArgs {
  uint8_t *arena;
  uint32_t arena_len;
  const uint32_t *off;
  const uint16_t *len;
  const uint32_t *meta;
  uint32_t n;
  const cgpu_ip_addr *src;  // optional
  uint32_t src_stride;
  const cgpu_ip_addr *dst;  // optional
  uint32_t dst_stride;
  uint8_t *status;          // optional
};
hipError_t launch_set_ip(const SetIpArgs &a, hipStream_t s);

}  // namespace cgpu
