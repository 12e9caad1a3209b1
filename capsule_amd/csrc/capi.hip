// capi.hip — the extern "C" boundary declared in include/capsule_gpu.h.
//
// Error handling follows the reference's FFI conventions
// (core/src/ffi.rs:86-141, core/src/dpdk/mod.rs:62-70): every entry point
// returns 0 or a negative errno-style code and records it in a thread-local
// slot readable through cgpu_last_error(), the `_rte_errno()` analogue of
// ffi/src/shim.c:24-26.  Contexts are independent (one per core thread /
// RX queue) and no global lock is taken on the launch path.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <dlfcn.h>
#include <unistd.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>
#include <random>
#include <vector>

#include "capsule_gpu.h"
#include "kernels.hpp"

// How a nat64 call orders itself behind the map's previous call: it waits
// on the previous call's completion event unless both calls ran on the same
// stream, told by stream id (hipStreamGetId: never reused, unlike a handle a
// destroyed stream may hand to a new one).  A wait on a still-pending event
// of the same stream costs ~1.4 us per call on the stream (measured,
// DESIGN.md §3.2).

namespace {

thread_local int g_last_error = 0;

// A stream's id (0 if the runtime cannot tell).  hipStreamGetId is looked
// up at run time: the HIP runtime in the process may predate it (ROCm 7.0's
// has no hip_7.1 symbols), and then every call waits.
unsigned long long stream_id(void *stream) {
  typedef hipError_t (*get_id_fn)(hipStream_t, unsigned long long *);
  static const get_id_fn get_id = (get_id_fn)dlsym(RTLD_DEFAULT, "hipStreamGetId");
  unsigned long long id = 0;
  if (!get_id || get_id((hipStream_t)stream, &id) != hipSuccess) return 0;
  return id;
}

int fail(int code) {
  g_last_error = code;
  return code;
}

int ok() {
  g_last_error = 0;
  return 0;
}

int hip_fail(hipError_t e) {
  (void)e;
  return fail(CGPU_EIO);
}

// Makes a context's device current for one entry point and gives the
// calling thread its own current device back on return: a core thread may
// drive contexts of several GPUs, and a NULL stream means "the current
// device's", so every call that allocates, copies or launches runs inside
// one of these.
class DeviceGuard {
 public:
  explicit DeviceGuard(int dev) : dev_(dev) {
    if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
    ok_ = prev_ == dev || hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev_ >= 0 && prev_ != dev_) (void)hipSetDevice(prev_);
  }
  bool ok() const { return ok_; }

 private:
  int dev_, prev_ = -1;
  bool ok_ = false;
};

}  // namespace

struct cgpu_ctx {
  int device;
  hipStream_t stream = nullptr;  // used by the synchronous host entry points
  // pinned + device staging for cgpu_parse_host
  uint8_t *h_arena = nullptr, *d_arena = nullptr;
  size_t arena_cap = 0;
  uint8_t *h_desc = nullptr, *d_desc = nullptr;  // off[n] | len[n] | outputs
  size_t desc_cap = 0;
  // zero-copy ingress: the device arena the gather lays bursts out in, and
  // (nat64 over mbufs) the rewritten frames; both grow on demand
  uint8_t *d_zc = nullptr, *d_out = nullptr;
  size_t zc_cap = 0, out_cap = 0;
  uint32_t *gb_counts = nullptr;  // cgpu_group_by scratch
  size_t gb_cap = 0;              // entries
  // host regions registered for zero-copy ingress
  cgpu::HostRegion reg[cgpu::kMaxRegions];
  bool reg_owned[cgpu::kMaxRegions];  // registered here (else: the caller's pinned allocation)
  uint32_t nreg = 0;
  // the device error word (kernels.hpp kDevErrSched), and whether a call
  // since it was last read took the wave schedule
  uint32_t *dev_err = nullptr;
  bool err_pending = false;
  // cgpu_parse_frames' direct path: page-locked host memory the kernel
  // reads its descriptors from and writes its results to (no copies).
  // Slots 0 and 1 carry the asynchronous bursts (cgpu_parse_frames_submit,
  // ticket & 1), slot 2 the synchronous calls.
  struct IoSlot {
    uint8_t *h = nullptr, *d = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;
    bool pending = false;  // submitted, not yet waited for
    int rc = 0;            // a burst the gather path ran at submit: its result
    uint32_t ticket = 0, n = 0;
    size_t o_meta = 0, o_csum = 0, o_hash = 0, o_fields = 0;
    uint32_t *meta = nullptr, *csum = nullptr;
    uint64_t *hash = nullptr;
    cgpu_hdr_record *fields = nullptr;
  } io[3];
  uint32_t next_ticket = 1;
  uint32_t sched_spins = cgpu::kSchedSpins;
  // The rows kernels' wave schedules (kernels.hpp ParseArgs::sched): waves
  // resident on this device, and one granule buffer per stream the context
  // has launched on, with the tag of its latest call.  Calls on one stream
  // run in order, so no buffer is ever read by two calls at once.  Streams
  // are told apart by id where the HIP runtime can tell (hipStreamGetId, ids
  // are never reused), else by handle.
  uint32_t resident_waves = 0;
  struct Sched {
    unsigned long long key;
    unsigned long long *buf;
    uint32_t tag;
    // whether the stream's latest ordered batch had spans of more than one
    // class (written by its first ordering workgroup; 1 until then)
    volatile uint32_t *spread_h;
    uint32_t *spread_d;
  };
  std::vector<Sched> sched;
};

namespace {

// Resident waves of the rows kernels: the CU count x 32 (8 waves per SIMD).
uint32_t resident_waves(int device) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
    return 0;
  return (uint32_t)cus * cgpu::kResidentWavesPerCU;
}

#ifdef CGPU_TEST_HOOKS
// Test build only (libcapsule_gpu_test.so; the product library reads no
// environment): a decimal value of `name` within [lo, hi], else `dflt`.
uint32_t test_hook(const char *name, uint32_t lo, uint32_t hi, uint32_t dflt) {
  const char *e = getenv(name);
  if (!e) return dflt;
  char *end = nullptr;
  const unsigned long v = strtoul(e, &end, 0);
  if (end != e && *end == '\0' && v >= lo && v <= hi) {
    fprintf(stderr, "capsule_gpu: test hook %s=%lu active\n", name, v);
    return (uint32_t)v;
  }
  fprintf(stderr, "capsule_gpu: ignoring malformed %s\n", name);
  return dflt;
}
#endif

// The schedule buffer of `key` (a stream), allocated on first use and
// zeroed on `stream`, ordered before the launch that first reads it;
// nullptr if it cannot be had (the call then runs unordered).
cgpu_ctx::Sched *sched_buffer(cgpu_ctx *c, unsigned long long key, hipStream_t stream) {
  for (auto &x : c->sched)
    if (x.key == key) return &x;
  unsigned long long *buf = nullptr;
  const size_t bytes = sizeof(unsigned long long) * cgpu::kSchedMax;
  if (hipMalloc((void **)&buf, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (hipMemsetAsync(buf, 0, bytes, stream) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipFree(buf);
    return nullptr;
  }
  // the spread word: page-locked and mapped (nullptr if it cannot be had:
  // every batch is then taken to vary)
  void *h = nullptr;
  uint32_t *d = nullptr;
  if (hipHostMalloc(&h, 4, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
    *(volatile uint32_t *)h = 1u;
    if (hipHostGetDevicePointer((void **)&d, h, 0) != hipSuccess) {
      (void)hipGetLastError();
      (void)hipHostFree(h);
      h = nullptr;
      d = nullptr;
    }
  } else {
    (void)hipGetLastError();
    h = nullptr;
  }
  c->sched.push_back(cgpu_ctx::Sched{key, buf, 0u, (volatile uint32_t *)h, d});
  return &c->sched.back();
}

unsigned long long sched_key(void *stream) {
  const unsigned long long sid = stream_id(stream);
  return sid ? sid : (unsigned long long)(uintptr_t)stream | (1ull << 63);
}

// Gives a call of a.n frames on `stream` its wave schedule when the launch
// is more than one round of waves: the last min(groups - resident / 2,
// kSchedMax) groups of 64 frames, rounded down to whole lists of 256, are
// ordered longest span first (parse.hip).  The kernel ignores it unless it
// runs the rows variant.  The schedule is an optimisation, never needed for
// a result: a stream that is being captured into a graph (replays of one
// graph would share a buffer and a tag) or a buffer that cannot be
// allocated leaves the call unordered.
void set_schedule(cgpu_ctx *c, cgpu::ParseArgs &a, void *stream) {
  a.sched = nullptr;
  a.sched_spread = nullptr;
  a.dev_err = c->dev_err;
  a.sched_spins = c->sched_spins;
  const uint32_t groups = (a.n + 63u) / 64u;
  if (c->resident_waves == 0 || groups <= c->resident_waves) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing((hipStream_t)stream, &cs) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  if (cs != hipStreamCaptureStatusNone) return;
  cgpu_ctx::Sched *b = sched_buffer(c, sched_key(stream), (hipStream_t)stream);
  if (!b) return;
  // Every group after the first half round is ordered (whole lists of 256
  // groups, one ordering workgroup each): the second half of the first
  // round's waves then take the longest groups too (IMIX with checksums
  // 77.6-78.1 -> 75.8-76.2 us against ordering from the second round on,
  // DESIGN.md section 3.1).  Those waves wait for the order, which buys
  // nothing when every group has one span (256-B frames: +1-2 us): when the
  // stream's latest ordered batch was such, only the groups after the first
  // round are ordered.  (A guess from the previous batch, read without a
  // synchronisation; results never depend on it.)
  const bool spread = b->spread_h == nullptr || *b->spread_h != 0u;
  const uint32_t over = groups - (spread ? c->resident_waves / 2u : c->resident_waves);
  const uint32_t n_sched = (over < cgpu::kSchedMax ? over : cgpu::kSchedMax) / 256u * 256u;
  if (n_sched == 0) return;
  if (++b->tag == 0u) b->tag = 1u;  // tags are never 0: a zeroed granule matches no call
  a.sched_spread = b->spread_d;
  a.sched = b->buf;
  a.sched_n = n_sched;
  a.sched_from = groups - n_sched;
  a.sched_tag = b->tag;
  c->err_pending = true;
}

// Reads and clears the context's device error word on its stream (after
// the caller has synchronised the streams whose calls it covers): CGPU_EIO
// if a wave gave up on the schedule.
int take_dev_err(cgpu_ctx *c) {
  uint32_t w = 0;
  if (hipMemcpyAsync(&w, c->dev_err, 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return CGPU_EIO;
  if (w == 0) return 0;
  if (hipMemsetAsync(c->dev_err, 0, 4, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return CGPU_EIO;
  return CGPU_EIO;
}

// The end of a synchronous entry point that ran on the context's stream.
int sync_done(cgpu_ctx *c) {
  if (!c->err_pending) return 0;
  c->err_pending = false;
  return take_dev_err(c);
}

}  // namespace

struct cgpu_portmap {
  cgpu_ctx *ctx;
  cgpu::PortMapDev dev;
  void *mem;
  // per-call scratch
  uint32_t *pkt_slot = nullptr;
  uint32_t *chunks = nullptr;
  cgpu::u32x4 *stash_key = nullptr;
  uint16_t *stash_port = nullptr;
  uint32_t *stash_c0 = nullptr;
  uint8_t *wave_flag = nullptr;
  uint32_t scratch_n = 0;
  uint32_t calls = 0;  // 6to4 calls: parity of the deferred-list counter
  // recorded on the stream of every call that uses the map: calls on one
  // map are stream-ordered (the map is stateful), so waiting for it waits
  // for the map's work without stalling other contexts' streams on the same
  // GPU, and it stays valid after the caller destroys that stream
  hipEvent_t done = nullptr;
  // the stream of the latest call (compared, never used: it may be gone);
  // a call on another stream first waits for `done`
  unsigned long long last_sid = 0;  // stream id of the map's previous call (0: none known)
  uint32_t room = 2048u;  // Nat64Args::room of the next call (65535 inside cgpu_nat64_mbufs)
};

extern "C" {

int cgpu_abi_version(void) { return CGPU_ABI_VERSION; }

int cgpu_last_error(void) { return g_last_error; }

const char *cgpu_strerror(int code) {
  switch (code) {
    case CGPU_OK: return "success";
    case CGPU_EINVAL: return "invalid argument";
    case CGPU_ENOMEM: return "out of memory";
    case CGPU_ENODEV: return "no such device";
    case CGPU_EIO: return "HIP runtime error";
    case CGPU_ENOSPC: return "port table full";
    case CGPU_EBUSY: return "two bursts already in flight";
    default: return "unknown error";
  }
}

const char *cgpu_pkt_status_str(int s) {
  switch (s) {
    case CGPU_PKT_OK: return "ok";
    case CGPU_PKT_ETH_BAD_OFFSET: return "Ethernet: bad offset";
    case CGPU_PKT_ETH_OUT_OF_BUFFER: return "Ethernet: out of buffer";
    case CGPU_PKT_NOT_IPV4: return "not an IPv4 packet.";
    case CGPU_PKT_NOT_IPV6: return "not an IPv6 packet.";
    case CGPU_PKT_NOT_IP: return "not an IP packet.";
    case CGPU_PKT_L3_BAD_OFFSET: return "IP: bad offset";
    case CGPU_PKT_L3_OUT_OF_BUFFER: return "IP: out of buffer";
    case CGPU_PKT_NOT_UDP: return "not a UDP packet.";
    case CGPU_PKT_NOT_TCP: return "not a TCP packet.";
    case CGPU_PKT_NOT_L4: return "not a packet of an accepted L4 type.";
    case CGPU_PKT_NOT_ICMPV4: return "not an ICMPv4 packet.";
    case CGPU_PKT_NOT_ICMPV6: return "not an ICMPv6 packet.";
    case CGPU_PKT_EXT_BAD_OFFSET: return "IPv6 extension: bad offset";
    case CGPU_PKT_EXT_OUT_OF_BUFFER: return "IPv6 extension: out of buffer";
    case CGPU_PKT_SRH_INCONSISTENT: return "Packet has inconsistent segment list length.";
    case CGPU_PKT_L4_BAD_OFFSET: return "L4: bad offset";
    case CGPU_PKT_L4_OUT_OF_BUFFER: return "L4: out of buffer";
    case CGPU_PKT_NOT_RESIZED: return "buffer not resized";
    case CGPU_PKT_TABLE_FULL: return "port table full";
    default: return "unknown status";
  }
}

int cgpu_ctx_create(int hip_device, cgpu_ctx **out) {
  if (!out) return fail(CGPU_EINVAL);
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || hip_device < 0 || hip_device >= count)
    return fail(CGPU_ENODEV);
  DeviceGuard dg(hip_device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  cgpu_ctx *c = new (std::nothrow) cgpu_ctx();
  if (!c) return fail(CGPU_ENOMEM);
  c->device = hip_device;
  c->resident_waves = resident_waves(hip_device);
#ifdef CGPU_TEST_HOOKS
  // CGPU_TEST_SCHED_WAVES: resident waves as the schedule counts them (small
  // batches then run several rounds and take it); CGPU_TEST_SCHED_SPINS:
  // granule polls before a wave gives up (0: every ordered wave gives up)
  c->resident_waves = test_hook("CGPU_TEST_SCHED_WAVES", 64u, 1u << 20, c->resident_waves);
  c->sched_spins = test_hook("CGPU_TEST_SCHED_SPINS", 0u, cgpu::kSchedSpins, c->sched_spins);
#endif
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return fail(CGPU_EIO);
  }
  // the device error word, and the schedule buffer of the context's own
  // stream (the synchronous entry points' calls)
  if (hipMalloc((void **)&c->dev_err, 4) != hipSuccess || hipMemsetAsync(c->dev_err, 0, 4, c->stream) != hipSuccess ||
      (c->resident_waves && !sched_buffer(c, sched_key(c->stream), c->stream)) ||
      hipStreamSynchronize(c->stream) != hipSuccess) {
    (void)hipGetLastError();
    cgpu_ctx_destroy(c);
    return fail(CGPU_ENOMEM);
  }
  *out = c;
  return ok();
}

int cgpu_ctx_check(cgpu_ctx *c, void *stream) {
  if (!c) return fail(CGPU_EINVAL);
  DeviceGuard dg(c->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return fail(CGPU_EIO);
  c->err_pending = false;
  if (int e = take_dev_err(c)) return fail(e);
  return ok();
}

void cgpu_ctx_destroy(cgpu_ctx *c) {
  if (!c) return;
  DeviceGuard dg(c->device);
  // nothing is freed or unpinned under a call still running on the
  // context's stream (the synchronous entry points' stream)
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->dev_err) (void)hipFree(c->dev_err);
  for (auto &x : c->io) {
    if (x.h) (void)hipHostFree(x.h);
    if (x.done) (void)hipEventDestroy(x.done);
  }
  if (c->h_arena) (void)hipHostFree(c->h_arena);
  if (c->d_arena) (void)hipFree(c->d_arena);
  if (c->h_desc) (void)hipHostFree(c->h_desc);
  if (c->d_desc) (void)hipFree(c->d_desc);
  if (c->gb_counts) (void)hipFree(c->gb_counts);
  for (auto &x : c->sched) {
    (void)hipFree(x.buf);
    if (x.spread_h) (void)hipHostFree((void *)x.spread_h);
  }
  if (c->d_out) (void)hipFree(c->d_out);
  if (c->d_zc) (void)hipFree(c->d_zc);
  for (uint32_t r = 0; r < c->nreg; ++r)
    if (c->reg_owned[r]) (void)hipHostUnregister((void *)(uintptr_t)c->reg[r].host_base);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

static int check_batch(const cgpu_batch *b) {
  if (!b) return CGPU_EINVAL;
  if (b->n == 0) return 0;
  if (!b->arena || !b->off || !b->len) return CGPU_EINVAL;
  if (b->arena_len > 0xffff0000ull) return CGPU_EINVAL;  // offsets above are "no read"
  if (b->n > CGPU_MAX_BATCH) return CGPU_EINVAL;          // 32-bit descriptor byte offsets
  return 0;
}

int cgpu_parse_batch(cgpu_ctx *ctx, const cgpu_batch *batch, uint32_t flags,
                     const cgpu_parse_out *out, void *stream) {
  if (!ctx || !out) return fail(CGPU_EINVAL);
  if (int e = check_batch(batch)) return fail(e);
  if (batch->n == 0) return ok();
  if (!out->meta) return fail(CGPU_EINVAL);
  if ((flags & CGPU_F_FLOW_HASH) && !out->flow_hash) return fail(CGPU_EINVAL);
  DeviceGuard dg(ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  // no L3 (L4) type named: every IP version (UDP and TCP) accepted
  if ((flags & (CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_V6)) == 0) flags |= CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_V6;
  if ((flags & (CGPU_F_ACCEPT_UDP | CGPU_F_ACCEPT_TCP | CGPU_F_ACCEPT_ICMP)) == 0)
    flags |= CGPU_F_ACCEPT_UDP | CGPU_F_ACCEPT_TCP;
  cgpu::ParseArgs a;
  a.arena = batch->arena;
  a.arena_len = (uint32_t)batch->arena_len;
  a.off = batch->off;
  a.len = batch->len;
  a.n = batch->n;
  a.accept = flags & (CGPU_F_ACCEPT_ALL | CGPU_F_ACCEPT_ICMP | CGPU_F_V6_EXT);
  a.meta = out->meta;
  a.csum = out->csum;
  a.hash = out->flow_hash;
  a.fields = out->fields;
  a.ext = out->ext;
  set_schedule(ctx, a, stream);
  hipError_t e = cgpu::launch_parse(a, flags, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e);
  return ok();
}

static int grow(uint8_t **h, uint8_t **d, size_t *cap, size_t need) {
  if (need <= *cap) return 0;
  size_t nc = need + need / 2 + 4096;
  if (*h) (void)hipHostFree(*h);
  if (*d) (void)hipFree(*d);
  *h = nullptr;
  *d = nullptr;
  *cap = 0;
  if (hipHostMalloc((void **)h, nc, hipHostMallocDefault) != hipSuccess) return CGPU_ENOMEM;
  if (hipMalloc((void **)d, nc) != hipSuccess) {
    (void)hipHostFree(*h);
    *h = nullptr;
    return CGPU_ENOMEM;
  }
  *cap = nc;
  return 0;
}

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }


}  // extern "C"

// Output layout of the per-context descriptor staging for n packets.
struct HostLayout {
  size_t off, len, meta, csum, hash, fields, end;
  HostLayout(uint32_t n, bool with_fields, size_t base = 0) {
    off = base;
    len = off + align_up(4ull * n, 256);
    meta = len + align_up(2ull * n, 256);
    csum = meta + align_up(4ull * n, 256);
    hash = csum + align_up(4ull * n, 256);
    fields = hash + align_up(8ull * n, 256);
    end = fields + (with_fields ? align_up(sizeof(cgpu_hdr_record) * (size_t)n, 256) : 0);
  }
};

// Parse the device batch described by `lay` inside ctx->d_desc and copy the
// outputs to the caller's host arrays at packet index `at`; asynchronous.
static int parse_and_return(cgpu_ctx *ctx, const uint8_t *arena, size_t arena_len, uint32_t n,
                            const HostLayout &lay, uint32_t flags, uint32_t *meta, uint32_t *csum,
                            uint64_t *flow_hash, cgpu_hdr_record *fields, uint32_t at) {
  hipStream_t s = ctx->stream;
  cgpu_batch b;
  b.arena = arena;
  b.arena_len = arena_len;
  b.off = (const uint32_t *)(ctx->d_desc + lay.off);
  b.len = (const uint16_t *)(ctx->d_desc + lay.len);
  b.n = n;
  cgpu_parse_out o;
  o.meta = (uint32_t *)(ctx->d_desc + lay.meta);
  o.csum = (uint32_t *)(ctx->d_desc + lay.csum);
  o.flow_hash = (uint64_t *)(ctx->d_desc + lay.hash);
  o.fields = fields ? (cgpu_hdr_record *)(ctx->d_desc + lay.fields) : nullptr;
  o.ext = nullptr;
  if (!csum) flags &= ~(CGPU_F_CSUM_IP | CGPU_F_CSUM_L4);
  if (!flow_hash) flags &= ~CGPU_F_FLOW_HASH;
  if (int e = cgpu_parse_batch(ctx, &b, flags, &o, s)) return e;
  if (hipMemcpyAsync(meta + at, o.meta, 4ull * n, hipMemcpyDeviceToHost, s) != hipSuccess)
    return fail(CGPU_EIO);
  if (csum && hipMemcpyAsync(csum + at, o.csum, 4ull * n, hipMemcpyDeviceToHost, s) != hipSuccess)
    return fail(CGPU_EIO);
  if (flow_hash &&
      hipMemcpyAsync(flow_hash + at, o.flow_hash, 8ull * n, hipMemcpyDeviceToHost, s) != hipSuccess)
    return fail(CGPU_EIO);
  if (fields && hipMemcpyAsync(fields + at, o.fields, sizeof(cgpu_hdr_record) * (size_t)n,
                               hipMemcpyDeviceToHost, s) != hipSuccess)
    return fail(CGPU_EIO);
  return 0;
}

// The staged host path: `get(i, p, len)` names packet i's bytes (false: bad
// pointer); the calling core gathers them into pinned staging at 64-byte
// slots (the mbuf data room layout), one DMA copies the burst.  Synchronous.
template <class Get>
static int parse_staged(cgpu_ctx *ctx, uint32_t n, Get get, uint32_t flags, uint32_t *meta,
                        uint32_t *csum, uint64_t *flow_hash, cgpu_hdr_record *fields) {
  DeviceGuard dg(ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  size_t total = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t *p;
    uint16_t l;
    if (!get(i, p, l)) return fail(CGPU_EINVAL);
    total += align_up(l, 64);
  }
  if (total >= (1ull << 32)) return fail(CGPU_EINVAL);
  if (int e = grow(&ctx->h_arena, &ctx->d_arena, &ctx->arena_cap, total + 64)) return fail(e);
  const HostLayout lay(n, fields != nullptr);
  if (int e = grow(&ctx->h_desc, &ctx->d_desc, &ctx->desc_cap, lay.end)) return fail(e);
  uint32_t *hoff = (uint32_t *)(ctx->h_desc + lay.off);
  uint16_t *hlen = (uint16_t *)(ctx->h_desc + lay.len);
  size_t pos = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t *p;
    uint16_t l;
    get(i, p, l);
    hoff[i] = (uint32_t)pos;
    hlen[i] = l;
    if (l) memcpy(ctx->h_arena + pos, p, l);
    pos += align_up(l, 64);
  }
  hipStream_t s = ctx->stream;
  if (hipMemcpyAsync(ctx->d_arena, ctx->h_arena, pos ? pos : 1, hipMemcpyHostToDevice, s) !=
      hipSuccess)
    return fail(CGPU_EIO);
  if (hipMemcpyAsync(ctx->d_desc, ctx->h_desc, lay.meta, hipMemcpyHostToDevice, s) != hipSuccess)
    return fail(CGPU_EIO);
  if (int e = parse_and_return(ctx, ctx->d_arena, pos ? pos : 1, n, lay, flags, meta, csum,
                               flow_hash, fields, 0))
    return e;
  if (hipStreamSynchronize(s) != hipSuccess) return fail(CGPU_EIO);
  if (int e = sync_done(ctx)) return fail(e);
  return ok();
}

// rte_mbuf field reads (DPDK 19.11 layout, ffi/src/bindings_rustdoc.rs:6869-6898)
static inline void mbuf_fields(const void *m, const uint8_t *&data, uint16_t &len) {
  const uint8_t *b = (const uint8_t *)m;
  uint8_t *buf_addr;
  uint16_t data_off;
  memcpy(&buf_addr, b + CGPU_MBUF_BUF_ADDR_OFF, sizeof buf_addr);
  memcpy(&data_off, b + CGPU_MBUF_DATA_OFF_OFF, sizeof data_off);
  memcpy(&len, b + CGPU_MBUF_DATA_LEN_OFF, sizeof len);
  data = buf_addr + data_off;
}

static int grow_dev(uint8_t **d, size_t *cap, size_t need) {
  if (need <= *cap) return 0;
  if (*d) (void)hipFree(*d);
  *d = nullptr;
  *cap = 0;
  if (hipMalloc((void **)d, need) != hipSuccess) return CGPU_ENOMEM;
  *cap = need;
  return 0;
}

namespace {

// Zero-copy gathers work in chunks of at most 2^20 mbufs whose arena stays
// below 4 GiB (u32 offsets); a chunk of jumbo frames that would not fit is
// cut shorter.
constexpr uint32_t kZcChunk = 1u << 20;
constexpr size_t kZcSlot = 2176;                  // an mbuf buffer: 128 headroom + 2048 room
constexpr uint64_t kZcArenaMax = 0xffff0000ull;   // cgpu_batch::arena_len limit

struct ZcCounters {  // device counters of one gather (16 bytes)
  unsigned long long cursor;
  uint32_t bad, pad;
};

// One zero-copy gather of mbufs[at, at + m) (the pointer array already at
// `ptrs` on the device).  arena = nullptr: validate the pointers only.
// frames != nullptr: `ptrs` is unused and the burst is (frames, flen) pairs,
// with ftail the frames' tailrooms for the egress records.
hipError_t gather_chunk(cgpu_ctx *ctx, const uint64_t *ptrs, uint32_t m, uint8_t *arena,
                        size_t arena_cap, uint32_t *off, uint16_t *len, ZcCounters *cnt,
                        uint32_t slot_extra, uint8_t *egress_base, uint32_t stride,
                        hipStream_t s, const uint64_t *frames = nullptr,
                        const uint16_t *flen = nullptr, const uint16_t *ftail = nullptr) {
  if (hipMemsetAsync(cnt, 0, sizeof(ZcCounters), s) != hipSuccess) return hipErrorUnknown;
  cgpu::GatherArgs g;
  g.mbufs = frames ? nullptr : ptrs;
  g.frames = frames;
  g.flen = flen;
  g.ftail = ftail;
  g.n = m;
  g.nreg = ctx->nreg;
  for (uint32_t r = 0; r < cgpu::kMaxRegions; ++r) g.reg[r] = ctx->reg[r];
  g.arena = arena;
  g.arena_cap = arena_cap;
  g.off = off;
  g.len = len;
  g.cursor = &cnt->cursor;
  g.bad = &cnt->bad;
  g.slot_extra = slot_extra;
  g.mb_dev = g.fr_dev = nullptr;
  g.pkt_len = g.tailroom = nullptr;
  if (egress_base) {  // per-mbuf egress records: mb | fr | pkt_len | tailroom, `stride` each
    g.mb_dev = (uint64_t *)egress_base;
    g.fr_dev = g.mb_dev + stride;
    g.pkt_len = (uint32_t *)(g.fr_dev + stride);
    g.tailroom = g.pkt_len + stride;
  }
  return cgpu::launch_mbuf_gather(g, s);
}

// The same gather from (frame address, length) pairs (device copies at
// `frames` / `flen`).
hipError_t gather_frames_chunk(cgpu_ctx *ctx, const uint64_t *frames, const uint16_t *flen,
                               uint32_t m, uint8_t *arena, size_t arena_cap, uint32_t *off,
                               uint16_t *len, ZcCounters *cnt, hipStream_t s) {
  if (hipMemsetAsync(cnt, 0, sizeof(ZcCounters), s) != hipSuccess) return hipErrorUnknown;
  cgpu::GatherArgs g;
  g.mbufs = nullptr;
  g.frames = frames;
  g.flen = flen;
  g.ftail = nullptr;
  g.n = m;
  g.nreg = ctx->nreg;
  for (uint32_t r = 0; r < cgpu::kMaxRegions; ++r) g.reg[r] = ctx->reg[r];
  g.arena = arena;
  g.arena_cap = arena_cap;
  g.off = off;
  g.len = len;
  g.cursor = &cnt->cursor;
  g.bad = &cnt->bad;
  g.slot_extra = 0;
  g.mb_dev = g.fr_dev = nullptr;
  g.pkt_len = g.tailroom = nullptr;
  return cgpu::launch_mbuf_gather(g, s);
}

}  // namespace

// Zero-copy: the device gathers the burst from registered host memory.  The
// parse runs right behind the gather; if the chunk's frames did not fit the
// arena (a jumbo mempool), the arena grows and the chunk is done again.
static int parse_zero_copy(cgpu_ctx *ctx, void *const *mbufs, uint32_t n, uint32_t flags,
                           uint32_t *meta, uint32_t *csum, uint64_t *flow_hash,
                           cgpu_hdr_record *fields) {
  if (ctx->nreg == 0) return fail(CGPU_EINVAL);
  DeviceGuard dg(ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  const uint32_t m0 = n < kZcChunk ? n : kZcChunk;
  if (int e = grow_dev(&ctx->d_zc, &ctx->zc_cap, (size_t)m0 * kZcSlot + 64)) return fail(e);
  const size_t ptrs = 0, counters = align_up(8ull * m0, 256);
  const HostLayout lay(m0, fields != nullptr, counters + 256);
  if (int e = grow(&ctx->h_desc, &ctx->d_desc, &ctx->desc_cap, lay.end)) return fail(e);
  hipStream_t s = ctx->stream;
  uint8_t *D = ctx->d_desc, *H = ctx->h_desc;
  ZcCounters *dcnt = (ZcCounters *)(D + counters), *hcnt = (ZcCounters *)(H + counters);
  uint32_t bad_total = 0;
  for (uint32_t at = 0; at < n;) {
    uint32_t m = n - at < m0 ? n - at : m0;
    for (;;) {
      memcpy(H + ptrs, mbufs + at, 8ull * m);
      if (hipMemcpyAsync(D + ptrs, H + ptrs, 8ull * m, hipMemcpyHostToDevice, s) != hipSuccess)
        return fail(CGPU_EIO);
      const size_t cap = ctx->zc_cap < kZcArenaMax ? ctx->zc_cap : kZcArenaMax;
      if (gather_chunk(ctx, (const uint64_t *)(D + ptrs), m, ctx->d_zc, cap,
                       (uint32_t *)(D + lay.off), (uint16_t *)(D + lay.len), dcnt, 0, nullptr,
                       0, s) != hipSuccess)
        return fail(CGPU_EIO);
      // The parse is queued behind the gather without waiting for its
      // cursor: in the common case the chunk fits and one sync serves both.
      // On an overflow (a chunk of frames larger than the arena so far, e.g.
      // the first burst from a jumbo mempool) the frames past `cap` were not
      // gathered, and the results this pass wrote for the chunk are
      // overwritten by the retry below; only that rare chunk is parsed twice.
      if (int e = parse_and_return(ctx, ctx->d_zc, cap, m, lay, flags, meta, csum, flow_hash,
                                   fields, at))
        return e;
      if (hipMemcpyAsync(hcnt, dcnt, sizeof(ZcCounters), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
        return fail(CGPU_EIO);
      const uint64_t need = hcnt->cursor + 64;
      if (need <= cap) break;
      if (need > kZcArenaMax) {  // fewer mbufs in this chunk
        m = (uint32_t)((uint64_t)m * (kZcArenaMax / 2) / need);
        if (m == 0) m = 1;
        continue;
      }
      if (int e = grow_dev(&ctx->d_zc, &ctx->zc_cap, need)) return fail(e);
    }
    bad_total += hcnt->bad;
    at += m;
  }
  if (int e = sync_done(ctx)) return fail(e);
  return bad_total ? fail(CGPU_EINVAL) : ok();
}

// Zero-copy from (frame address, length) pairs: as parse_zero_copy, with the
// pairs uploaded instead of mbuf pointers and no mbuf header read.
static int parse_frames_zero_copy(cgpu_ctx *ctx, const uint8_t *const *pkt, const uint16_t *len,
                                  uint32_t n, uint32_t flags, uint32_t *meta, uint32_t *csum,
                                  uint64_t *flow_hash, cgpu_hdr_record *fields) {
  if (ctx->nreg == 0) return fail(CGPU_EINVAL);
  DeviceGuard dg(ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  const uint32_t m0 = n < kZcChunk ? n : kZcChunk;
  if (int e = grow_dev(&ctx->d_zc, &ctx->zc_cap, (size_t)m0 * kZcSlot + 64)) return fail(e);
  const size_t ptrs = 0, lens = align_up(8ull * m0, 256), counters = lens + align_up(2ull * m0, 256);
  const HostLayout lay(m0, fields != nullptr, counters + 256);
  if (int e = grow(&ctx->h_desc, &ctx->d_desc, &ctx->desc_cap, lay.end)) return fail(e);
  hipStream_t s = ctx->stream;
  uint8_t *D = ctx->d_desc, *H = ctx->h_desc;
  ZcCounters *dcnt = (ZcCounters *)(D + counters), *hcnt = (ZcCounters *)(H + counters);
  uint32_t bad_total = 0;
  for (uint32_t at = 0; at < n;) {
    uint32_t m = n - at < m0 ? n - at : m0;
    for (;;) {
      memcpy(H + ptrs, pkt + at, 8ull * m);
      memcpy(H + lens, len + at, 2ull * m);
      if (hipMemcpyAsync(D + ptrs, H + ptrs, lens + 2ull * m, hipMemcpyHostToDevice, s) != hipSuccess)
        return fail(CGPU_EIO);
      const size_t cap = ctx->zc_cap < kZcArenaMax ? ctx->zc_cap : kZcArenaMax;
      if (gather_frames_chunk(ctx, (const uint64_t *)(D + ptrs), (const uint16_t *)(D + lens), m,
                              ctx->d_zc, cap, (uint32_t *)(D + lay.off), (uint16_t *)(D + lay.len),
                              dcnt, s) != hipSuccess)
        return fail(CGPU_EIO);
      // parsed before the cursor is read back: see parse_zero_copy
      if (int e = parse_and_return(ctx, ctx->d_zc, cap, m, lay, flags, meta, csum, flow_hash,
                                   fields, at))
        return e;
      if (hipMemcpyAsync(hcnt, dcnt, sizeof(ZcCounters), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
        return fail(CGPU_EIO);
      const uint64_t need = hcnt->cursor + 64;
      if (need <= cap) break;
      if (need > kZcArenaMax) {  // fewer frames in this chunk
        m = (uint32_t)((uint64_t)m * (kZcArenaMax / 2) / need);
        if (m == 0) m = 1;
        continue;
      }
      if (int e = grow_dev(&ctx->d_zc, &ctx->zc_cap, need)) return fail(e);
    }
    bad_total += hcnt->bad;
    at += m;
  }
  if (int e = sync_done(ctx)) return fail(e);
  return bad_total ? fail(CGPU_EINVAL) : ok();
}

// Zero-copy from (frame address, length) pairs, direct: when every frame of
// the burst lies in one registered region within a 4 GiB window, the parse
// kernel reads the frames through the device's mapping of that window, its
// descriptors (each frame's offset in the window, its length) from
// page-locked host memory, and writes its results there: one launch and
// one synchronisation per call, no copy engine and no gather: about 20 us
// per call against the gather path's 73 us, which matters at the RX path's
// burst sizes (RX_BURST_MAX = 32 per rte_eth_rx_burst, port.rs:149-171,
// aggregated by the caller), and as fast as the gather up to 2^18 frames
// (DESIGN.md §8).  Bursts of more than one gather chunk, or spread over
// several regions, take the gather path.  Returns 1 when the burst does not
// qualify (then nothing ran).
constexpr uint32_t kDirectMax = kZcChunk;

// Lays the burst's descriptors out in `slot` and launches the parse on the
// context's stream; returns 1 when the burst does not qualify (then nothing
// ran), else 0 or a (recorded) failure.
static int direct_launch(cgpu_ctx *ctx, cgpu_ctx::IoSlot &slot, const uint8_t *const *pkt,
                         const uint16_t *len, uint32_t n, uint32_t flags, uint32_t *meta,
                         uint32_t *csum, uint64_t *flow_hash, cgpu_hdr_record *fields) {
  if (n > kDirectMax) return 1;
  // one region holds every frame
  uint32_t r = 0;
  const uint64_t a0 = (uint64_t)(uintptr_t)pkt[0];
  for (; r < ctx->nreg; ++r)
    if (a0 >= ctx->reg[r].host_base && a0 + len[0] <= ctx->reg[r].host_base + ctx->reg[r].bytes) break;
  if (r == ctx->nreg) return 1;
  const uint64_t rb = ctx->reg[r].host_base, re = rb + ctx->reg[r].bytes;
  uint64_t lo = a0, hi = a0 + len[0];
  for (uint32_t i = 1; i < n; ++i) {
    const uint64_t a = (uint64_t)(uintptr_t)pkt[i], e = a + len[i];
    if (a < rb || e > re) return 1;
    lo = a < lo ? a : lo;
    hi = e > hi ? e : hi;
  }
  lo &= ~(uint64_t)255u;  // a frame's alignment within the window is its own
  if (lo < rb) lo = rb;
  if (hi - lo > 0xffff0000ull) return 1;
  DeviceGuard dg(ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  const HostLayout lay(n, fields != nullptr);
  if (lay.end > slot.cap) {
    if (slot.h) (void)hipHostFree(slot.h);
    slot.h = slot.d = nullptr;
    slot.cap = 0;
    const size_t cap = align_up(lay.end + lay.end / 2, 1u << 16);
    if (hipHostMalloc((void **)&slot.h, cap, hipHostMallocDefault) != hipSuccess) return fail(CGPU_ENOMEM);
    if (hipHostGetDevicePointer((void **)&slot.d, slot.h, 0) != hipSuccess || !slot.d) {
      (void)hipHostFree(slot.h);
      slot.h = nullptr;
      return fail(CGPU_EIO);
    }
    slot.cap = cap;
  }
  if (!slot.done && hipEventCreateWithFlags(&slot.done, hipEventDisableTiming) != hipSuccess) {
    slot.done = nullptr;
    return fail(CGPU_EIO);
  }
  uint32_t *hoff = (uint32_t *)(slot.h + lay.off);
  for (uint32_t i = 0; i < n; ++i) hoff[i] = (uint32_t)((uint64_t)(uintptr_t)pkt[i] - lo);
  memcpy(slot.h + lay.len, len, 2ull * n);
  uint8_t *D = slot.d;
  cgpu_batch b;
  b.arena = (const uint8_t *)(uintptr_t)(ctx->reg[r].dev_base + (lo - rb));
  b.arena_len = hi - lo;
  b.off = (const uint32_t *)(D + lay.off);
  b.len = (const uint16_t *)(D + lay.len);
  b.n = n;
  cgpu_parse_out o;
  o.meta = (uint32_t *)(D + lay.meta);
  o.csum = csum ? (uint32_t *)(D + lay.csum) : nullptr;
  o.flow_hash = flow_hash ? (uint64_t *)(D + lay.hash) : nullptr;
  o.fields = fields ? (cgpu_hdr_record *)(D + lay.fields) : nullptr;
  o.ext = nullptr;
  if (!csum) flags &= ~(CGPU_F_CSUM_IP | CGPU_F_CSUM_L4);
  if (!flow_hash) flags &= ~CGPU_F_FLOW_HASH;
  if (int e = cgpu_parse_batch(ctx, &b, flags, &o, ctx->stream)) return e;
  if (hipEventRecord(slot.done, ctx->stream) != hipSuccess) return fail(CGPU_EIO);
  slot.n = n;
  slot.o_meta = lay.meta;
  slot.o_csum = lay.csum;
  slot.o_hash = lay.hash;
  slot.o_fields = lay.fields;
  slot.meta = meta;
  slot.csum = csum;
  slot.hash = flow_hash;
  slot.fields = fields;
  return 0;
}

// Waits for the slot's burst and copies its results into the caller's
// arrays.  (Polling the event instead of the blocking wait measured the
// same: 20.0 against 20.2 us per 32-frame call)
static int direct_finish(cgpu_ctx *ctx, cgpu_ctx::IoSlot &slot) {
  DeviceGuard dg(ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  if (hipEventSynchronize(slot.done) != hipSuccess) return fail(CGPU_EIO);
  const uint32_t n = slot.n;
  memcpy(slot.meta, slot.h + slot.o_meta, 4ull * n);
  if (slot.csum) memcpy(slot.csum, slot.h + slot.o_csum, 4ull * n);
  if (slot.hash) memcpy(slot.hash, slot.h + slot.o_hash, 8ull * n);
  if (slot.fields) memcpy(slot.fields, slot.h + slot.o_fields, sizeof(cgpu_hdr_record) * (size_t)n);
  if (int e = sync_done(ctx)) return fail(e);
  return ok();
}

static int parse_frames_direct(cgpu_ctx *ctx, const uint8_t *const *pkt, const uint16_t *len,
                               uint32_t n, uint32_t flags, uint32_t *meta, uint32_t *csum,
                               uint64_t *flow_hash, cgpu_hdr_record *fields) {
  cgpu_ctx::IoSlot &slot = ctx->io[2];
  const int d = direct_launch(ctx, slot, pkt, len, n, flags, meta, csum, flow_hash, fields);
  if (d != 0) return d;
  return direct_finish(ctx, slot);
}

// rte_mbuf bursts on the direct path: the calling core reads each mbuf's
// data address and length (the header lines it has just written in
// rte_eth_rx_burst, so in its cache) after checking that the header lies in
// a registered region and that data_off + data_len <= buf_len, then runs
// the burst as frame pairs.  Returns 1 when the burst does not qualify
// (then the device gather runs it, and rejects what is invalid).
static int parse_mbufs_direct(cgpu_ctx *ctx, void *const *mbufs, uint32_t n, uint32_t flags,
                              uint32_t *meta, uint32_t *csum, uint64_t *flow_hash,
                              cgpu_hdr_record *fields) {
  if (n > kDirectMax) return 1;
  thread_local std::vector<const uint8_t *> pkt;
  thread_local std::vector<uint16_t> len;
  pkt.resize(n);
  len.resize(n);
  uint32_t r = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t m = (uint64_t)(uintptr_t)mbufs[i];
    auto inside = [&](uint32_t q) {
      return m >= ctx->reg[q].host_base && m + CGPU_MBUF_SIZE <= ctx->reg[q].host_base + ctx->reg[q].bytes;
    };
    if (!inside(r)) {
      for (r = 0; r < ctx->nreg && !inside(r); ++r) {
      }
      if (r == ctx->nreg) return 1;
    }
    uint16_t blen, doff;
    memcpy(&blen, (const uint8_t *)mbufs[i] + CGPU_MBUF_BUF_LEN_OFF, 2);
    memcpy(&doff, (const uint8_t *)mbufs[i] + CGPU_MBUF_DATA_OFF_OFF, 2);
    mbuf_fields(mbufs[i], pkt[i], len[i]);
    if ((uint32_t)doff + len[i] > blen) return 1;
  }
  return parse_frames_direct(ctx, pkt.data(), len.data(), n, flags, meta, csum, flow_hash, fields);
}

extern "C" {

int cgpu_parse_host(cgpu_ctx *ctx, const uint8_t *const *pkt, const uint16_t *len, uint32_t n,
                    uint32_t flags, uint32_t *meta, uint32_t *csum, uint64_t *flow_hash,
                    cgpu_hdr_record *fields) {
  if (!ctx) return fail(CGPU_EINVAL);
  if (n == 0) return ok();
  if (!pkt || !len || !meta) return fail(CGPU_EINVAL);
  auto get = [&](uint32_t i, const uint8_t *&p, uint16_t &l) {
    p = pkt[i];
    l = len[i];
    return p != nullptr || l == 0;
  };
  return parse_staged(ctx, n, get, flags, meta, csum, flow_hash, fields);
}

int cgpu_parse_frames(cgpu_ctx *ctx, const uint8_t *const *pkt, const uint16_t *len, uint32_t n,
                      uint32_t flags, uint32_t ingress, uint32_t *meta, uint32_t *csum,
                      uint64_t *flow_hash, cgpu_hdr_record *fields) {
  if (!ctx) return fail(CGPU_EINVAL);
  if (n == 0) return ok();
  if (!pkt || !len || !meta) return fail(CGPU_EINVAL);
  if (ingress == CGPU_INGRESS_ZERO_COPY) {
    if (ctx->nreg == 0) return fail(CGPU_EINVAL);
    const int d = parse_frames_direct(ctx, pkt, len, n, flags, meta, csum, flow_hash, fields);
    if (d <= 0) return d;
    return parse_frames_zero_copy(ctx, pkt, len, n, flags, meta, csum, flow_hash, fields);
  }
  if (ingress != CGPU_INGRESS_STAGE) return fail(CGPU_EINVAL);
  return cgpu_parse_host(ctx, pkt, len, n, flags, meta, csum, flow_hash, fields);
}

int cgpu_parse_frames_submit(cgpu_ctx *ctx, const uint8_t *const *pkt, const uint16_t *len,
                             uint32_t n, uint32_t flags, uint32_t *meta, uint32_t *csum,
                             uint64_t *flow_hash, uint32_t *ticket) {
  if (!ctx || !ticket) return fail(CGPU_EINVAL);
  if (n != 0 && (!pkt || !len || !meta)) return fail(CGPU_EINVAL);
  if (ctx->nreg == 0) return fail(CGPU_EINVAL);
  const uint32_t t = ctx->next_ticket;
  cgpu_ctx::IoSlot &slot = ctx->io[t & 1u];
  if (slot.pending) return fail(CGPU_EBUSY);  // two bursts in flight already
  int d = 1;
  if (n != 0) {
    d = direct_launch(ctx, slot, pkt, len, n, flags, meta, csum, flow_hash, nullptr);
    if (d < 0) return d;
  }
  // a burst that does not qualify for the direct path (or an empty one)
  // runs now, synchronously; its wait returns the result
  slot.rc = d == 0 ? 0 : (n == 0 ? 0 : parse_frames_zero_copy(ctx, pkt, len, n, flags, meta, csum,
                                                               flow_hash, nullptr));
  slot.n = d == 0 ? n : 0;
  slot.pending = true;
  slot.ticket = t;
  ctx->next_ticket = t + 1u == 0u ? 1u : t + 1u;
  *ticket = t;
  return ok();
}

int cgpu_parse_frames_wait(cgpu_ctx *ctx, uint32_t ticket) {
  if (!ctx) return fail(CGPU_EINVAL);
  cgpu_ctx::IoSlot &slot = ctx->io[ticket & 1u];
  if (!slot.pending || slot.ticket != ticket) return fail(CGPU_EINVAL);
  slot.pending = false;
  if (slot.n == 0) return slot.rc ? fail(slot.rc) : ok();
  return direct_finish(ctx, slot);
}

// Host regions (DESIGN.md §14 "Host registration"): the library borrows
// host memory only where it can tell that the range is the caller's for
// the registration's lifetime.  A range must be whole pages: hipHostRegister
// pins and maps whole pages, so a partial page would pin (and, for a
// pageable copy's on-the-fly pinning, alias) bytes of allocations the
// caller does not own.  Memory that is already page-locked is accepted only
// when the whole range lies inside ONE pinned allocation (hipHostMalloc'd,
// torch pinned memory); a range that merely overlaps someone's pinned pages
// is refused rather than mapped through a registration whose lifetime the
// library does not control.  Regions of one context never share a page.
int cgpu_host_register(cgpu_ctx *ctx, void *base, size_t bytes) {
  if (!ctx || !base || bytes == 0) return fail(CGPU_EINVAL);
  static const uint64_t page = (uint64_t)sysconf(_SC_PAGESIZE);
  const uint64_t lo = (uint64_t)(uintptr_t)base, hi = lo + bytes;
  if (lo % page || bytes % page || hi < lo) return fail(CGPU_EINVAL);
  if (ctx->nreg >= cgpu::kMaxRegions) return fail(CGPU_EINVAL);
  for (uint32_t r = 0; r < ctx->nreg; ++r) {
    const cgpu::HostRegion &g = ctx->reg[r];
    if (lo < g.host_base + g.bytes && g.host_base < hi) return fail(CGPU_EINVAL);
  }
  DeviceGuard dg(ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  hipPointerAttribute_t attr;
  bool locked = hipPointerGetAttributes(&attr, base) == hipSuccess && attr.type == hipMemoryTypeHost;
  (void)hipGetLastError();
  if (!locked) {  // the last byte must not be page-locked either
    hipPointerAttribute_t at2;
    const bool last = hipPointerGetAttributes(&at2, (void *)(uintptr_t)(hi - 1)) == hipSuccess &&
                      at2.type == hipMemoryTypeHost;
    (void)hipGetLastError();
    if (last) return fail(CGPU_EINVAL);
  } else {  // one pinned allocation holds the whole range
    hipDeviceptr_t pb = nullptr;
    size_t ps = 0;
    const bool whole = hipMemGetAddressRange(&pb, &ps, base) == hipSuccess &&
                       (uint64_t)(uintptr_t)pb <= lo && hi <= (uint64_t)(uintptr_t)pb + ps;
    (void)hipGetLastError();
    if (!whole) return fail(CGPU_EINVAL);
  }
  const bool owned = !locked;
  if (owned && hipHostRegister(base, bytes, hipHostRegisterMapped) != hipSuccess) {
    (void)hipGetLastError();
    return fail(CGPU_ENOMEM);
  }
  void *dev = nullptr;
  if (hipHostGetDevicePointer(&dev, base, 0) != hipSuccess || !dev) {
    (void)hipGetLastError();
    if (owned) (void)hipHostUnregister(base);
    return fail(CGPU_EIO);
  }
  cgpu::HostRegion &r = ctx->reg[ctx->nreg];
  r.host_base = lo;
  r.dev_base = (uint64_t)(uintptr_t)dev;
  r.bytes = bytes;
  ctx->reg_owned[ctx->nreg] = owned;
  ++ctx->nreg;
  return ok();
}

// Every entry point that reads or writes registered memory runs on the
// context's stream and has synchronised it before returning; the sync here
// also covers a call that failed part-way, so no device access to the
// region can follow its unpinning.
int cgpu_host_unregister(cgpu_ctx *ctx, void *base) {
  if (!ctx || !base) return fail(CGPU_EINVAL);
  for (uint32_t r = 0; r < ctx->nreg; ++r) {
    if (ctx->reg[r].host_base != (uint64_t)(uintptr_t)base) continue;
    DeviceGuard dg(ctx->device);
    if (!dg.ok()) return fail(CGPU_ENODEV);
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) return fail(CGPU_EIO);
    if (ctx->reg_owned[r] && hipHostUnregister(base) != hipSuccess) return fail(CGPU_EIO);
    for (uint32_t q = r + 1; q < ctx->nreg; ++q) {
      ctx->reg[q - 1] = ctx->reg[q];
      ctx->reg_owned[q - 1] = ctx->reg_owned[q];
    }
    --ctx->nreg;
    ctx->reg[ctx->nreg] = cgpu::HostRegion{0, 0, 0};
    return ok();
  }
  return fail(CGPU_EINVAL);
}

int cgpu_parse_mbufs(cgpu_ctx *ctx, void *const *mbufs, uint32_t n, uint32_t flags,
                     uint32_t ingress, uint32_t *meta, uint32_t *csum, uint64_t *flow_hash,
                     cgpu_hdr_record *fields) {
  if (!ctx) return fail(CGPU_EINVAL);
  if (n == 0) return ok();
  if (!mbufs || !meta) return fail(CGPU_EINVAL);
  if (ingress == CGPU_INGRESS_ZERO_COPY) {
    if (ctx->nreg == 0) return fail(CGPU_EINVAL);
    const int d = parse_mbufs_direct(ctx, mbufs, n, flags, meta, csum, flow_hash, fields);
    if (d <= 0) return d;
    return parse_zero_copy(ctx, mbufs, n, flags, meta, csum, flow_hash, fields);
  }
  if (ingress != CGPU_INGRESS_STAGE) return fail(CGPU_EINVAL);
  auto get = [&](uint32_t i, const uint8_t *&p, uint16_t &l) {
    if (!mbufs[i]) return false;
    mbuf_fields(mbufs[i], p, l);
    return p != nullptr || l == 0;
  };
  return parse_staged(ctx, n, get, flags, meta, csum, flow_hash, fields);
}

int cgpu_portmap_create(cgpu_ctx *ctx, uint32_t capacity_log2, uint16_t first_port,
                        cgpu_portmap **out) {
  if (!ctx || !out || capacity_log2 < 4 || capacity_log2 > 29) return fail(CGPU_EINVAL);
  *out = nullptr;
  DeviceGuard dg(ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  const size_t cap = (size_t)1 << capacity_log2;
  const size_t o_rev = 256;
  const size_t o_slots = o_rev + 65536 * 20;
  const size_t bytes = o_slots + cap * sizeof(cgpu::PortSlot);
  void *mem = nullptr;
  if (hipMalloc(&mem, bytes) != hipSuccess) return fail(CGPU_ENOMEM);
  cgpu_portmap *pm = new (std::nothrow) cgpu_portmap();
  if (!pm) {
    (void)hipFree(mem);
    return fail(CGPU_ENOMEM);
  }
  pm->ctx = ctx;
  pm->mem = mem;
  uint8_t *p = (uint8_t *)mem;
  pm->dev.state = (uint32_t *)p;
  pm->dev.rev = (uint32_t *)(p + o_rev);
  pm->dev.slots = (cgpu::PortSlot *)(p + o_slots);
  pm->dev.cap_mask = (uint32_t)(cap - 1);
  // per-map random hash seeds (crafted keys cannot collide on purpose)
  {
    std::random_device rd;
    pm->dev.seed_hash = rd();
    pm->dev.seed_tag = rd();
    for (int j = 0; j < 5; ++j) {  // odd, and not trivially small
      pm->dev.mul_hash[j] = rd() | 0x80000001u;
      pm->dev.mul_tag[j] = rd() | 0x80000001u;
    }
  }
  pm->dev.tag_mask = 0xffffffffu;
#ifdef CGPU_TEST_HOOKS
  // CGPU_TEST_NAT64_TAG_MASK: keep only these bits of the claim tags, so
  // that distinct keys collide on them and the tail's repair runs (every
  // batch then takes the serial repair: slow, never wrong)
  pm->dev.tag_mask = test_hook("CGPU_TEST_NAT64_TAG_MASK", 1u, 0xffffffffu, 0xffffffffu);
#endif
  if (hipEventCreateWithFlags(&pm->done, hipEventDisableTiming) != hipSuccess) {
    (void)hipFree(mem);
    delete pm;
    return fail(CGPU_EIO);
  }
  if (cgpu::launch_portmap_init(pm->dev, first_port, ctx->stream) != hipSuccess ||
      hipEventRecord(pm->done, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess) {
    (void)hipEventDestroy(pm->done);
    (void)hipFree(mem);
    delete pm;
    return fail(CGPU_EIO);
  }
  *out = pm;
  return ok();
}

int cgpu_portmap_reset(cgpu_portmap *pm, uint16_t first_port, void *stream) {
  if (!pm) return fail(CGPU_EINVAL);
  DeviceGuard dg(pm->ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  // behind the map's earlier calls, whatever stream they ran on
  if (hipStreamWaitEvent((hipStream_t)stream, pm->done, 0) != hipSuccess) return fail(CGPU_EIO);
  hipError_t e = cgpu::launch_portmap_init(pm->dev, first_port, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e);
  if (hipEventRecord(pm->done, (hipStream_t)stream) != hipSuccess) return fail(CGPU_EIO);
  pm->last_sid = stream_id(stream);
  return ok();
}

void cgpu_portmap_destroy(cgpu_portmap *pm) {
  if (!pm) return;
  DeviceGuard dg(pm->ctx->device);
  (void)hipEventSynchronize(pm->done);
  (void)hipEventDestroy(pm->done);
  if (pm->pkt_slot) (void)hipFree(pm->pkt_slot);
  (void)hipFree(pm->mem);
  delete pm;
}

static int read_state(cgpu_portmap *pm, uint32_t st[4]) {
  DeviceGuard dg(pm->ctx->device);
  if (!dg.ok()) return CGPU_ENODEV;
  // behind the map's latest call (its event), then on the context's stream
  if (hipEventSynchronize(pm->done) != hipSuccess ||
      hipMemcpyAsync(st, pm->dev.state, 16, hipMemcpyDeviceToHost, pm->ctx->stream) != hipSuccess ||
      hipStreamSynchronize(pm->ctx->stream) != hipSuccess)
    return CGPU_EIO;
  return 0;
}

int cgpu_portmap_next_port(cgpu_portmap *pm, uint16_t *next_port) {
  if (!pm || !next_port) return fail(CGPU_EINVAL);
  uint32_t st[4];
  if (int e = read_state(pm, st)) return fail(e);
  *next_port = (uint16_t)st[0];
  return ok();
}

int cgpu_portmap_size(cgpu_portmap *pm, uint32_t *entries) {
  if (!pm || !entries) return fail(CGPU_EINVAL);
  uint32_t st[4];
  if (int e = read_state(pm, st)) return fail(e);
  *entries = st[1];
  return ok();
}

static int nat64_call(bool to4, cgpu_ctx *ctx, cgpu_portmap *pm, const cgpu_batch *in, uint8_t *out_arena,
                    uint64_t out_arena_len, const uint32_t *out_off, uint16_t *out_len,
                    uint8_t *disposition, uint8_t *status, void *stream) {
  if (!ctx || !pm) return fail(CGPU_EINVAL);
  if (int e = check_batch(in)) return fail(e);
  if (in->n == 0) return ok();
  if (!out_arena || !out_off || !out_len || !disposition || !status) return fail(CGPU_EINVAL);
  if (out_arena_len > 0xffff0000ull) return fail(CGPU_EINVAL);
  if (in->n >= 0x7fffffffu) return fail(CGPU_EINVAL);
  DeviceGuard dg(ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  if (pm->scratch_n < in->n) {
    // the map's previous call (any stream) may still be using the old
    // scratch: wait for it before the scratch is freed and replaced
    if (pm->pkt_slot && hipEventSynchronize(pm->done) != hipSuccess) return fail(CGPU_EIO);
    if (pm->pkt_slot) (void)hipFree(pm->pkt_slot);
    pm->pkt_slot = nullptr;
    pm->scratch_n = 0;
    void *m = nullptr;
    const size_t o_chunks = align_up(4ull * in->n, 4096);
    // counts, bases, 8-word masks per chunk, the tail's list of tag
    // collisions and its control lines
    const size_t o_key = o_chunks + align_up(cgpu::nat64_chunk_bytes(in->n), 256);
    const size_t o_port = o_key + align_up(16ull * in->n, 256);
    const size_t o_c0 = o_port + align_up(2ull * in->n, 256);
    const size_t o_wf = o_c0 + align_up(4ull * in->n, 256);
    const size_t o_end = o_wf + align_up(in->n / 32u + 1u, 256);
    if (hipMalloc(&m, o_end) != hipSuccess) return fail(CGPU_ENOMEM);
    pm->pkt_slot = (uint32_t *)m;
    pm->chunks = (uint32_t *)((uint8_t *)m + o_chunks);
    pm->stash_key = (cgpu::u32x4 *)((uint8_t *)m + o_key);
    pm->stash_port = (uint16_t *)((uint8_t *)m + o_port);
    pm->stash_c0 = (uint32_t *)((uint8_t *)m + o_c0);
    pm->wave_flag = (uint8_t *)m + o_wf;
    // the tail's control lines start at zero; its last workgroup leaves them so
    if (hipMemsetAsync((uint8_t *)pm->chunks + cgpu::nat64_ctl_offset(in->n), 0,
                       cgpu::nat64_chunk_bytes(in->n) - cgpu::nat64_ctl_offset(in->n),
                       (hipStream_t)stream) != hipSuccess) {
      (void)hipFree(m);
      pm->pkt_slot = nullptr;
      return fail(CGPU_EIO);
    }
    pm->scratch_n = in->n;
  }
  cgpu::Nat64Args a;
  a.arena = in->arena;
  a.arena_len = (uint32_t)in->arena_len;
  a.off = in->off;
  a.len = in->len;
  a.n = in->n;
  a.out_arena = out_arena;
  a.out_arena_len = (uint32_t)out_arena_len;
  a.out_off = out_off;
  a.out_len = out_len;
  a.disposition = disposition;
  a.status = status;
  a.pkt_slot = pm->pkt_slot;
  a.wave_flag = pm->wave_flag;
  a.chunks = pm->chunks;
  a.ctl = pm->chunks + cgpu::nat64_ctl_offset(pm->scratch_n) / 4u;
  a.stash_key = pm->stash_key;
  a.stash_port = pm->stash_port;
  a.stash_c0 = pm->stash_c0;
  a.par = pm->calls & 1u;
  a.room = pm->room;
  a.pm = pm->dev;
  // Calls on one map are ordered: behind the previous call's completion
  // event, whatever stream it ran on.  On the previous call's own stream the
  // order is the stream's; the stream is recognised by its id, never by its
  // handle (a destroyed stream's handle can come back for a new stream while
  // the old one's work is still pending).
  const unsigned long long sid = stream_id(stream);
  if ((sid == 0 || sid != pm->last_sid) &&
      hipStreamWaitEvent((hipStream_t)stream, pm->done, 0) != hipSuccess)
    return fail(CGPU_EIO);
  pm->last_sid = sid;
  // the completion event rides on the call's last kernel (no marker packet)
  hipError_t e = to4 ? cgpu::launch_nat64_6to4(a, (hipStream_t)stream, pm->done)
                     : cgpu::launch_nat64_4to6(a, (hipStream_t)stream, pm->done);
  if (e != hipSuccess) return hip_fail(e);
  if (to4) ++pm->calls;
  return ok();
}

int cgpu_nat64_6to4(cgpu_ctx *ctx, cgpu_portmap *pm, const cgpu_batch *in, uint8_t *out_arena,
                    uint64_t out_arena_len, const uint32_t *out_off, uint16_t *out_len,
                    uint8_t *disposition, uint8_t *status, void *stream) {
  return nat64_call(true, ctx, pm, in, out_arena, out_arena_len, out_off, out_len, disposition,
                    status, stream);
}

int cgpu_nat64_4to6(cgpu_ctx *ctx, cgpu_portmap *pm, const cgpu_batch *in, uint8_t *out_arena,
                    uint64_t out_arena_len, const uint32_t *out_off, uint16_t *out_len,
                    uint8_t *disposition, uint8_t *status, void *stream) {
  return nat64_call(false, ctx, pm, in, out_arena, out_arena_len, out_off, out_len, disposition,
                    status, stream);
}

// nat64 over an rte_mbuf burst: zero-copy gather, the device rewrite, the
// ACT frames scattered back into their mbufs (cgpu_nat64_mbufs).  The call
// is all or nothing: every mbuf pointer and frame is validated before the
// first frame is rewritten or the port map changes (a burst of more than one
// chunk is validated chunk by chunk first).
// mbufs, or (frames, flen, ftail, out_len) for frame pairs: the device then
// reads and writes only the frames, and reports out_len for the caller to
// set data_len / pkt_len.
static int nat64_mbufs(bool to4, cgpu_ctx *ctx, cgpu_portmap *pm, void *const *mbufs, uint32_t n,
                       uint8_t *disposition, uint8_t *status, const uint8_t *const *frames = nullptr,
                       const uint16_t *flen = nullptr, const uint16_t *ftail = nullptr,
                       uint16_t *out_len = nullptr) {
  if (!ctx || !pm) return fail(CGPU_EINVAL);
  if (n == 0) return ok();
  const bool fm = frames != nullptr;
  if ((!fm && !mbufs) || (fm && (!flen || !out_len || (!to4 && !ftail))) || !disposition ||
      !status || ctx->nreg == 0)
    return fail(CGPU_EINVAL);
  DeviceGuard dg(ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  const uint32_t m0 = n < kZcChunk ? n : kZcChunk;
  const size_t want = (size_t)m0 * kZcSlot + 64;  // >= round_up(2048 + 20, 64) per frame
  if (int e = grow_dev(&ctx->d_zc, &ctx->zc_cap, want)) return fail(e);
  if (int e = grow_dev(&ctx->d_out, &ctx->out_cap, want)) return fail(e);
  // descriptor area: ptrs | off | len | out_len | disp | status | egress records | counters
  const size_t o_ptr = 0, o_off = align_up(8ull * m0, 256), o_len = o_off + align_up(4ull * m0, 256);
  const size_t o_olen = o_len + align_up(2ull * m0, 256), o_disp = o_olen + align_up(2ull * m0, 256);
  const size_t o_st = o_disp + align_up(m0, 256), o_eg = o_st + align_up(m0, 256);
  const size_t o_fl = o_eg + align_up(24ull * m0, 256), o_ft = o_fl + align_up(2ull * m0, 256);
  const size_t o_cnt = o_ft + align_up(2ull * m0, 256);
  if (int e = grow(&ctx->h_desc, &ctx->d_desc, &ctx->desc_cap, o_cnt + 256)) return fail(e);
  uint8_t *D = ctx->d_desc, *H = ctx->h_desc;
  ZcCounters *dcnt = (ZcCounters *)(D + o_cnt), *hcnt = (ZcCounters *)(H + o_cnt);
  hipStream_t s = ctx->stream;
  const uint32_t slot_extra = to4 ? 0u : 20u;  // 4to6 frames grow by 20 B in their slot
  auto upload = [&](uint32_t at, uint32_t m) {
    if (!fm) {
      memcpy(H + o_ptr, mbufs + at, 8ull * m);
      return hipMemcpyAsync(D + o_ptr, H + o_ptr, 8ull * m, hipMemcpyHostToDevice, s) == hipSuccess;
    }
    memcpy(H + o_ptr, frames + at, 8ull * m);
    memcpy(H + o_fl, flen + at, 2ull * m);
    if (ftail) memcpy(H + o_ft, ftail + at, 2ull * m);
    return hipMemcpyAsync(D + o_ptr, H + o_ptr, 8ull * m, hipMemcpyHostToDevice, s) == hipSuccess &&
           hipMemcpyAsync(D + o_fl, H + o_fl, o_cnt - o_fl, hipMemcpyHostToDevice, s) == hipSuccess;
  };
  const uint64_t *d_frames = fm ? (const uint64_t *)(D + o_ptr) : nullptr;
  const uint16_t *d_flen = fm ? (const uint16_t *)(D + o_fl) : nullptr;
  const uint16_t *d_ftail = fm && ftail ? (const uint16_t *)(D + o_ft) : nullptr;
  if (n > m0) {  // validate every chunk before anything is written
    uint32_t bad = 0;
    for (uint32_t at = 0; at < n; at += m0) {
      const uint32_t m = n - at < m0 ? n - at : m0;
      if (!upload(at, m) ||
          gather_chunk(ctx, (const uint64_t *)(D + o_ptr), m, nullptr, 0, nullptr, nullptr, dcnt,
                       0, nullptr, 0, s, d_frames, d_flen, d_ftail) != hipSuccess ||
          hipMemcpyAsync(hcnt, dcnt, sizeof(ZcCounters), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
        return fail(CGPU_EIO);
      bad += hcnt->bad;
    }
    if (bad) return fail(CGPU_EINVAL);
  }
  for (uint32_t at = 0; at < n;) {
    uint32_t m = n - at < m0 ? n - at : m0;
    size_t cap;
    for (;;) {
      cap = ctx->zc_cap < kZcArenaMax ? ctx->zc_cap : kZcArenaMax;
      if (!upload(at, m) ||
          gather_chunk(ctx, (const uint64_t *)(D + o_ptr), m, ctx->d_zc, cap,
                       (uint32_t *)(D + o_off), (uint16_t *)(D + o_len), dcnt, slot_extra,
                       D + o_eg, m0, s, d_frames, d_flen, d_ftail) != hipSuccess ||
          hipMemcpyAsync(hcnt, dcnt, sizeof(ZcCounters), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
        return fail(CGPU_EIO);
      if (hcnt->bad) return fail(CGPU_EINVAL);  // before any rewrite of this burst
      const uint64_t need = hcnt->cursor + 64;
      if (need <= cap) break;
      if (need > kZcArenaMax) {
        m = (uint32_t)((uint64_t)m * (kZcArenaMax / 2) / need);
        if (m == 0) m = 1;
        continue;
      }
      if (int e = grow_dev(&ctx->d_zc, &ctx->zc_cap, need)) return fail(e);
      if (int e = grow_dev(&ctx->d_out, &ctx->out_cap, need)) return fail(e);
    }
    cgpu_batch in;
    in.arena = ctx->d_zc;
    in.arena_len = cap;
    in.off = (const uint32_t *)(D + o_off);
    in.len = (const uint16_t *)(D + o_len);
    in.n = m;
    pm->room = 65535u;  // the scatter applies each mbuf's real tailroom
    const int e = nat64_call(to4, ctx, pm, &in, ctx->d_out, cap, in.off,
                             (uint16_t *)(D + o_olen), D + o_disp, D + o_st, s);
    pm->room = 2048u;
    if (e) return e;
    const uint64_t *mb = (const uint64_t *)(D + o_eg);
    cgpu::ScatterArgs sc;
    sc.out_arena = ctx->d_out;
    sc.out_off = in.off;
    sc.out_len = (const uint16_t *)(D + o_olen);
    sc.disposition = D + o_disp;
    sc.status = D + o_st;
    sc.mb_dev = mb;
    sc.fr_dev = mb + m0;
    sc.pkt_len = (const uint32_t *)(mb + 2 * (size_t)m0);
    sc.tailroom = sc.pkt_len + m0;
    sc.in_len = in.len;
    sc.n = m;
    sc.delta = to4 ? -20 : 20;
    if (cgpu::launch_mbuf_scatter(sc, s) != hipSuccess) return fail(CGPU_EIO);
    if (hipMemcpyAsync(H + o_disp, D + o_disp, o_eg - o_disp, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return fail(CGPU_EIO);
    memcpy(disposition + at, H + o_disp, m);
    memcpy(status + at, H + o_st, m);
    if (fm) {  // out_len of ACT frames (0 otherwise), for the caller's data_len
      if (hipMemcpyAsync(H + o_olen, D + o_olen, 2ull * m, hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
        return fail(CGPU_EIO);
      const uint16_t *ol = (const uint16_t *)(H + o_olen);
      for (uint32_t j = 0; j < m; ++j) out_len[at + j] = disposition[at + j] == CGPU_ACT ? ol[j] : 0;
    }
    at += m;
  }
  return ok();
}

// nat64 over frame pairs, direct: when every frame (with the 20 bytes a
// 4to6 rewrite may grow into, where its tailroom allows it) lies in one
// registered region, the fused kernel reads the frames through the device's
// mapping of that region, its descriptors from page-locked host memory, and
// writes the dispositions, statuses and new lengths there; the scatter
// writes every ACT frame back into its own buffer.  One synchronisation per
// call, no gather and no copies.  6to4 rewrites each frame in
// place (its output, 20 B shorter, starts where it does: every output byte
// j comes from input byte j + 20 or later, which the kernel has loaded
// before it stores j); 4to6 output passes through a device arena (frame i
// at i * kNatSlot) and the scatter, since a frame longer than one 256-B
// pass would read bytes its own first pass had already grown over.
// Returns 1 when the burst does not qualify (then nothing ran).
constexpr uint32_t kNatSlot = 2112;  // >= 2048 + 20, a multiple of 64

static int nat64_frames_direct(bool to4, cgpu_ctx *ctx, cgpu_portmap *pm,
                               const uint8_t *const *frames, const uint16_t *flen,
                               const uint16_t *ftail, uint32_t n, uint16_t *out_len,
                               uint8_t *disposition, uint8_t *status) {
  if (n > kDirectMax) return 1;
  uint32_t r = 0;
  const uint64_t a0 = (uint64_t)(uintptr_t)frames[0];
  for (; r < ctx->nreg; ++r)
    if (a0 >= ctx->reg[r].host_base && a0 + flen[0] <= ctx->reg[r].host_base + ctx->reg[r].bytes) break;
  if (r == ctx->nreg) return 1;
  const uint64_t rb = ctx->reg[r].host_base, re = rb + ctx->reg[r].bytes;
  uint64_t lo = a0, hi = a0 + flen[0];
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t a = (uint64_t)(uintptr_t)frames[i];
    if (flen[i] > 2048u) return 1;
    // the bytes the call may write: 4to6 grows a frame with the room by 20
    const uint64_t e = a + flen[i] + (!to4 && ftail[i] > 20u ? 20u : 0u);
    if (a < rb || e > re) return 1;
    lo = a < lo ? a : lo;
    hi = e > hi ? e : hi;
  }
  lo &= ~(uint64_t)255u;
  if (lo < rb) lo = rb;
  if (hi - lo > 0xffff0000ull) return 1;
  DeviceGuard dg(ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  if (int e = grow_dev(&ctx->d_out, &ctx->out_cap, (size_t)n * kNatSlot + 64)) return fail(e);
  // page-locked: off | len | out_off | out_len | disp | status | fr_dev | tailroom
  const size_t o_off = 0, o_len = align_up(4ull * n, 256), o_oo = o_len + align_up(2ull * n, 256);
  const size_t o_ol = o_oo + align_up(4ull * n, 256), o_d = o_ol + align_up(2ull * n, 256);
  const size_t o_st = o_d + align_up(n, 256), o_fr = o_st + align_up(n, 256);
  const size_t o_tr = o_fr + align_up(8ull * n, 256), o_end = o_tr + align_up(4ull * n, 256);
  cgpu_ctx::IoSlot &slot = ctx->io[2];
  if (o_end > slot.cap) {
    if (slot.h) (void)hipHostFree(slot.h);
    slot.h = slot.d = nullptr;
    slot.cap = 0;
    const size_t cap = align_up(o_end + o_end / 2, 1u << 16);
    if (hipHostMalloc((void **)&slot.h, cap, hipHostMallocDefault) != hipSuccess) return fail(CGPU_ENOMEM);
    if (hipHostGetDevicePointer((void **)&slot.d, slot.h, 0) != hipSuccess || !slot.d) {
      (void)hipHostFree(slot.h);
      slot.h = nullptr;
      return fail(CGPU_EIO);
    }
    slot.cap = cap;
  }
  uint8_t *H = slot.h, *D = slot.d;
  uint32_t *hoff = (uint32_t *)(H + o_off), *hoo = (uint32_t *)(H + o_oo), *htr = (uint32_t *)(H + o_tr);
  uint64_t *hfr = (uint64_t *)(H + o_fr);
  const uint64_t db = ctx->reg[r].dev_base - rb;  // host address -> device address
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t a = (uint64_t)(uintptr_t)frames[i];
    hoff[i] = (uint32_t)(a - lo);
    hoo[i] = i * kNatSlot;
    hfr[i] = flen[i] ? a + db : 0ull;  // an empty frame is never ACT
    htr[i] = ftail ? ftail[i] : 0u;
  }
  memcpy(H + o_len, flen, 2ull * n);
  cgpu_batch in;
  in.arena = (const uint8_t *)(uintptr_t)(ctx->reg[r].dev_base + (lo - rb));
  in.arena_len = hi - lo;
  in.off = (const uint32_t *)(D + o_off);
  in.len = (const uint16_t *)(D + o_len);
  in.n = n;
  pm->room = 65535u;  // the scatter applies each frame's real tailroom
  // 6to4: in place, out_off = off over the same window
  uint8_t *oa = to4 ? (uint8_t *)(uintptr_t)in.arena : ctx->d_out;
  const uint64_t oa_len = to4 ? in.arena_len : (uint64_t)n * kNatSlot + 64;
  const uint32_t *oo = to4 ? in.off : (const uint32_t *)(D + o_oo);
  const int e = nat64_call(to4, ctx, pm, &in, oa, oa_len, oo, (uint16_t *)(D + o_ol), D + o_d, D + o_st,
                           ctx->stream);
  pm->room = 2048u;
  if (e) return e;
  if (to4) {
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) return fail(CGPU_EIO);
    memcpy(disposition, H + o_d, n);
    memcpy(status, H + o_st, n);
    const uint16_t *ol = (const uint16_t *)(H + o_ol);
    for (uint32_t i = 0; i < n; ++i) out_len[i] = disposition[i] == CGPU_ACT ? ol[i] : 0;
    return ok();
  }
  cgpu::ScatterArgs sc;
  sc.out_arena = ctx->d_out;
  sc.out_off = (const uint32_t *)(D + o_oo);
  sc.out_len = (const uint16_t *)(D + o_ol);
  sc.disposition = D + o_d;
  sc.status = D + o_st;
  sc.mb_dev = nullptr;
  sc.fr_dev = (const uint64_t *)(D + o_fr);
  sc.pkt_len = nullptr;
  sc.tailroom = (const uint32_t *)(D + o_tr);
  sc.in_len = in.len;
  sc.n = n;
  sc.delta = to4 ? -20 : 20;
  if (cgpu::launch_mbuf_scatter(sc, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess)
    return fail(CGPU_EIO);
  memcpy(disposition, H + o_d, n);
  memcpy(status, H + o_st, n);
  const uint16_t *ol = (const uint16_t *)(H + o_ol);
  for (uint32_t i = 0; i < n; ++i) out_len[i] = disposition[i] == CGPU_ACT ? ol[i] : 0;
  return ok();
}

int cgpu_nat64_mbufs(cgpu_ctx *ctx, cgpu_portmap *pm, uint32_t direction, void *const *mbufs,
                     uint32_t n, uint8_t *disposition, uint8_t *status) {
  if (direction != CGPU_NAT64_6TO4 && direction != CGPU_NAT64_4TO6) return fail(CGPU_EINVAL);
  return nat64_mbufs(direction == CGPU_NAT64_6TO4, ctx, pm, mbufs, n, disposition, status);
}

int cgpu_nat64_frames(cgpu_ctx *ctx, cgpu_portmap *pm, uint32_t direction,
                      const uint8_t *const *frames, const uint16_t *len, const uint16_t *tailroom,
                      uint32_t n, uint16_t *out_len, uint8_t *disposition, uint8_t *status) {
  if (direction != CGPU_NAT64_6TO4 && direction != CGPU_NAT64_4TO6) return fail(CGPU_EINVAL);
  if (n != 0 && !frames) return fail(CGPU_EINVAL);
  const bool to4 = direction == CGPU_NAT64_6TO4;
  if (ctx && pm && n != 0 && len && out_len && disposition && status && ctx->nreg != 0 &&
      (to4 || tailroom)) {
    const int d = nat64_frames_direct(to4, ctx, pm, frames, len, tailroom, n, out_len, disposition, status);
    if (d <= 0) return d;
  }
  return nat64_mbufs(to4, ctx, pm, nullptr, n, disposition, status, frames, len, tailroom, out_len);
}

int cgpu_group_by(cgpu_ctx *ctx, const void *key, uint32_t key_kind, uint32_t n,
                  uint32_t n_groups, uint32_t *idx, uint32_t *group_off, void *stream) {
  if (!ctx || !group_off || n_groups < 1 || n_groups > 64) return fail(CGPU_EINVAL);
  if (key_kind != CGPU_KEY_U8 && key_kind != CGPU_KEY_META_CLASS) return fail(CGPU_EINVAL);
  if (n > (1u << 28)) return fail(CGPU_EINVAL);
  if (n == 0) {
    if (hipMemsetAsync(group_off, 0, 4ull * (n_groups + 1), (hipStream_t)stream) != hipSuccess)
      return fail(CGPU_EIO);
    return ok();
  }
  if (!key || !idx) return fail(CGPU_EINVAL);
  DeviceGuard dg(ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  const uint32_t tiles = cgpu::group_by_tiles(n);
  const size_t need = (size_t)tiles * n_groups;
  if (ctx->gb_cap < need) {
    if (ctx->gb_counts) (void)hipFree(ctx->gb_counts);
    ctx->gb_counts = nullptr;
    ctx->gb_cap = 0;
    if (hipMalloc(&ctx->gb_counts, 4 * need) != hipSuccess) return fail(CGPU_ENOMEM);
    ctx->gb_cap = need;
  }
  cgpu::GroupByArgs a;
  a.key = key;
  a.kind = key_kind;
  a.n = n;
  a.groups = n_groups;
  a.tiles = tiles;
  a.counts = ctx->gb_counts;
  a.idx = idx;
  a.group_off = group_off;
  hipError_t e = cgpu::launch_group_by(a, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e);
  return ok();
}

int cgpu_set_ip(cgpu_ctx *ctx, uint8_t *arena, uint64_t arena_len, const uint32_t *off,
                const uint16_t *len, const uint32_t *meta, uint32_t n, const cgpu_ip_addr *src,
                uint32_t src_stride, const cgpu_ip_addr *dst, uint32_t dst_stride,
                uint8_t *status, void *stream) {
  if (!ctx || n > CGPU_MAX_BATCH || src_stride > 1u || dst_stride > 1u) return fail(CGPU_EINVAL);
  if (n == 0) return ok();
  if (!arena || !off || !len || !meta || arena_len > 0xffff0000ull) return fail(CGPU_EINVAL);
  DeviceGuard dg(ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  cgpu::SetIpArgs a;
  a.arena = arena;
  a.arena_len = (uint32_t)arena_len;
  a.off = off;
  a.len = len;
  a.meta = meta;
  a.n = n;
  a.src = src;
  a.src_stride = src_stride;
  a.dst = dst;
  a.dst_stride = dst_stride;
  a.status = status;
  hipError_t e = cgpu::launch_set_ip(a, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e);
  return ok();
}

int cgpu_reconcile(cgpu_ctx *ctx, uint8_t *arena, uint64_t arena_len, const uint32_t *off,
                   const uint16_t *len, const uint32_t *meta, uint32_t n, uint32_t flags,
                   uint32_t depth, uint8_t *status, void *stream) {
  if (!ctx || n > CGPU_MAX_BATCH) return fail(CGPU_EINVAL);
  if (depth != CGPU_LAYER_L2 && depth != CGPU_LAYER_L3 && depth != CGPU_LAYER_L4)
    return fail(CGPU_EINVAL);
  if (n == 0) return ok();
  if (!arena || !off || !len || !meta || arena_len > 0xffff0000ull) return fail(CGPU_EINVAL);
  DeviceGuard dg(ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  // the accept-set defaults of cgpu_parse_batch
  if ((flags & (CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_V6)) == 0) flags |= CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_V6;
  if ((flags & (CGPU_F_ACCEPT_UDP | CGPU_F_ACCEPT_TCP | CGPU_F_ACCEPT_ICMP)) == 0)
    flags |= CGPU_F_ACCEPT_UDP | CGPU_F_ACCEPT_TCP;
  cgpu::ParseArgs a{};
  a.arena = arena;
  a.arena_len = (uint32_t)arena_len;
  a.off = off;
  a.len = len;
  a.n = n;
  a.accept = flags & (CGPU_F_ACCEPT_ALL | CGPU_F_ACCEPT_ICMP | CGPU_F_V6_EXT);
  a.wr_arena = arena;
  a.meta_in = meta;
  a.depth = depth;
  a.rstatus = status;
  set_schedule(ctx, a, stream);
  hipError_t e = cgpu::launch_reconcile(a, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e);
  return ok();
}

// cgpu_reconcile over frames in registered host memory: each region's
// frames are one arena window (its base the lowest frame address rounded
// down to 256 B, so a frame's alignment within the window is its own), and
// the reconcile kernel runs on the device's mapping of that window.
int cgpu_reconcile_frames(cgpu_ctx *ctx, uint8_t *const *frames, const uint16_t *len,
                          const uint32_t *meta, uint32_t n, uint32_t flags, uint32_t depth,
                          uint8_t *status) {
  if (!ctx || n > CGPU_MAX_BATCH) return fail(CGPU_EINVAL);
  if (depth != CGPU_LAYER_L2 && depth != CGPU_LAYER_L3 && depth != CGPU_LAYER_L4)
    return fail(CGPU_EINVAL);
  if (n == 0) return ok();
  if (!frames || !len || !meta || ctx->nreg == 0) return fail(CGPU_EINVAL);
  // every frame inside one registered region (checked before anything runs)
  std::vector<uint8_t> region(n);
  uint64_t lo[cgpu::kMaxRegions], hi[cgpu::kMaxRegions];
  uint32_t cnt[cgpu::kMaxRegions] = {};
  uint32_t last = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t a = (uint64_t)(uintptr_t)frames[i], e = a + len[i];
    auto inside = [&](uint32_t r) {
      const cgpu::HostRegion &g = ctx->reg[r];
      return a >= g.host_base && e <= g.host_base + g.bytes && (a != 0 || len[i] == 0);
    };
    uint32_t r = last;
    if (!inside(r)) {
      for (r = 0; r < ctx->nreg && !inside(r); ++r) {
      }
      if (r == ctx->nreg) return fail(CGPU_EINVAL);
      last = r;
    }
    region[i] = (uint8_t)r;
    if (cnt[r]++ == 0) {
      lo[r] = a;
      hi[r] = e;
    } else {
      lo[r] = a < lo[r] ? a : lo[r];
      hi[r] = e > hi[r] ? e : hi[r];
    }
  }
  for (uint32_t r = 0; r < ctx->nreg; ++r) {
    if (!cnt[r]) continue;
    lo[r] &= ~(uint64_t)255u;
    if (lo[r] < ctx->reg[r].host_base) lo[r] = ctx->reg[r].host_base;
    if (hi[r] - lo[r] > 0xffff0000ull) return fail(CGPU_EINVAL);
  }
  DeviceGuard dg(ctx->device);
  if (!dg.ok()) return fail(CGPU_ENODEV);
  // off u32 | len u16 | meta u32 | status u8 in page-locked host memory the
  // kernels read and write through its device mapping (no copies), each
  // region's frames in their own range; one synchronisation for the call
  const size_t o_off = 0, o_len = align_up(4ull * n, 256), o_meta = o_len + align_up(2ull * n, 256);
  const size_t o_st = o_meta + align_up(4ull * n, 256), o_end = o_st + align_up(n, 256);
  cgpu_ctx::IoSlot &slot = ctx->io[2];
  if (o_end > slot.cap) {
    if (slot.h) (void)hipHostFree(slot.h);
    slot.h = slot.d = nullptr;
    slot.cap = 0;
    const size_t cap = align_up(o_end + o_end / 2, 1u << 16);
    if (hipHostMalloc((void **)&slot.h, cap, hipHostMallocDefault) != hipSuccess) return fail(CGPU_ENOMEM);
    if (hipHostGetDevicePointer((void **)&slot.d, slot.h, 0) != hipSuccess || !slot.d) {
      (void)hipHostFree(slot.h);
      slot.h = nullptr;
      return fail(CGPU_EIO);
    }
    slot.cap = cap;
  }
  uint8_t *D = slot.d, *H = slot.h;
  hipStream_t s = ctx->stream;
  if ((flags & (CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_V6)) == 0) flags |= CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_V6;
  if ((flags & (CGPU_F_ACCEPT_UDP | CGPU_F_ACCEPT_TCP | CGPU_F_ACCEPT_ICMP)) == 0)
    flags |= CGPU_F_ACCEPT_UDP | CGPU_F_ACCEPT_TCP;
  uint32_t first[cgpu::kMaxRegions], fill[cgpu::kMaxRegions];
  for (uint32_t r = 0, acc = 0; r < ctx->nreg; ++r) {
    first[r] = fill[r] = acc;
    acc += cnt[r];
  }
  uint32_t *ho = (uint32_t *)(H + o_off), *hm = (uint32_t *)(H + o_meta);
  uint16_t *hl = (uint16_t *)(H + o_len);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t r = region[i], q = fill[r]++;
    ho[q] = (uint32_t)((uint64_t)(uintptr_t)frames[i] - lo[r]);
    hl[q] = len[i];
    hm[q] = meta[i];
  }
  for (uint32_t r = 0; r < ctx->nreg; ++r) {
    if (!cnt[r]) continue;
    uint8_t *win = (uint8_t *)(uintptr_t)(ctx->reg[r].dev_base + (lo[r] - ctx->reg[r].host_base));
    cgpu::ParseArgs a{};
    a.arena = win;
    a.arena_len = (uint32_t)(hi[r] - lo[r]);
    a.off = (const uint32_t *)(D + o_off) + first[r];
    a.len = (const uint16_t *)(D + o_len) + first[r];
    a.n = cnt[r];
    a.accept = flags & (CGPU_F_ACCEPT_ALL | CGPU_F_ACCEPT_ICMP | CGPU_F_V6_EXT);
    a.wr_arena = win;
    a.meta_in = (const uint32_t *)(D + o_meta) + first[r];
    a.depth = depth;
    a.rstatus = D + o_st + first[r];
    set_schedule(ctx, a, s);
    hipError_t e = cgpu::launch_reconcile(a, s);
    if (e != hipSuccess) return hip_fail(e);
  }
  if (hipStreamSynchronize(s) != hipSuccess) return fail(CGPU_EIO);
  if (status) {
    for (uint32_t r = 0; r < ctx->nreg; ++r) fill[r] = first[r];
    for (uint32_t i = 0; i < n; ++i) status[i] = H[o_st + fill[region[i]]++];
  }
  if (int e = sync_done(ctx)) return fail(e);
  return ok();
}

}  // extern "C"
