// microbench.hip — roofline calibration and ablations for the parse kernel.
//
//   stream_read   : coalesced dwordx4 grid-stride read of the arena (the
//                   achievable HBM read bandwidth on this box)
//   aos_window    : one lane per packet loads its own 64 B (the parse
//                   kernel's access pattern with no compute), writes 4 B
//   parse[flags]  : cgpu_parse_batch through the C ABI with feature subsets
//
// Each case rotates over R copies of the batch (> 256 MiB Infinity Cache)
// and reports mean device time per launch from hipEvents around a run of
// back-to-back launches.  Build: make -C tools ; run: tools/microbench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <vector>

#include "capsule_gpu.h"

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(2);                                                                \
    }                                                                         \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void stream_read(const u32x4 *p, size_t n16, uint32_t *out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256ull) {
    u32x4 v = __builtin_nontemporal_load(p + i);
    acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;  // practically never: keeps the loads
}

__global__ __launch_bounds__(256) void aos_window(const uint8_t *arena, const uint32_t *off,
                                                  uint32_t n, uint32_t *out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const u32x4 *q = reinterpret_cast<const u32x4 *>(arena + off[i]);
  u32x4 a = q[0], b = q[1], c = q[2], d = q[3];
  u32x4 s = a + b + c + d;
  out[i] = s[0] ^ s[1] ^ s[2] ^ s[3];
}

// AoS with a cache policy on the loads (AUX: 1 = glc, 2 = slc, 3 = both)
template <int AUX>
__global__ __launch_bounds__(256) void aos_window_aux(const uint8_t *arena, const uint32_t *off,
                                                      uint32_t n, uint32_t *out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(arena), (short)0, (int)(n * 64u), 0x00020000);
  const uint32_t o = off[i];
  u32x4 s = {0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < 4; ++c) s += __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(o + 16u * c), 0, AUX);
  out[i] = s[0] ^ s[1] ^ s[2] ^ s[3];
}

// AoS without the descriptor dependency (offset = 64 i): bounds the cost of
// the off[i] -> arena load chain
__global__ __launch_bounds__(256) void aos_nodesc(const uint8_t *arena, uint32_t n, uint32_t *out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(arena), (short)0, (int)(n * 64u), 0x00020000);
  u32x4 s = {0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < 4; ++c) s += __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(64u * i + 16u * c), 0, 0);
  out[i] = s[0] ^ s[1] ^ s[2] ^ s[3];
}

// AoS, grid-stride over packet groups with the next group's descriptor and
// window loads issued before the current group's are consumed
template <int GRID>
__global__ __launch_bounds__(256) void aos_loop(const uint8_t *arena, const uint32_t *off,
                                                uint32_t n, uint32_t *out) {
  auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(arena), (short)0, (int)(n * 64u), 0x00020000);
  uint32_t i = blockIdx.x * 256u + threadIdx.x;
  const uint32_t stride = GRID * 256u;
  uint32_t o = i < n ? off[i] : 0xffffff00u;
  u32x4 v[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(o + 16u * c), 0, 0);
  for (; i < n; i += stride) {
    const uint32_t j = i + stride;
    const uint32_t on = j < n ? off[j] : 0xffffff00u;
    u32x4 s = v[0] + v[1] + v[2] + v[3];
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(on + 16u * c), 0, 0);
    out[i] = s[0] ^ s[1] ^ s[2] ^ s[3];
  }
}

// LDS staging: the wave loads the 4 KiB span of its 64 packets coalesced
// (lane L, instruction c -> bytes 1024c + 16L), writes it to LDS with the
// 16-B chunk index XOR-swizzled by bits 8-9, then each lane reads its own 64 B.
__device__ __forceinline__ uint32_t swz(uint32_t a) { return a ^ (((a >> 8) & 3u) << 4); }

__global__ __launch_bounds__(256) void lds_window(const uint8_t *arena, const uint32_t *off,
                                                  uint32_t n, uint32_t *out) {
  __shared__ u32x4 lds[4][256];
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(arena), (short)0, (int)(n * 64u), 0x00020000);
  const uint32_t o = i < n ? off[i] : 0u;
  const uint32_t base = __builtin_amdgcn_readfirstlane(o);
  u32x4 v[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(base + 1024u * c + 16u * lane), 0, 0);
  char *L = reinterpret_cast<char *>(&lds[w][0]);
#pragma unroll
  for (int c = 0; c < 4; ++c) *reinterpret_cast<u32x4 *>(L + swz(1024u * c + 16u * lane)) = v[c];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  const uint32_t r = o - base;
  u32x4 s = {0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < 4; ++c) s += *reinterpret_cast<const u32x4 *>(L + swz(r + 16u * c));
  if (i < n) out[i] = s[0] ^ s[1] ^ s[2] ^ s[3];
}

// nat64-shaped data movement: 4 lanes per 256-B frame, 4 x 16-B chunks per
// lane, output chunk c <- input bytes [16c + SHIFT, 16c + SHIFT + 16).
template <int SHIFT>
__global__ __launch_bounds__(256) void copy_frames(const uint8_t *in, uint8_t *out, uint32_t n,
                                                   uint32_t new_len) {
  const uint32_t g = threadIdx.x & 3u, p = blockIdx.x * 64u + threadIdx.x / 4u;
  if (p >= n) return;
  auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(in), (short)0, (int)(n * 256u), 0x00020000);
  auto os = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)(n * 256u), 0x00020000);
  u32x4 v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t c = 4u * g + j;
    v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(16u * c < new_len ? p * 256u + 16u * c + SHIFT : 0xffffff00u), 0, 0);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t c = 4u * g + j;
    __builtin_amdgcn_raw_buffer_store_b128(v[j], os, (int)(16u * c + 16u <= new_len ? p * 256u + 16u * c : 0xffffff00u), 0, 0);
  }
}

// the nat64 6to4 shape on the copy_map mapping: 236-B output, chunks >= 2
// read from input + 20 (dword-aligned, not 16-B aligned), last chunk b96
template <int G, int AUX>
__global__ __launch_bounds__(256) void copy_shift(const uint8_t *in, uint8_t *out, uint32_t n) {
  constexpr int C = 16 / G;
  const uint32_t g = threadIdx.x % G, p = blockIdx.x * (256 / G) + threadIdx.x / G;
  if (p >= n) return;
  auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(in), (short)0, (int)(n * 256u), 0x00020000);
  auto os = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)(n * 256u), 0x00020000);
  u32x4 v[C];
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const uint32_t c = (uint32_t)j * G + g;
    const uint32_t src = c < 2u ? 16u * c : 16u * c + 20u;
    v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(16u * c < 236u ? p * 256u + src : 0xffffff00u), 0, AUX);
  }
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const uint32_t c = (uint32_t)j * G + g;
    if (16u * c + 16u <= 236u)
      __builtin_amdgcn_raw_buffer_store_b128(v[j], os, (int)(p * 256u + 16u * c), 0, AUX);
    else if (16u * c < 236u)
      __builtin_amdgcn_raw_buffer_store_b96(__builtin_shufflevector(v[j], v[j], 0, 1, 2), os,
                                            (int)(p * 256u + 16u * c), 0, AUX);
  }
}

// the nat64 6to4 shape in rows of 16 lanes (the rows path of nat64.hip):
// aligned 16-B loads, output chunk l >= 2 = {in(l+1).yzw, in(l+2).x} by DPP
// row shifts, 236-B output, last chunk b96
template <int CTRL>
__device__ __forceinline__ uint32_t dppz_mb(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, true);
}
template <uint32_t OSTRIDE>
__global__ __launch_bounds__(256) void copy_rows_dpp(const uint8_t *in, uint8_t *out, uint32_t n) {
  const uint32_t l = threadIdx.x & 15u, p = blockIdx.x * 16u + threadIdx.x / 16u;
  auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(in), (short)0, (int)(n * 256u), 0x00020000);
  auto os = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)(n * 256u), 0x00020000);
  const u32x4 A = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(p < n ? p * 256u + 16u * l : 0xffffff00u), 0, 0);
  u32x4 o = {dppz_mb<0x101>(A[1]), dppz_mb<0x101>(A[2]), dppz_mb<0x101>(A[3]), dppz_mb<0x102>(A[0])};
  if (l < 2u) o = A;
  if (p >= n) return;
  if (16u * l + 16u <= 236u)
    __builtin_amdgcn_raw_buffer_store_b128(o, os, (int)(p * OSTRIDE + 16u * l), 0, 0);
  else if (16u * l < 236u)
    __builtin_amdgcn_raw_buffer_store_b96(__builtin_shufflevector(o, o, 0, 1, 2), os, (int)(p * OSTRIDE + 16u * l), 0, 0);
}

// copy mapping sweep: G lanes per 256-B frame, 16/G chunks per lane, chunk
// order contiguous per lane (IL=false) or interleaved across the group (IL=true),
// cache policy AUX on loads and stores.
template <int G, bool IL, int AUX>
__global__ __launch_bounds__(256) void copy_map(const uint8_t *in, uint8_t *out, uint32_t n) {
  constexpr int C = 16 / G;
  const uint32_t g = threadIdx.x % G, p = blockIdx.x * (256 / G) + threadIdx.x / G;
  if (p >= n) return;
  auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(in), (short)0, (int)(n * 256u), 0x00020000);
  auto os = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)(n * 256u), 0x00020000);
  u32x4 v[C];
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const uint32_t c = IL ? (uint32_t)j * G + g : g * C + j;
    v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(p * 256u + 16u * c), 0, AUX);
  }
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const uint32_t c = IL ? (uint32_t)j * G + g : g * C + j;
    __builtin_amdgcn_raw_buffer_store_b128(v[j], os, (int)(p * 256u + 16u * c), 0, AUX);
  }
}

static uint32_t lcg(uint64_t &s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return (uint32_t)(s >> 33);
}

int main(int argc, char **argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
  const int iters = argc > 2 ? atoi(argv[2]) : 400;
  const uint32_t L = 64;
  const size_t bytes = (size_t)n * L;
  const int R = 8;
  const char *filter = argc > 3 ? argv[3] : "";
  // synthetic IPv4/UDP frames (checksums are not reconciled: timing only)
  std::vector<uint8_t> h(bytes);
  uint64_t s = 12345;
  for (size_t i = 0; i < bytes; ++i) h[i] = (uint8_t)lcg(s);
  for (uint32_t i = 0; i < n; ++i) {
    uint8_t *f = &h[(size_t)i * L];
    f[12] = 0x08; f[13] = 0x00; f[14] = 0x45; f[23] = 17;
  }
  std::vector<uint32_t> ho(n);
  std::vector<uint16_t> hl(n, (uint16_t)L);
  for (uint32_t i = 0; i < n; ++i) ho[i] = i * L;
  uint8_t *arena[R];
  uint32_t *off[R];
  uint16_t *len[R];
  for (int r = 0; r < R; ++r) {
    CK(hipMalloc(&arena[r], bytes));
    CK(hipMalloc(&off[r], 4ull * n));
    CK(hipMalloc(&len[r], 2ull * n));
    CK(hipMemcpy(arena[r], h.data(), bytes, hipMemcpyHostToDevice));
    CK(hipMemcpy(off[r], ho.data(), 4ull * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(len[r], hl.data(), 2ull * n, hipMemcpyHostToDevice));
  }
  uint32_t *meta, *csum, *scratch;
  uint64_t *hash;
  CK(hipMalloc(&meta, 4ull * n));
  CK(hipMalloc(&csum, 4ull * n));
  CK(hipMalloc(&hash, 8ull * n));
  CK(hipMalloc(&scratch, 4ull * n + 4096 * 4));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  cgpu_ctx *ctx;
  if (cgpu_ctx_create(0, &ctx)) { fprintf(stderr, "ctx\n"); return 2; }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  auto time_it = [&](const char *name, double algo_bytes, auto &&launch) {
    if (filter[0] && !strstr(name, filter)) return;
    for (int w = 0; w < 20; ++w) launch(w % R);
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(e0, st));
    for (int k = 0; k < iters; ++k) launch(k % R);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / iters;
    printf("{\"case\": \"%s\", \"us\": %.3f, \"GBps\": %.1f, \"Mpps\": %.1f}\n", name, us,
           algo_bytes / (us * 1e-6) / 1e9, n / us);
    fflush(stdout);
  };

  const double algo = (double)bytes + 6.0 * n;
  for (int grid : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, sizeof nm, "stream_read_grid%d", grid);
    time_it(nm, (double)bytes, [&](int r) {
      hipLaunchKernelGGL(stream_read, dim3(grid), dim3(256), 0, st, (const u32x4 *)arena[r],
                         bytes / 16, scratch);
    });
  }
  time_it("aos_window64", algo - 2.0 * n, [&](int r) {
    hipLaunchKernelGGL(aos_window, dim3((n + 255) / 256), dim3(256), 0, st, arena[r], off[r], n,
                       scratch);
  });
#define AOSAUX(AUX)                                                                           \
  time_it("aos_window64_aux" #AUX, algo - 2.0 * n, [&](int r) {                               \
    hipLaunchKernelGGL(aos_window_aux<AUX>, dim3((n + 255) / 256), dim3(256), 0, st, arena[r], \
                       off[r], n, scratch);                                                   \
  });
  AOSAUX(0) AOSAUX(1) AOSAUX(2) AOSAUX(3)
  time_it("aos_nodesc64", algo - 6.0 * n, [&](int r) {
    hipLaunchKernelGGL(aos_nodesc, dim3((n + 255) / 256), dim3(256), 0, st, arena[r], n, scratch);
  });
#define AOSLOOP(G)                                                                          \
  time_it("aos_loop64_grid" #G, algo - 2.0 * n, [&](int r) {                                \
    hipLaunchKernelGGL(aos_loop<G>, dim3(G), dim3(256), 0, st, arena[r], off[r], n, scratch); \
  });
  AOSLOOP(1024) AOSLOOP(2048) AOSLOOP(4096)
  time_it("lds_window64", algo - 2.0 * n, [&](int r) {
    hipLaunchKernelGGL(lds_window, dim3((n + 255) / 256), dim3(256), 0, st, arena[r], off[r], n,
                       scratch);
  });
  struct {
    const char *name;
    uint32_t flags;
    bool csum_out;
  } cases[] = {
      {"parse_only", CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_UDP, false},
      {"parse_csum", CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_UDP | CGPU_F_CSUM_IP | CGPU_F_CSUM_L4, true},
      {"parse_hash", CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_UDP | CGPU_F_FLOW_HASH, false},
      {"parse_csum_hash",
       CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_UDP | CGPU_F_CSUM_IP | CGPU_F_CSUM_L4 | CGPU_F_FLOW_HASH,
       true},
      {"parse_verify_hash",
       CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_UDP | CGPU_F_CSUM_IP | CGPU_F_CSUM_L4 | CGPU_F_FLOW_HASH,
       false},
  };
  for (auto &c : cases) {
    time_it(c.name, algo, [&](int r) {
      cgpu_batch b = {arena[r], bytes, off[r], len[r], n};
      cgpu_parse_out o = {meta, c.csum_out ? csum : nullptr, hash, nullptr, nullptr};
      if (cgpu_parse_batch(ctx, &b, c.flags, &o, st)) { fprintf(stderr, "parse\n"); exit(2); }
    });
  }
  {  // the bench config with consecutive launches alternating between 2 / 4
     // streams (independent bursts, as separate RX queues would submit them):
     // wall time per launch over the timed run
    const uint32_t fl = CGPU_F_ACCEPT_V4 | CGPU_F_ACCEPT_UDP | CGPU_F_CSUM_IP | CGPU_F_CSUM_L4 | CGPU_F_FLOW_HASH;
    for (int ns : {1, 2, 4}) {
      hipStream_t ss[4];
      uint32_t *m2[4];
      uint64_t *h2[4];
      for (int q = 0; q < ns; ++q) {
        CK(hipStreamCreateWithFlags(&ss[q], hipStreamNonBlocking));
        CK(hipMalloc(&m2[q], 4ull * n));
        CK(hipMalloc(&h2[q], 8ull * n));
      }
      auto go = [&](int k) {
        cgpu_batch b = {arena[k % R], bytes, off[k % R], len[k % R], n};
        cgpu_parse_out o = {m2[k % ns], nullptr, h2[k % ns], nullptr, nullptr};
        if (cgpu_parse_batch(ctx, &b, fl, &o, ss[k % ns])) { fprintf(stderr, "parse\n"); exit(2); }
      };
      for (int k = 0; k < 20; ++k) go(k);
      CK(hipDeviceSynchronize());
      auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; k < iters; ++k) go(k);
      CK(hipDeviceSynchronize());
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
      printf("{\"case\": \"parse_verify_hash_streams%d_wall\", \"us\": %.3f, \"GBps\": %.1f, \"Mpps\": %.1f}\n", ns, us,
             algo / (us * 1e-6) / 1e9, n / us);
      fflush(stdout);
      for (int q = 0; q < ns; ++q) {
        CK(hipStreamDestroy(ss[q]));
        CK(hipFree(m2[q]));
        CK(hipFree(h2[q]));
      }
    }
  }
  {  // nat64-shaped copies over 1M x 256-B frames (separate, larger arena)
    const uint32_t nf = n;
    uint8_t *fin[4], *fouts[4];
    for (int r = 0; r < 4; ++r) CK(hipMalloc(&fin[r], (size_t)nf * 256));
    for (int r = 0; r < 4; ++r) CK(hipMalloc(&fouts[r], (size_t)nf * 256));
    // outputs rotate like the inputs (one fixed 256 MiB output would stay in
    // the Infinity Cache and absorb the writes)
    uint8_t *fout = fouts[0];
    (void)fout;
    for (int r = 0; r < 4; ++r) CK(hipMemset(fin[r], r, (size_t)nf * 256));
    const double fb = (double)nf * (256 + 240);
    time_it("copy_frames_shift20_240B", fb, [&](int r) {
      hipLaunchKernelGGL(copy_frames<20>, dim3((nf + 63) / 64), dim3(256), 0, st, fin[r % 4], fouts[r % 4], nf, 240u);
    });
#define MAPCASE(G, IL, AUX)                                                                 \
  time_it("copy_map_G" #G "_IL" #IL "_aux" #AUX, (double)nf * 512, [&](int r) {               \
    hipLaunchKernelGGL((copy_map<G, IL, AUX>), dim3((nf * G + 255) / 256), dim3(256), 0, st,  \
                       fin[r % 4], fouts[r % 4], nf);                                                 \
  });
    MAPCASE(1, false, 0) MAPCASE(2, false, 0) MAPCASE(4, false, 0) MAPCASE(4, true, 0)
    MAPCASE(8, true, 0) MAPCASE(16, true, 0) MAPCASE(16, true, 2) MAPCASE(4, true, 2)
    MAPCASE(16, true, 1)
#define SHIFTCASE(G, AUX)                                                                   \
  time_it("copy_shift20_G" #G "_aux" #AUX, (double)nf * (256 + 236), [&](int r) {             \
    hipLaunchKernelGGL((copy_shift<G, AUX>), dim3((nf * G + 255) / 256), dim3(256), 0, st,    \
                       fin[r % 4], fouts[r % 4], nf);                                               \
  });
    SHIFTCASE(4, 0) SHIFTCASE(8, 0) SHIFTCASE(16, 0) SHIFTCASE(16, 2) SHIFTCASE(4, 2)
    time_it("copy_rows_dpp_236B_slots256", (double)nf * (256 + 236), [&](int r) {
      hipLaunchKernelGGL(copy_rows_dpp<256>, dim3((nf + 15) / 16), dim3(256), 0, st, fin[r % 4], fouts[r % 4], nf);
    });
    time_it("copy_rows_dpp_236B_packed", (double)nf * (256 + 236), [&](int r) {
      hipLaunchKernelGGL(copy_rows_dpp<236>, dim3((nf + 15) / 16), dim3(256), 0, st, fin[r % 4], fouts[r % 4], nf);
    });
    time_it("copy_frames_shift0_256B", (double)nf * 512, [&](int r) {
      hipLaunchKernelGGL(copy_frames<0>, dim3((nf + 63) / 64), dim3(256), 0, st, fin[r % 4], fouts[r % 4], nf, 256u);
    });
  }
  cgpu_ctx_destroy(ctx);
  return 0;
}
