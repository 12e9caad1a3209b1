// launch_gap.hip — what a kernel that finds nothing to do costs on the
// stream timeline, and what a per-call hipEventRecord costs, behind a real
// HBM-streaming kernel (the nat64 tail design question: how many "exit at
// once" launches may follow the fused kernel in the steady state).
//
// Per iteration: one streaming kernel (reads 256 MiB, ~45 us), then m empty
// kernels of g workgroups (each reads one flag word and returns), optionally
// a hipEventRecord.  Mean device time per iteration from events around 200
// back-to-back iterations, minus the m = 0 case.
//   build: hipcc -O3 --offload-arch=gfx950 tools/launch_gap.hip -o tools/launch_gap
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(2);                                                                \
    }                                                                         \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void stream(const u32x4 *p, size_t n16, uint32_t *out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256ull) {
    u32x4 v = p[i];
    acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;
}

// The same streams with the first and last wall-clock reading of each
// workgroup (100 MHz): the kernel's active span, to set against its share of
// the stream's timeline.
__global__ __launch_bounds__(256) void stream_clk(const u32x4 *p, size_t n16, uint32_t *out,
                                                  unsigned long long *clk) {
  const unsigned long long t0 = wall_clock64();
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256ull) {
    u32x4 v = p[i];
    acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t0;
    clk[2 * blockIdx.x + 1] = wall_clock64();
  }
}
__global__ __launch_bounds__(256) void write_clk(u32x4 *p, size_t n16, unsigned long long *clk) {
  const unsigned long long t0 = wall_clock64();
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256ull)
    p[i] = u32x4{(uint32_t)i, 1u, 2u, 3u};
  __syncthreads();
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t0;
    clk[2 * blockIdx.x + 1] = wall_clock64();
  }
}

// 64 B per lane (one frame in a 64-B slot): read it and write it back in
// place, or write it to another buffer (the reconcile kernel's store pattern
// against a copy's).
__global__ __launch_bounds__(256) void rmw64(u32x4 *p, u32x4 *q, size_t nframes) {
  const size_t f = blockIdx.x * 256ull + threadIdx.x;
  if (f >= nframes) return;
  u32x4 v[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] = p[4 * f + c];
  v[1][0] ^= 0x00010000u;  // change a field (a 2-B store's worth)
#pragma unroll
  for (int c = 0; c < 4; ++c) q[4 * f + c] = v[c];
}

__global__ __launch_bounds__(256) void empty(const uint32_t *flag, uint32_t *out) {
  if (*flag == 0u) return;  // the steady state: nothing deferred
  out[blockIdx.x * 256 + threadIdx.x] = 1u;
}

int main() {
  const size_t bytes = 256ull << 20;
  u32x4 *buf;
  uint32_t *flag, *out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMemset(buf, 1, bytes));
  CK(hipMalloc(&flag, 4));
  CK(hipMemset(flag, 0, 4));
  CK(hipMalloc(&out, 4 << 20));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b, rec;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventCreateWithFlags(&rec, hipEventDisableTiming));
  const int iters = 200;
  double base = 0;
  const int grids[] = {1, 64, 256, 1024};
  for (int ev = 0; ev < 2; ++ev) {
    for (int gi = 0; gi < 4; ++gi) {
      for (int m = 0; m <= 4; ++m) {
        if (m == 0 && gi > 0) continue;
        for (int rep = 0; rep < 2; ++rep) {  // rep 0 warms up
          CK(hipEventRecord(a, s));
          for (int it = 0; it < iters; ++it) {
            hipLaunchKernelGGL(stream, dim3(2048), dim3(256), 0, s, buf, bytes / 16, out);
            for (int k = 0; k < m; ++k)
              hipLaunchKernelGGL(empty, dim3(grids[gi]), dim3(256), 0, s, flag, out);
            if (ev) CK(hipEventRecord(rec, s));
          }
          CK(hipEventRecord(b, s));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          const double us = ms * 1e3 / iters;
          if (rep == 1) {
            if (m == 0 && ev == 0) base = us;
            printf("event_record=%d grid=%4d empty_kernels=%d  us/iter=%8.2f  extra=%7.2f\n", ev,
                   m ? grids[gi] : 0, m, us, us - base);
          }
        }
      }
    }
  }
  // the ways a call can leave a completion marker / order itself after the
  // previous call (the nat64 port map's cross-call ordering)
  hipEvent_t rec_t;
  CK(hipEventCreate(&rec_t));
  const char *names[] = {"ext_launch stop event (no timing flag)", "ext_launch stop event (timing)",
                         "event_record + wait_event same stream", "wait_event only (old event)",
                         "ext_launch stop event + wait on it next iter"};
  for (int mode = 0; mode < 5; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(a, s));
      for (int it = 0; it < iters; ++it) {
        if (mode == 4) CK(hipStreamWaitEvent(s, rec, 0));  // the previous iteration's, not yet complete
        if (mode == 0 || mode == 4)
          hipExtLaunchKernelGGL(stream, dim3(2048), dim3(256), 0, s, nullptr, rec, 0, buf, bytes / 16, out);
        else if (mode == 1)
          hipExtLaunchKernelGGL(stream, dim3(2048), dim3(256), 0, s, nullptr, rec_t, 0, buf, bytes / 16, out);
        else
          hipLaunchKernelGGL(stream, dim3(2048), dim3(256), 0, s, buf, bytes / 16, out);
        if (mode == 2) CK(hipEventRecord(rec, s));
        if (mode == 2 || mode == 3) CK(hipStreamWaitEvent(s, rec, 0));
      }
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      const double us = ms * 1e3 / iters;
      if (rep == 1) printf("%-42s us/iter=%8.2f  extra=%7.2f\n", names[mode], us, us - base);
    }
  }
  // a kernel's active span against its share of the stream (back to back):
  // reads only, and writes (whose dirty L2 lines the end-of-kernel release
  // writes back)
  {
    unsigned long long *clk, hclk[2 * 2048];
    CK(hipMalloc(&clk, sizeof(hclk)));
    for (int wr = 0; wr < 2; ++wr) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a, s));
        for (int it = 0; it < iters; ++it) {
          if (wr) hipLaunchKernelGGL(write_clk, dim3(2048), dim3(256), 0, s, buf, bytes / 16, clk);
          else hipLaunchKernelGGL(stream_clk, dim3(2048), dim3(256), 0, s, buf, bytes / 16, out, clk);
        }
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        CK(hipMemcpy(hclk, clk, sizeof(hclk), hipMemcpyDeviceToHost));
        unsigned long long lo = ~0ull, hi = 0;
        for (int k = 0; k < 2048; ++k) {
          lo = hclk[2 * k] < lo ? hclk[2 * k] : lo;
          hi = hclk[2 * k + 1] > hi ? hclk[2 * k + 1] : hi;
        }
        if (rep == 1)
          printf("%s 256 MiB: %.2f us per launch on the stream, last launch's workgroups active %.2f us\n",
                 wr ? "write" : "read ", ms * 1e3 / iters, (hi - lo) / 100.0);
      }
    }
    CK(hipFree(clk));
  }
  // 1 Mi 64-B frames: in place vs into another buffer, rotating over 4
  // copies (256 MiB, past the 256 MiB MALL with the second buffer)
  {
    const size_t nf = 1u << 20, fb = nf * 64;
    u32x4 *src, *dst;
    CK(hipMalloc(&src, 4 * fb));
    CK(hipMalloc(&dst, 4 * fb));
    CK(hipMemset(src, 3, 4 * fb));
    for (int mode = 0; mode < 2; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a, s));
        for (int it = 0; it < iters; ++it) {
          u32x4 *p = src + (it & 3) * (fb / 16);
          u32x4 *q = mode ? dst + (it & 3) * (fb / 16) : p;
          hipLaunchKernelGGL(rmw64, dim3(nf / 256), dim3(256), 0, s, p, q, nf);
        }
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep == 1)
          printf("1 Mi x 64 B, 64 B per lane, %s: %.2f us per launch (%.0f GB/s read + write)\n",
                 mode ? "into another buffer" : "in place", ms * 1e3 / iters, 2.0 * fb / (ms * 1e-3 / iters) / 1e9);
      }
    }
    CK(hipFree(src));
    CK(hipFree(dst));
  }
  // stream ids: are they reused after a destroy (the nat64 map's "same
  // stream as the previous call" test must not be fooled by a new stream
  // that got an old handle)?
  unsigned long long prev_id = 0;
  int handle_reuse = 0, id_reuse = 0;
  void *prev_h = nullptr;
  for (int k = 0; k < 64; ++k) {
    hipStream_t t;
    CK(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
    unsigned long long id;
    CK(hipStreamGetId(t, &id));
    if ((void *)t == prev_h) ++handle_reuse;
    if (k && id == prev_id) ++id_reuse;
    if (k < 4) printf("stream %p id %llu\n", (void *)t, id);
    prev_h = (void *)t;
    prev_id = id;
    CK(hipStreamDestroy(t));
  }
  unsigned long long id0;
  CK(hipStreamGetId(s, &id0));
  printf("64 create/destroy: handle reused %d times, id reused %d times; bench stream id %llu\n",
         handle_reuse, id_reuse, id0);
  return 0;
}
