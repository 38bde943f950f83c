// hbm_probe.hip — measured HBM read-stream peak for the bench's roofline ("also report a
// measured read-stream peak"): non-temporal 16-B loads over R buffers of 512 MiB cycled per launch
// (cold: nothing left in the 256 MiB Infinity Cache), two tile shapes, best reported. Not part of
// libmpjx: a measurement helper bench.py loads from tools/libhbm_probe.so.
//   extern "C" double hbm_read_peak_GBps(int launches)   (< 0 on a HIP error)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

using v4u = unsigned int __attribute__((ext_vector_type(4)));

template <int TH, int U>
__global__ __launch_bounds__(TH) void k_read(const v4u* p, long nv, unsigned* sink) {
  const long base = (long)blockIdx.x * TH * U;
  unsigned x = 0;
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * TH + threadIdx.x;
    if (i < nv) {
      const v4u v = __builtin_nontemporal_load(p + i);
      x ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
  }
  if (x == 0x9E3779B9u && threadIdx.x == 0) sink[0] = x;  // keeps the loads; practically never true
}

template <int TH, int U>
static double run(const std::vector<v4u*>& bufs, long nv, unsigned* sink, int launches, hipStream_t s) {
  const unsigned g = (unsigned)((nv + (long)TH * U - 1) / ((long)TH * U));
  const int R = (int)bufs.size();
  for (int i = 0; i < R; i++) k_read<TH, U><<<g, TH, 0, s>>>(bufs[i], nv, sink);
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -1;
  (void)hipEventRecord(e0, s);
  for (int i = 0; i < launches; i++) k_read<TH, U><<<g, TH, 0, s>>>(bufs[i % R], nv, sink);
  (void)hipEventRecord(e1, s);
  if (hipStreamSynchronize(s) != hipSuccess) return -1;
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return (double)nv * 16 * launches / (ms * 1e-3) / 1e9;
}

extern "C" double hbm_read_peak_GBps(int launches) {
  const long bytes = 512L << 20, nv = bytes / 16;
  const int R = 4;
  std::vector<v4u*> bufs(R, nullptr);
  unsigned* sink = nullptr;
  hipStream_t s = nullptr;
  double best = -1;
  bool ok = hipStreamCreate(&s) == hipSuccess && hipMalloc(&sink, 16) == hipSuccess;
  for (int i = 0; ok && i < R; i++) ok = hipMalloc(&bufs[i], bytes) == hipSuccess && hipMemset(bufs[i], 1, bytes) == hipSuccess;
  if (ok) {
    best = std::max(run<1024, 1>(bufs, nv, sink, launches, s), run<256, 4>(bufs, nv, sink, launches, s));
    best = std::max(best, run<512, 2>(bufs, nv, sink, launches, s));
  }
  for (auto* b : bufs)
    if (b) (void)hipFree(b);
  if (sink) (void)hipFree(sink);
  if (s) (void)hipStreamDestroy(s);
  return ok ? best : -1;
}
