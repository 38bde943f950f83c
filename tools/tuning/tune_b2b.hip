// tune_b2b.hip — sustained (back-to-back) rate of combine-kernel variants, 2 x 256 MiB double SUM.
// Each variant runs 20 launches back to back with events around each (as bench.py does); variants
// are interleaved over rounds. Also tests the HBM placement hypothesis: `in` skewed against `inout`.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune_b2b.hip -o tools/tune_b2b
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

using v4u = unsigned int __attribute__((ext_vector_type(4)));
using d2 = double __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v4u add(v4u a, v4u b) {
  d2 x, y;
  __builtin_memcpy(&x, &a, 16);
  __builtin_memcpy(&y, &b, 16);
  x = x + y;
  v4u r;
  __builtin_memcpy(&r, &x, 16);
  return r;
}

// T threads, U loads per operand per lane, TPB tiles per block (software-pipelined when > 1)
template <int T, int U, int TPB, bool INTERLEAVE>
__global__ __launch_bounds__(T) void k(v4u* io, const v4u* in, long nv) {
  const long tile = (long)T * U;
  long base = (long)blockIdx.x * tile * TPB;
#pragma unroll
  for (int t = 0; t < TPB; t++, base += tile) {
    if (base >= nv) return;
    v4u a[U], b[U];
    if (INTERLEAVE) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        long i = base + u * T + threadIdx.x;
        a[u] = __builtin_nontemporal_load(in + i);
        b[u] = __builtin_nontemporal_load(io + i);
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) a[u] = __builtin_nontemporal_load(in + base + u * T + threadIdx.x);
#pragma unroll
      for (int u = 0; u < U; u++) b[u] = __builtin_nontemporal_load(io + base + u * T + threadIdx.x);
    }
#pragma unroll
    for (int u = 0; u < U; u++) __builtin_nontemporal_store(add(a[u], b[u]), io + base + u * T + threadIdx.x);
  }
}

__global__ void k_fill(unsigned long long* p, long n, unsigned long long seed) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (i + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    p[i] = __double_as_longlong((double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0);
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 5;
  const long n = 256L * (1 << 20) / 8, nv = n / 2;
  const double S = n * 8.0;
  char* big;
  const size_t skew_max = 64 << 20;
  CK(hipMalloc(&big, 2 * n * 8 + skew_max + 4096));
  v4u* io = (v4u*)big;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  struct Var { std::string name; std::function<void(hipStream_t)> f; std::vector<double> us; };
  std::vector<Var> V;
  auto in_at = [&](size_t skew) { return (const v4u*)(big + n * 8 + skew); };
  auto grid = [&](int T, int U, int TPB) { return (unsigned)((nv + (long)T * U * TPB - 1) / ((long)T * U * TPB)); };
  for (size_t skew : {(size_t)0, (size_t)4096, (size_t)65536, (size_t)(1 << 20) + 4096, (size_t)(32 << 20) + 8192}) {
    const v4u* in = in_at(skew);
    V.push_back({"U4 T256 skew " + std::to_string(skew), [=](hipStream_t st) { k<256, 4, 1, false><<<grid(256, 4, 1), 256, 0, st>>>(io, in, nv); }, {}});
  }
  const v4u* in0 = in_at(4096);
  V.push_back({"U4 T256 interleave", [=](hipStream_t st) { k<256, 4, 1, true><<<grid(256, 4, 1), 256, 0, st>>>(io, in0, nv); }, {}});
  V.push_back({"U8 T256", [=](hipStream_t st) { k<256, 8, 1, false><<<grid(256, 8, 1), 256, 0, st>>>(io, in0, nv); }, {}});
  V.push_back({"U2 T256", [=](hipStream_t st) { k<256, 2, 1, false><<<grid(256, 2, 1), 256, 0, st>>>(io, in0, nv); }, {}});
  V.push_back({"U4 T256 TPB2", [=](hipStream_t st) { k<256, 4, 2, false><<<grid(256, 4, 2), 256, 0, st>>>(io, in0, nv); }, {}});
  V.push_back({"U4 T256 TPB4", [=](hipStream_t st) { k<256, 4, 4, false><<<grid(256, 4, 4), 256, 0, st>>>(io, in0, nv); }, {}});
  V.push_back({"U2 T512", [=](hipStream_t st) { k<512, 2, 1, false><<<grid(512, 2, 1), 512, 0, st>>>(io, in0, nv); }, {}});
  V.push_back({"U4 T512", [=](hipStream_t st) { k<512, 4, 1, false><<<grid(512, 4, 1), 512, 0, st>>>(io, in0, nv); }, {}});
  V.push_back({"U1 T1024", [=](hipStream_t st) { k<1024, 1, 1, false><<<grid(1024, 1, 1), 1024, 0, st>>>(io, in0, nv); }, {}});
  k_fill<<<4096, 256>>>((unsigned long long*)big, (2 * n * 8 + skew_max) / 8, 7);
  CK(hipDeviceSynchronize());
  const int K = 20;
  std::vector<hipEvent_t> e0(K), e1(K);
  for (int i = 0; i < K; i++) { CK(hipEventCreate(&e0[i])); CK(hipEventCreate(&e1[i])); }
  for (int r = 0; r < rounds; r++)
    for (auto& v : V) {
      for (int w = 0; w < 3; w++) v.f(s);
      for (int i = 0; i < K; i++) { CK(hipEventRecord(e0[i], s)); v.f(s); CK(hipEventRecord(e1[i], s)); }
      CK(hipStreamSynchronize(s));
      double tot = 0;
      for (int i = 0; i < K; i++) { float ms; CK(hipEventElapsedTime(&ms, e0[i], e1[i])); tot += ms; }
      v.us.push_back(tot / K * 1e3);
    }
  printf("%-34s %9s %9s %9s\n", "variant (b2b x20)", "med_us", "min_us", "GB/s");
  for (auto& v : V) {
    std::sort(v.us.begin(), v.us.end());
    double med = v.us[v.us.size() / 2];
    printf("%-34s %9.1f %9.1f %9.1f\n", v.name.c_str(), med, v.us[0], 3 * S / (med * 1e-6) / 1e9);
  }
}
