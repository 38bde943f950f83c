// tune_policy.hip — cache-policy variants of the configs[1] combine (2 x 256 MiB double SUM,
// inout = in + inout), sustained back to back: 20 launches between one event pair (bench.py's
// method), variants interleaved over rounds, median reported. Question it answers: the mpjbuf
// combine (NT loads of acc, plain 8-B loads of the payload, NT stores) ran 114.7 us against 121-123
// for k_pway (NT loads of both operands, NT stores) — is it the load policy of one stream?
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune_policy.hip -o tools/tune_policy
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

enum Pol { PLAIN = 0, NT = 1, HALVES = 2 };  // HALVES: two plain 8-B loads

template <int P>
__device__ __forceinline__ v4u ld(const v4u* p) {
  if constexpr (P == NT) {
    return __builtin_nontemporal_load(p);
  } else if constexpr (P == HALVES) {
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
    unsigned long long lo = q[0], hi = q[1];
    v4u v;
    __builtin_memcpy(&v, &lo, 8);
    __builtin_memcpy(reinterpret_cast<char*>(&v) + 8, &hi, 8);
    return v;
  } else {
    return *p;
  }
}

// U = 4 loads per operand per lane, 256 threads, one tile per block (the shipped k_pway shape)
template <int PIO, int PIN, bool NTST>
__global__ __launch_bounds__(256) void k(v4u* io, const v4u* in, long nv) {
  constexpr int U = 4, T = 256;
  const long base = (long)blockIdx.x * T * U;
  v4u a[U], b[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < nv) {
      b[u] = ld<PIO>(io + i);
      a[u] = ld<PIN>(in + i);
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < nv) {
      if (NTST) __builtin_nontemporal_store(add(a[u], b[u]), io + i);
      else io[i] = add(a[u], b[u]);
    }
  }
}

// copy dst = src, 256 MiB (Reduce's arraycopy at P = 1, the IPC push)
template <int PS, bool NTST>
__global__ __launch_bounds__(256) void kc(v4u* dst, const v4u* src, long nv) {
  constexpr int U = 4, T = 256;
  const long base = (long)blockIdx.x * T * U;
  v4u a[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < nv) a[u] = ld<PS>(src + i);
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < nv) {
      if (NTST) __builtin_nontemporal_store(a[u], dst + i);
      else dst[i] = a[u];
    }
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
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  const long n = 256L * (1 << 20) / 8, nv = n / 2;
  const double S = n * 8.0;
  v4u *io, *in;
  CK(hipMalloc(&io, n * 8));
  CK(hipMalloc(&in, n * 8));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  struct Var { std::string name; std::function<void(hipStream_t)> f; std::vector<double> us; };
  std::vector<Var> V;
  const unsigned grid = (unsigned)((nv + 1023) / 1024);
#define VAR(name, a, b, c) V.push_back({name, [=](hipStream_t st) { k<a, b, c><<<grid, 256, 0, st>>>(io, in, nv); }, {}})
  VAR("io NT   in NT     st NT (shipped)", NT, NT, true);
  VAR("io NT   in plain  st NT", NT, PLAIN, true);
  VAR("io NT   in halves st NT (mpjbuf)", NT, HALVES, true);
  VAR("io plain in NT    st NT", PLAIN, NT, true);
  VAR("io plain in plain st NT", PLAIN, PLAIN, true);
  VAR("io NT   in NT     st plain", NT, NT, false);
  VAR("io plain in plain st plain", PLAIN, PLAIN, false);
  VAR("io halves in halves st NT", HALVES, HALVES, true);
  const size_t nc = V.size();  // copies below: 2 S of traffic
#define CVAR(name, a, c) V.push_back({name, [=](hipStream_t st) { kc<a, c><<<grid, 256, 0, st>>>(io, in, nv); }, {}})
  CVAR("copy ld NT    st NT (shipped)", NT, true);
  CVAR("copy ld plain st NT", PLAIN, true);
  CVAR("copy ld NT    st plain", NT, false);
  CVAR("copy ld plain st plain", PLAIN, false);
  k_fill<<<4096, 256>>>((unsigned long long*)io, n, 7);
  k_fill<<<4096, 256>>>((unsigned long long*)in, n, 9);
  CK(hipDeviceSynchronize());
  const int K = 20;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; r++)
    for (auto& v : V) {
      for (int w = 0; w < 3; w++) v.f(s);
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < K; i++) v.f(s);
      CK(hipEventRecord(e1, s));
      CK(hipStreamSynchronize(s));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms / K * 1e3);
    }
  printf("%-36s %9s %9s %9s %7s\n", "variant (20 b2b launches, 1 event pair)", "med_us", "min_us", "GB/s", "frac");
  for (size_t k = 0; k < V.size(); k++) {
    auto& v = V[k];
    std::sort(v.us.begin(), v.us.end());
    const double med = v.us[v.us.size() / 2];
    const double bytes = (k < nc ? 3 : 2) * S;
    printf("%-36s %9.1f %9.1f %9.1f %7.3f\n", v.name.c_str(), med, v.us[0], bytes / (med * 1e-6) / 1e9,
           bytes / (med * 1e-6) / 8e12);
  }
}
