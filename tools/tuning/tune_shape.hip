// tune_shape.hip — tile shape, load order and block->tile mapping of the in-place combine under the
// round-2 policy (accumulator non-temporal, other operand default policy, non-temporal stores);
// 2 x 256 MiB double SUM, 20 back-to-back launches between one event pair, interleaved rounds.
// XCD: consecutive workgroups are dispatched round-robin over the 8 XCDs; the remap gives each XCD
// one contiguous eighth of the vector instead of every 8th tile.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune_shape.hip -o tools/tune_shape
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

template <int T, int U, bool IN_FIRST, bool XCD>
__global__ __launch_bounds__(T) void k(v4u* io, const v4u* in, long nv) {
  long b = blockIdx.x;
  if (XCD) {  // gridDim.x is a multiple of 8 here
    const long per = gridDim.x / 8;
    b = (b % 8) * per + b / 8;
  }
  const long base = b * T * U;
  v4u a[U], c[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < nv) {
      if (IN_FIRST) {
        a[u] = in[i];
        c[u] = __builtin_nontemporal_load(io + i);
      } else {
        c[u] = __builtin_nontemporal_load(io + i);
        a[u] = in[i];
      }
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < nv) {
      d2 x, y;
      __builtin_memcpy(&x, &a[u], 16);
      __builtin_memcpy(&y, &c[u], 16);
      x = x + y;
      v4u r;
      __builtin_memcpy(&r, &x, 16);
      __builtin_nontemporal_store(r, io + i);
    }
  }
}

// copy dst = src with default-policy loads and non-temporal stores (k_copies' large-copy policy)
template <int T, int U>
__global__ __launch_bounds__(T) void kc(v4u* dst, const v4u* src, long nv) {
  const long base = (long)blockIdx.x * T * U;
  v4u a[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < nv) a[u] = src[i];
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < nv) __builtin_nontemporal_store(a[u], dst + i);
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
  k_fill<<<4096, 256>>>((unsigned long long*)io, n, 7);
  k_fill<<<4096, 256>>>((unsigned long long*)in, n, 9);
  CK(hipDeviceSynchronize());
  hipStream_t s;
  CK(hipStreamCreate(&s));
  struct Var { std::string name; std::function<void(hipStream_t)> f; std::vector<double> us; };
  std::vector<Var> V;
  auto grid = [&](int T, int U) { return (unsigned)((nv + (long)T * U - 1) / ((long)T * U)); };
#define VAR(T, U, INF, X) V.push_back({std::string("T" #T " U" #U) + (INF ? " in-first" : " acc-first") + (X ? " xcd" : ""), \
      [=](hipStream_t st) { k<T, U, INF, X><<<grid(T, U), T, 0, st>>>(io, in, nv); }, {}})
  VAR(256, 4, false, false);  // shipped
  VAR(256, 4, true, false);
  VAR(256, 4, false, true);
  VAR(256, 2, false, false);
  VAR(256, 8, false, false);
  VAR(512, 2, false, false);
  VAR(512, 4, false, false);
  VAR(128, 8, false, false);
  VAR(1024, 1, false, false);
  VAR(64, 16, false, false);
  const size_t nc = V.size();  // copies below: 2 S of traffic
#define CVAR(T, U) V.push_back({std::string("copy T" #T " U" #U), \
      [=](hipStream_t st) { kc<T, U><<<grid(T, U), T, 0, st>>>(io, in, nv); }, {}})
  CVAR(256, 4);  // shipped
  CVAR(256, 2);
  CVAR(256, 8);
  CVAR(512, 2);
  CVAR(1024, 1);
  CVAR(512, 4);
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
