// tune_policy3.hip — the library's own k_pway (csrc/mpjx_kernels.hpp) against tune_policy's simple
// kernel on the same in-place 2 x 256 MiB double SUM buffers: why did POL 2 (accumulator
// non-temporal, other operand default policy) measure 141.6 us inside bench.py while the simple
// kernel with that policy measured 110.4 us? Sustained: 20 launches between one event pair,
// variants interleaved over rounds.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/tune_policy3.hip -o tools/tune_policy3
#include "../mpjexpress_amd/csrc/mpjx_kernels.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

namespace mpjx {
size_t nt_min_bytes() { return kNonTemporalBytes; }
bool inplace_policy_on() { return true; }
}  // namespace mpjx

using mpjx::v4u;
using d2 = double __attribute__((ext_vector_type(2)));

template <bool NTIN>
__global__ __launch_bounds__(256) void k_simple(v4u* io, const v4u* in, long nv) {
  constexpr int U = 4, T = 256;
  const long base = (long)blockIdx.x * T * U;
  v4u a[U], b[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < nv) {
      b[u] = __builtin_nontemporal_load(io + i);
      a[u] = NTIN ? __builtin_nontemporal_load(in + i) : in[i];
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < nv) {
      d2 x, y;
      __builtin_memcpy(&x, &a[u], 16);
      __builtin_memcpy(&y, &b[u], 16);
      x = x + y;
      v4u r;
      __builtin_memcpy(&r, &x, 16);
      __builtin_nontemporal_store(r, io + i);
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
  k_fill<<<4096, 256>>>((unsigned long long*)io, n, 7);
  k_fill<<<4096, 256>>>((unsigned long long*)in, n, 9);
  CK(hipDeviceSynchronize());
  hipStream_t s;
  CK(hipStreamCreate(&s));
  mpjx::PwayArgs a{};
  a.in[0] = io;  // acc (arr[i]) — the in-place combine, as mpjx_combine passes it
  a.in[1] = in;
  a.out[0] = io;
  a.n = n;
  const unsigned grid = (unsigned)((nv + 1023) / 1024);
  struct Var { std::string name; std::function<void(hipStream_t)> f; std::vector<double> us; };
  std::vector<Var> V;
  using F = mpjx::Sum<double>;
  V.push_back({"k_pway POL1 (all NT)", [=](hipStream_t st) { mpjx::launch_one<F, 2, mpjx::K_FOLD, 2, 1>(a, st); }, {}});
  V.push_back({"k_pway POL2 (acc NT, in default)", [=](hipStream_t st) { mpjx::launch_one<F, 2, mpjx::K_FOLD, 2, 2>(a, st); }, {}});
  V.push_back({"simple all NT", [=](hipStream_t st) { k_simple<true><<<grid, 256, 0, st>>>(io, in, nv); }, {}});
  V.push_back({"simple acc NT, in default", [=](hipStream_t st) { k_simple<false><<<grid, 256, 0, st>>>(io, in, nv); }, {}});
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
  for (auto& v : V) {
    std::sort(v.us.begin(), v.us.end());
    const double med = v.us[v.us.size() / 2];
    printf("%-36s %9.1f %9.1f %9.1f %7.3f\n", v.name.c_str(), med, v.us[0], 3 * S / (med * 1e-6) / 1e9,
           3 * S / (med * 1e-6) / 8e12);
  }
}
