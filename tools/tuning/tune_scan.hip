// tune_scan.hip — the write-heavy Scan kernel (P inputs, P outputs: out[r] = in[r-1] + (... + (in[0] +
// in[r])), double SUM) under load/store policy and unroll variants; slices contiguous in one pool
// (as the exchange slots are). 20 back-to-back launches between one event pair, interleaved rounds.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune_scan.hip -o tools/tune_scan
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

struct Args {
  const v4u* in[8];
  v4u* out[8];
  long nv;
};

template <bool NT>
__device__ __forceinline__ v4u ld(const v4u* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(v4u* p, v4u v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <bool NT, int P, int... Is>
__device__ __forceinline__ void load_all(v4u (&x)[P], const Args& a, long i, std::integer_sequence<int, Is...>) {
  ((x[Is] = ld<NT>(a.in[Is] + i)), ...);
}

template <int P, bool NTL, bool NTS, int U>
__global__ __launch_bounds__(256) void k(Args a) {
  constexpr int T = 256;
  const long base = (long)blockIdx.x * T * U;
  v4u x[U][P];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < a.nv) load_all<NTL>(x[u], a, i, std::make_integer_sequence<int, P>{});
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < a.nv) {
#pragma unroll
      for (int r = 0; r < P; r++) {
        d2 acc;
        __builtin_memcpy(&acc, &x[u][r], 16);
#pragma unroll
        for (int j = 0; j < r; j++) {
          d2 v;
          __builtin_memcpy(&v, &x[u][j], 16);
          acc = v + acc;
        }
        v4u o;
        __builtin_memcpy(&o, &acc, 16);
        st<NTS>(a.out[r] + i, o);
      }
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

struct Var {
  std::string name;
  std::function<void(hipStream_t)> f;
  double bytes;
  std::vector<double> us;
};

template <int P, bool NTL, bool NTS, int U>
static Var make(long mib, Args a) {
  const unsigned grid = (unsigned)((a.nv + 256L * U - 1) / (256L * U));
  char name[96];
  snprintf(name, sizeof name, "SCAN P=%d %3ldMiB ld %-5s st %-5s U%d", P, mib, NTL ? "NT" : "plain",
           NTS ? "NT" : "plain", U);
  return {name, [=](hipStream_t st) { k<P, NTL, NTS, U><<<grid, 256, 0, st>>>(a); }, 2.0 * P * a.nv * 16, {}};
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 5;
  const size_t cap = 16L * (256L << 20);
  char* pool;
  CK(hipMalloc(&pool, cap));
  k_fill<<<4096, 256>>>((unsigned long long*)pool, (long)(cap / 8), 5);
  CK(hipDeviceSynchronize());
  auto args = [&](int P, long slice) {
    Args a{};
    for (int p = 0; p < P; p++) {
      a.in[p] = (const v4u*)(pool + p * slice);
      a.out[p] = (v4u*)(pool + (P + p) * slice);
    }
    a.nv = slice / 16;
    return a;
  };
  std::vector<Var> V;
  for (long mib : {8L, 32L, 256L}) {
    const long sl = mib << 20;
    Args a2 = args(2, sl), a8 = args(8, sl);
    V.push_back(make<2, true, true, 4>(mib, a2));
    V.push_back(make<2, false, false, 4>(mib, a2));
    V.push_back(make<2, false, true, 4>(mib, a2));
    V.push_back(make<2, true, false, 4>(mib, a2));
    V.push_back(make<2, false, true, 2>(mib, a2));
    V.push_back(make<8, true, true, 1>(mib, a8));
    V.push_back(make<8, false, false, 1>(mib, a8));
    V.push_back(make<8, false, true, 1>(mib, a8));
    V.push_back(make<8, true, false, 1>(mib, a8));
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
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
  printf("%-44s %9s %9s %9s %7s\n", "variant (20 b2b launches, 1 event pair)", "med_us", "min_us", "GB/s", "frac");
  for (auto& v : V) {
    std::sort(v.us.begin(), v.us.end());
    const double med = v.us[v.us.size() / 2];
    printf("%-44s %9.1f %9.1f %9.1f %7.3f\n", v.name.c_str(), med, v.us[0], v.bytes / (med * 1e-6) / 1e9,
           v.bytes / (med * 1e-6) / 8e12);
  }
}
