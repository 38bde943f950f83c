// tune_combine.hip — A/B harness for the streaming structure of the combine kernel (SUM double,
// inout = in + inout, 2 x 256 MiB) plus copy / read-only reference streams that give this box's
// achievable HBM rates. Variants are timed interleaved in one process (hipEvents, median of rounds).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune_combine.hip -o tools/tune_combine \
//          -Lmpjexpress_amd/lib -lmpjx -Wl,-rpath,\$ORIGIN/../mpjexpress_amd/lib
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

extern "C" int mpjx_combine(int op, int type, void* inout, const void* in, long count, void* stream);

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

using v4u = unsigned int __attribute__((ext_vector_type(4)));
using d2 = double __attribute__((ext_vector_type(2)));

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
__device__ __forceinline__ v4u add(v4u a, v4u b) {
  d2 x, y;
  __builtin_memcpy(&x, &a, 16);
  __builtin_memcpy(&y, &b, 16);
  x = x + y;
  v4u r;
  __builtin_memcpy(&r, &x, 16);
  return r;
}

// A: grid-stride, U in flight per lane, strided by the whole grid (current library structure)
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_gs(v4u* io, const v4u* in, long nv) {
  long stride = (long)gridDim.x * blockDim.x;
  for (long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x; i0 < nv; i0 += stride * U) {
    v4u a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      long i = i0 + u * stride;
      if (i < nv) { a[u] = ld<NTL>(in + i); b[u] = ld<NTL>(io + i); }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      long i = i0 + u * stride;
      if (i < nv) st<NTS>(io + i, add(a[u], b[u]));
    }
  }
}

// B: block-tiled: a block owns tiles of 256*U consecutive vectors (U loads per lane 256 apart),
// tiles grid-strided
template <int U, bool NTL, bool NTS, int T = 256>
__global__ __launch_bounds__(T) void k_tile(v4u* io, const v4u* in, long nv) {
  const long tile = (long)T * U;
  for (long base = (long)blockIdx.x * tile; base < nv; base += (long)gridDim.x * tile) {
    v4u a[U], b[U];
    if (base + tile <= nv) {
#pragma unroll
      for (int u = 0; u < U; u++) { long i = base + u * T + threadIdx.x; a[u] = ld<NTL>(in + i); b[u] = ld<NTL>(io + i); }
#pragma unroll
      for (int u = 0; u < U; u++) { long i = base + u * T + threadIdx.x; st<NTS>(io + i, add(a[u], b[u])); }
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) { long i = base + u * T + threadIdx.x; if (i < nv) { a[u] = ld<NTL>(in + i); b[u] = ld<NTL>(io + i); } }
#pragma unroll
      for (int u = 0; u < U; u++) { long i = base + u * T + threadIdx.x; if (i < nv) st<NTS>(io + i, add(a[u], b[u])); }
    }
  }
}

// C: contiguous chunk per block (each block streams nv/grid consecutive vectors)
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_chunk(v4u* io, const v4u* in, long nv) {
  long per = (nv + gridDim.x - 1) / gridDim.x;
  per = (per + 256 * U - 1) / (256 * U) * (256 * U);
  long beg = (long)blockIdx.x * per, end = std::min(nv, beg + per);
  for (long base = beg; base < end; base += 256 * U) {
    v4u a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) { long i = base + u * 256 + threadIdx.x; if (i < end) { a[u] = ld<NTL>(in + i); b[u] = ld<NTL>(io + i); } }
#pragma unroll
    for (int u = 0; u < U; u++) { long i = base + u * 256 + threadIdx.x; if (i < end) st<NTS>(io + i, add(a[u], b[u])); }
  }
}

// references: copy (1R+1W) and read-only (1R, reduced so it is not dead)
template <int U>
__global__ __launch_bounds__(256) void k_copy(v4u* dst, const v4u* src, long nv) {
  const long tile = 256L * U;
  for (long base = (long)blockIdx.x * tile; base < nv; base += (long)gridDim.x * tile) {
    v4u a[U];
#pragma unroll
    for (int u = 0; u < U; u++) { long i = base + u * 256 + threadIdx.x; if (i < nv) a[u] = src[i]; }
#pragma unroll
    for (int u = 0; u < U; u++) { long i = base + u * 256 + threadIdx.x; if (i < nv) dst[i] = a[u]; }
  }
}
template <int U>
__global__ __launch_bounds__(256) void k_read(const v4u* src, long nv, unsigned* sink) {
  const long tile = 256L * U;
  v4u acc = {0, 0, 0, 0};
  for (long base = (long)blockIdx.x * tile; base < nv; base += (long)gridDim.x * tile) {
#pragma unroll
    for (int u = 0; u < U; u++) { long i = base + u * 256 + threadIdx.x; if (i < nv) acc ^= src[i]; }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345679u) sink[0] = 1;
}

__global__ void k_fill(unsigned long long* p, long n, unsigned long long seed) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (i + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    double d = (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
    p[i] = __double_as_longlong(d);
  }
}
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_read_nt(const v4u* src, long nv, unsigned* sink) {
  const long tile = 256L * U;
  v4u acc = {0, 0, 0, 0};
  for (long base = (long)blockIdx.x * tile; base < nv; base += (long)gridDim.x * tile) {
#pragma unroll
    for (int u = 0; u < U; u++) { long i = base + u * 256 + threadIdx.x; if (i < nv) acc ^= ld<NT>(src + i); }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345679u) sink[0] = 1;
}

struct Var {
  std::string name;
  double bytes;
  std::function<void(hipStream_t)> run;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  long mib = argc > 1 ? atol(argv[1]) : 256;
  int rounds = argc > 2 ? atoi(argv[2]) : 15;
  long n = mib * (1L << 20) / 8, nv = n / 2;
  double S = n * 8.0;
  v4u *io, *in, *dst;
  unsigned* sink;
  CK(hipMalloc(&io, n * 8));
  CK(hipMalloc(&in, n * 8));
  CK(hipMalloc(&dst, n * 8));
  CK(hipMalloc(&sink, 4));
  k_fill<<<4096, 256>>>((unsigned long long*)io, n, 1);
  k_fill<<<4096, 256>>>((unsigned long long*)in, n, 2);
  CK(hipDeviceSynchronize());
  hipStream_t s;
  CK(hipStreamCreate(&s));
  std::vector<Var> V;
  auto add_var = [&](std::string nm, double bytes, std::function<void(hipStream_t)> f) { V.push_back({nm, bytes, f, {}}); };
  auto gridf = [&](int U, int per_cu) { long g = (nv + 256L * U - 1) / (256L * U); return (unsigned)std::min<long>(g, 256L * per_cu); };
  auto full = [&](int U) { return (unsigned)((nv + 256L * U - 1) / (256L * U)); };

  add_var("gs U4 g2048 (lib)", 3 * S, [&](hipStream_t st) { k_gs<4, false, false><<<2048, 256, 0, st>>>(io, in, nv); });
  add_var("gs U4 g2048 NTL", 3 * S, [&](hipStream_t st) { k_gs<4, true, false><<<2048, 256, 0, st>>>(io, in, nv); });
  add_var("tile U4 full", 3 * S, [&](hipStream_t st) { k_tile<4, false, false><<<full(4), 256, 0, st>>>(io, in, nv); });
  add_var("tile U1 full NTL", 3 * S, [&](hipStream_t st) { k_tile<1, true, false><<<full(1), 256, 0, st>>>(io, in, nv); });
  add_var("tile U2 full NTL", 3 * S, [&](hipStream_t st) { k_tile<2, true, false><<<full(2), 256, 0, st>>>(io, in, nv); });
  add_var("tile U4 full NTL", 3 * S, [&](hipStream_t st) { k_tile<4, true, false><<<full(4), 256, 0, st>>>(io, in, nv); });
  add_var("tile U8 full NTL", 3 * S, [&](hipStream_t st) { k_tile<8, true, false><<<full(8), 256, 0, st>>>(io, in, nv); });
  for (int pc : {4, 8, 16, 32})
    add_var("tile U4 NTL " + std::to_string(pc) + "/CU", 3 * S, [&, pc](hipStream_t st) { k_tile<4, true, false><<<gridf(4, pc), 256, 0, st>>>(io, in, nv); });
  for (int pc : {8, 16})
    add_var("tile U2 NTL " + std::to_string(pc) + "/CU", 3 * S, [&, pc](hipStream_t st) { k_tile<2, true, false><<<gridf(2, pc), 256, 0, st>>>(io, in, nv); });
  add_var("tile U4 full NTL+NTS", 3 * S, [&](hipStream_t st) { k_tile<4, true, true><<<full(4), 256, 0, st>>>(io, in, nv); });
  add_var("tile U4 T512 full NTL", 3 * S, [&](hipStream_t st) { k_tile<4, true, false, 512><<<(unsigned)((nv + 2047) / 2048), 512, 0, st>>>(io, in, nv); });
  add_var("tile U2 T1024 full NTL", 3 * S, [&](hipStream_t st) { k_tile<2, true, false, 1024><<<(unsigned)((nv + 2047) / 2048), 1024, 0, st>>>(io, in, nv); });
  add_var("chunk U4 2048 NTL", 3 * S, [&](hipStream_t st) { k_chunk<4, true, false><<<2048, 256, 0, st>>>(io, in, nv); });
  add_var("read U8 2048 (ref)", 1 * S, [&](hipStream_t st) { k_read<8><<<2048, 256, 0, st>>>(in, nv, sink); });
  add_var("read NT U8 2048 (ref)", 1 * S, [&](hipStream_t st) { k_read_nt<8, true><<<2048, 256, 0, st>>>(in, nv, sink); });
  add_var("read NT U4 full (ref)", 1 * S, [&](hipStream_t st) { k_read_nt<4, true><<<full(4), 256, 0, st>>>(in, nv, sink); });
  add_var("read NT U8 4096 (ref)", 1 * S, [&](hipStream_t st) { k_read_nt<8, true><<<4096, 256, 0, st>>>(in, nv, sink); });
  add_var("hipMemcpyDtoD (ref)", 2 * S, [&](hipStream_t st) { CK(hipMemcpyAsync(dst, in, n * 8, hipMemcpyDeviceToDevice, st)); });

  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (auto& v : V) v.run(s);  // warm
  CK(hipStreamSynchronize(s));
  for (int r = 0; r < rounds; r++) {
    for (auto& v : V) {
      CK(hipEventRecord(a, s));
      v.run(s);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      v.ms.push_back(ms);
    }
  }
  printf("%-26s %10s %10s %10s\n", "variant", "med_us", "min_us", "GB/s(med)");
  for (auto& v : V) {
    std::sort(v.ms.begin(), v.ms.end());
    double med = v.ms[v.ms.size() / 2] * 1e-3, mn = v.ms[0] * 1e-3;
    printf("%-26s %10.1f %10.1f %10.1f\n", v.name.c_str(), med * 1e6, mn * 1e6, v.bytes / med / 1e9);
  }

  // back-to-back launches (as bench.py issues them): events around each launch, no host sync between
  auto b2b = [&](const char* nm, std::function<void(hipStream_t)> f) {
    const int K = 20;
    std::vector<hipEvent_t> e0(K), e1(K);
    for (int i = 0; i < K; i++) { CK(hipEventCreate(&e0[i])); CK(hipEventCreate(&e1[i])); }
    for (int w = 0; w < 5; w++) f(s);
    for (int i = 0; i < K; i++) { CK(hipEventRecord(e0[i], s)); f(s); CK(hipEventRecord(e1[i], s)); }
    CK(hipStreamSynchronize(s));
    std::vector<float> v(K);
    for (int i = 0; i < K; i++) CK(hipEventElapsedTime(&v[i], e0[i], e1[i]));
    std::sort(v.begin(), v.end());
    double avg = 0; for (float x : v) avg += x; avg /= K;
    printf("b2b %-22s avg %8.1f us  med %8.1f us  min %8.1f  -> %7.1f GB/s (avg)\n", nm, avg * 1e3, v[K / 2] * 1e3, v[0] * 1e3, 3 * S / (avg * 1e-3) / 1e9);
  };
  b2b("tile U4 NTL+NTS", [&](hipStream_t st) { k_tile<4, true, true><<<full(4), 256, 0, st>>>(io, in, nv); });
  b2b("libmpjx combine", [&](hipStream_t st) { if (mpjx_combine(3, 8, io, in, n, st)) exit(2); });
  b2b("tile U4 NTL+NTS", [&](hipStream_t st) { k_tile<4, true, true><<<full(4), 256, 0, st>>>(io, in, nv); });
  b2b("libmpjx combine", [&](hipStream_t st) { if (mpjx_combine(3, 8, io, in, n, st)) exit(2); });
  return 0;
}
