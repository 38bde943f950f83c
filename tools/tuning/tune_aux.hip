// tune_aux.hip — beyond the load/store policy pairs of tune_cold.hip, for the configs[1] in-place
// fold (inout = in + inout, 2 x 256 MiB double) on COLD operands (R independent pairs cycled per
// launch): the cache-policy bits of buffer loads/stores (aux: 1 = sc0, 2 = nt, 16 = sc1) and a
// persistent grid (G blocks striding over the vector) against the shipped one-tile-per-block form
// (1024 lanes x one 16-B vector per operand, global_load/store ... nt).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune_aux.hip -o tools/tune_aux
// Run:   tools/tune_aux [rounds=9] [cold_sets=4]
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

// shipped form: one 16-B vector per operand per lane, one tile per block, global nt
__global__ __launch_bounds__(1024) void k_tile(v4u* io, const v4u* in, long nv) {
  const long i = (long)blockIdx.x * 1024 + threadIdx.x;
  if (i < nv) {
    v4u a = __builtin_nontemporal_load(io + i), b = __builtin_nontemporal_load(in + i);
    __builtin_nontemporal_store(add(b, a), io + i);
  }
}

// persistent: G blocks stride over the vector
__global__ __launch_bounds__(1024) void k_persist(v4u* io, const v4u* in, long nv) {
  for (long i = (long)blockIdx.x * 1024 + threadIdx.x; i < nv; i += (long)gridDim.x * 1024) {
    v4u a = __builtin_nontemporal_load(io + i), b = __builtin_nontemporal_load(in + i);
    __builtin_nontemporal_store(add(b, a), io + i);
  }
}

// buffer loads/stores with explicit cache-policy bits (one rsrc per operand; 256 MiB < 2^31)
template <int LA, int SA>
__global__ __launch_bounds__(1024) void k_buf(v4u* io, const v4u* in, long nv) {
  const long i = (long)blockIdx.x * 1024 + threadIdx.x;
  if (i >= nv) return;
  __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void*)io, 0, 0x7fffffff, 0x00020000);
  __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, 0x7fffffff, 0x00020000);
  const int off = (int)(i * 16);
  v4u a = __builtin_amdgcn_raw_buffer_load_b128(rio, off, 0, LA);
  v4u b = __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, LA);
  __builtin_amdgcn_raw_buffer_store_b128(add(b, a), rio, off, 0, SA);
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
  const int rounds = argc > 1 ? atoi(argv[1]) : 9;
  const int R = argc > 2 ? atoi(argv[2]) : 4;
  const long bytes = 256L << 20, n = bytes / 8, nv = bytes / 16;
  std::vector<v4u*> io(R), in(R);
  for (int r = 0; r < R; r++) {
    CK(hipMalloc(&io[r], bytes));
    CK(hipMalloc(&in[r], bytes));
    k_fill<<<4096, 256>>>((unsigned long long*)io[r], n, 2 * r + 1);
    k_fill<<<4096, 256>>>((unsigned long long*)in[r], n, 2 * r + 2);
  }
  CK(hipDeviceSynchronize());
  struct Var { std::string name; std::function<void(v4u*, const v4u*, hipStream_t)> f; std::vector<double> us; };
  std::vector<Var> V;
  const unsigned tiles = (unsigned)((nv + 1023) / 1024);
  V.push_back({"tile 1024x1 global nt (shipped)", [=](v4u* a, const v4u* b, hipStream_t s) { k_tile<<<tiles, 1024, 0, s>>>(a, b, nv); }, {}});
  for (unsigned g : {512u, 1024u, 2048u, 4096u, 8192u}) {
    char nm[64];
    snprintf(nm, sizeof nm, "persistent %u blocks x 1024", g);
    V.push_back({nm, [=](v4u* a, const v4u* b, hipStream_t s) { k_persist<<<g, 1024, 0, s>>>(a, b, nv); }, {}});
  }
#define BUF(la, sa) V.push_back({"buffer ld aux " #la " st aux " #sa, [=](v4u* a, const v4u* b, hipStream_t s) { k_buf<la, sa><<<tiles, 1024, 0, s>>>(a, b, nv); }, {}})
  BUF(2, 2);
  BUF(18, 2);
  BUF(3, 2);
  BUF(19, 2);
  BUF(2, 3);
  BUF(2, 18);
  BUF(2, 19);
  BUF(0, 2);
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int K = 20;
  for (int r = 0; r < rounds; r++)
    for (auto& v : V) {
      for (int w = 0; w < 3; w++) v.f(io[w % R], in[w % R], s);
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < K; i++) v.f(io[(i + 3) % R], in[(i + 3) % R], s);
      CK(hipEventRecord(e1, s));
      CK(hipStreamSynchronize(s));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms / K * 1e3);
    }
  printf("cold: %d operand pairs cycled per launch; 2 x 256 MiB double in-place fold, 805,306,368 B per launch\n", R);
  printf("%-40s %9s %9s %7s\n", "variant", "med_us", "min_us", "frac");
  for (auto& v : V) {
    std::sort(v.us.begin(), v.us.end());
    const double med = v.us[v.us.size() / 2];
    printf("%-40s %9.1f %9.1f %7.3f\n", v.name.c_str(), med, v.us[0], 3.0 * bytes / (med * 1e-6) / 8e12);
  }
}
