// tune_grid.hip — block -> tile mapping of the streaming P-way kernels (round 3):
// K_MST-like P=4 sum of 64 MiB slices and K_SCAN P=8 on 32 MiB slices, the two BASELINE combine
// shapes below 0.78 of 8 TB/s. The library launches one 1024-lane tile per block (map 0). Variants:
//   map 1: persistent grid of G = 256*k blocks, grid-stride over tiles
//   map 2: one tile per block, XCD-contiguous (block b on XCD b%8 takes tile (b%8)*(NT/8) + b/8)
//   map 3: G = NT/m blocks, each walking m consecutive tiles
//   map 4: persistent grid, each XCD's blocks grid-striding over that XCD's contiguous 1/8
// Operands live in ONE allocation per set at a stride of slice + 4 KiB (the engines' layout), cold:
// R sets cycled so no launch finds its operands in the Infinity Cache. Median of rounds, 20 launches
// per event pair, variants interleaved. Output: one JSON line per variant.
// Run: tune_grid [rounds=7] [skew=4096] [sweep=1]
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tuning/tune_grid.hip -o tools/tuning/tune_grid
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

struct Args {
  const v4u* in[8];
  v4u* out[8];
  long nv;     // vectors per operand
  long ntile;  // tiles of TH vectors
  int m;       // map 3: tiles per block
};

template <int P, bool SCAN, int TH, int MASK, bool NTS>
__device__ __forceinline__ void tile(const Args& a, long t) {
  const long i = t * TH + threadIdx.x;
  if (i >= a.nv) return;
  v4u x[P];
#pragma unroll
  for (int p = 0; p < P; p++) {
    if ((MASK >> p) & 1) x[p] = __builtin_nontemporal_load(a.in[p] + i);
    else x[p] = a.in[p][i];
  }
  if constexpr (SCAN) {
#pragma unroll
    for (int r = 0; r < P; r++) {
      v4u acc = x[r];
#pragma unroll
      for (int k = 0; k < r; k++) acc = add(x[k], acc);
      if constexpr (NTS) __builtin_nontemporal_store(acc, a.out[r] + i);
      else a.out[r][i] = acc;
    }
  } else {
    v4u acc = x[0];
#pragma unroll
    for (int k = 1; k < P; k++) acc = add(x[k], acc);
    if constexpr (NTS) __builtin_nontemporal_store(acc, a.out[0] + i);
    else a.out[0][i] = acc;
  }
}

template <int P, bool SCAN, int TH, int MAP, int MASK, bool NTS>
__global__ __launch_bounds__(TH) void kg(Args a) {
  const long b = blockIdx.x, G = gridDim.x;
  if constexpr (MAP == 0) {
    tile<P, SCAN, TH, MASK, NTS>(a, b);
  } else if constexpr (MAP == 1) {
    for (long t = b; t < a.ntile; t += G) tile<P, SCAN, TH, MASK, NTS>(a, t);
  } else if constexpr (MAP == 2) {
    const long per = a.ntile / 8;
    tile<P, SCAN, TH, MASK, NTS>(a, (b % 8) * per + b / 8);
  } else if constexpr (MAP == 3) {
    for (long t = b * a.m, e = std::min(a.ntile, t + a.m); t < e; t++) tile<P, SCAN, TH, MASK, NTS>(a, t);
  } else {
    const long per = a.ntile / 8, x = b % 8, g = G / 8;
    for (long t = b / 8; t < per; t += g) tile<P, SCAN, TH, MASK, NTS>(a, x * per + t);
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

struct Shape {
  std::string name;
  int P;
  bool scan;
  long bytes;  // per slice
  std::vector<Args> sets;
};

struct Var {
  const Shape* sh;
  std::string name;
  unsigned grid;
  int m;
  std::function<void(const Args&, unsigned, hipStream_t)> f;
  std::vector<double> us;
};

template <int P, bool SCAN, int TH, int MAP, int MASK, bool NTS>
static void add(std::vector<Var>& V, const Shape& sh, unsigned k_or_m = 0) {
  const long nt = sh.bytes / 16 / TH;
  unsigned grid = (unsigned)nt;
  int m = 0;
  if (MAP == 1 || MAP == 4) grid = 256 * k_or_m;
  if (MAP == 3) {
    m = (int)k_or_m;
    grid = (unsigned)((nt + m - 1) / m);
  }
  char nm[128];
  snprintf(nm, sizeof nm, "TH%d map%d %s%u mask%X st%s", TH, MAP, MAP == 3 ? "m" : "k", k_or_m, MASK, NTS ? "NT" : "plain");
  V.push_back({&sh, nm, grid, m, [](const Args& a, unsigned g, hipStream_t s) { kg<P, SCAN, TH, MAP, MASK, NTS><<<g, TH, 0, s>>>(a); }, {}});
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  const long skew = argc > 2 ? atol(argv[2]) : 4096;
  const int sweep = argc > 3 ? atoi(argv[3]) : 1;  // 1: block -> tile maps; 2: policy x lanes
  std::vector<Shape> shapes = {{"MST P4 64MiB", 4, false, 64L << 20, {}},
                               {"SCAN P8 32MiB", 8, true, 32L << 20, {}},
                               {"MST P8 32MiB", 8, false, 32L << 20, {}}};
  unsigned long long seed = 1;
  for (auto& sh : shapes) {
    const long set_bytes = (sh.bytes + skew) * (sh.P + (sh.scan ? sh.P : 1));
    const int R = (int)std::max(3L, (1536L << 20) / set_bytes + 1);
    for (int r = 0; r < R; r++) {
      char* base;
      CK(hipMalloc(&base, set_bytes));
      Args a{};
      a.nv = sh.bytes / 16;
      for (int p = 0; p < sh.P; p++) {
        a.in[p] = (const v4u*)(base + p * (sh.bytes + skew));
        k_fill<<<4096, 256>>>((unsigned long long*)a.in[p], sh.bytes / 8, seed++);
      }
      for (int q = 0; q < (sh.scan ? sh.P : 1); q++) a.out[q] = (v4u*)(base + (sh.P + q) * (sh.bytes + skew));
      sh.sets.push_back(a);
    }
  }
  CK(hipDeviceSynchronize());
  std::vector<Var> V;
  for (auto& sh : shapes) {
    if (sweep == 2) {  // policy x lanes at one tile per block (the library's mapping)
      if (sh.P == 4) {
        add<4, false, 1024, 0, 0xE, true>(V, sh);
        add<4, false, 1024, 0, 0xF, true>(V, sh);
        add<4, false, 512, 0, 0xE, true>(V, sh);
        add<4, false, 512, 0, 0xF, true>(V, sh);
        add<4, false, 256, 0, 0xE, true>(V, sh);
        add<4, false, 256, 0, 0xF, true>(V, sh);
        add<4, false, 1024, 0, 0xC, true>(V, sh);
      } else if (sh.scan) {
        add<8, true, 1024, 0, 0xFE, true>(V, sh);
        add<8, true, 1024, 0, 0xFF, true>(V, sh);
        add<8, true, 512, 0, 0xFE, true>(V, sh);
        add<8, true, 512, 0, 0xFF, true>(V, sh);
        add<8, true, 256, 0, 0xFE, true>(V, sh);
        add<8, true, 256, 0, 0xFF, true>(V, sh);
      } else {
        add<8, false, 1024, 0, 0xFE, true>(V, sh);
        add<8, false, 1024, 0, 0xFF, true>(V, sh);
        add<8, false, 512, 0, 0xFE, true>(V, sh);
        add<8, false, 512, 0, 0xFF, true>(V, sh);
      }
      continue;
    }
    if (sh.P == 4) {
      add<4, false, 1024, 0, 0xE, true>(V, sh);
      add<4, false, 1024, 0, 0xF, true>(V, sh);
      add<4, false, 1024, 2, 0xE, true>(V, sh);
      for (unsigned k : {1u, 2u, 4u, 8u}) add<4, false, 1024, 1, 0xE, true>(V, sh, k);
      for (unsigned k : {2u, 4u}) add<4, false, 1024, 4, 0xE, true>(V, sh, k);
      for (unsigned m : {2u, 4u, 16u}) add<4, false, 1024, 3, 0xE, true>(V, sh, m);
      add<4, false, 512, 0, 0xE, true>(V, sh);
      for (unsigned k : {4u, 8u, 16u}) add<4, false, 512, 1, 0xE, true>(V, sh, k);
      add<4, false, 256, 0, 0xE, true>(V, sh);
      for (unsigned k : {8u, 16u}) add<4, false, 256, 1, 0xE, true>(V, sh, k);
    } else if (sh.scan) {
      add<8, true, 1024, 0, 0xFE, true>(V, sh);
      add<8, true, 1024, 2, 0xFE, true>(V, sh);
      for (unsigned k : {1u, 2u, 4u}) add<8, true, 1024, 1, 0xFE, true>(V, sh, k);
      for (unsigned k : {2u}) add<8, true, 1024, 4, 0xFE, true>(V, sh, k);
      for (unsigned m : {2u, 4u}) add<8, true, 1024, 3, 0xFE, true>(V, sh, m);
      add<8, true, 512, 0, 0xFE, true>(V, sh);
      for (unsigned k : {4u, 8u}) add<8, true, 512, 1, 0xFE, true>(V, sh, k);
    } else {
      add<8, false, 1024, 0, 0xFE, true>(V, sh);
      add<8, false, 1024, 2, 0xFE, true>(V, sh);
      for (unsigned k : {2u, 4u}) add<8, false, 1024, 1, 0xFE, true>(V, sh, k);
      for (unsigned m : {2u, 4u}) add<8, false, 1024, 3, 0xFE, true>(V, sh, m);
    }
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  constexpr int kLaunches = 20;
  for (int r = 0; r <= rounds; r++) {  // round 0 is warm-up
    for (auto& v : V) {
      Args a = v.sh->sets[0];
      for (auto& st : const_cast<Shape*>(v.sh)->sets) st.ntile = a.nv / (v.name.rfind("TH1024", 0) == 0 ? 1024 : v.name.rfind("TH512", 0) == 0 ? 512 : 256), st.m = v.m;
      const auto& sets = v.sh->sets;
      CK(hipEventRecord(e0, s));
      for (int l = 0; l < kLaunches; l++) v.f(sets[l % sets.size()], v.grid, s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(hipGetLastError());
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0) v.us.push_back(ms * 1000.0 / kLaunches);
    }
  }
  for (auto& v : V) {
    std::sort(v.us.begin(), v.us.end());
    const double med = v.us[v.us.size() / 2];
    const double bytes = (double)v.sh->bytes * (v.sh->P + (v.sh->scan ? v.sh->P : 1));
    printf("{\"shape\": \"%s\", \"variant\": \"%s\", \"grid\": %u, \"sets\": %zu, \"us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f}\n",
           v.sh->name.c_str(), v.name.c_str(), v.grid, v.sh->sets.size(), med, v.us[0], bytes / (med * 1e-6) / 8e12);
  }
  return 0;
}
