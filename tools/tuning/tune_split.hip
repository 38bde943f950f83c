// tune_split.hip — round 3, VERDICT r2 item 6 follow-up: why does K_MST P=4 on 64 MiB slices stay at
// 0.75 of 8 TB/s when the same kernel on 32 MiB slices reaches 0.79 and K_SCAN P=4 on 64 MiB 0.80+?
// Same kernel body as the library's streaming form (1024 lanes, one 16-B vector per operand per lane,
// operand 0 default policy, the rest and the stores non-temporal), cold (R sets cycled, >= 1.5 GiB
// between two uses of a set), operands in ONE allocation per set at slice + skew (the engines' layout).
// Variants per shape:
//   split k   the launch cut into k back-to-back launches over consecutive sub-ranges
//   region R  one launch; block b takes tile (b % R) * (NT / R) + b / R, so the blocks in flight stream
//             R distant regions of every operand at once (R = 8 was tune_grid's XCD-contiguous map)
// plus a slice-size sweep of the unsplit kernel (is 64 MiB special, or large P=4 launches in general?).
// Median of rounds, 20 launches per event pair, variants interleaved. One JSON line per variant.
//   library   the library's own k_pway instantiation for the shape (mpjx_kernels.hpp), same sets
// Run: tune_split [rounds=7] [skew=4096]
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tuning/tune_split.hip -o tools/tuning/tune_split
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../../mpjexpress_amd/csrc/mpjx_kernels.hpp"  // the library's k_pway, for an A/B in one process

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

constexpr int TH = 1024;

struct Args {
  const v4u* in[8];
  v4u* out[8];
  long t0;     // first tile of this launch
  long ntile;  // tiles in this launch
  int R;       // regions
};

template <int P, bool SCAN>
__device__ __forceinline__ void tile(const Args& a, long t) {
  const long i = t * TH + threadIdx.x;
  v4u x[P];
  x[0] = a.in[0][i];
#pragma unroll
  for (int p = 1; p < P; p++) x[p] = __builtin_nontemporal_load(a.in[p] + i);
  if constexpr (SCAN) {
#pragma unroll
    for (int r = 0; r < P; r++) {
      v4u acc = x[r];
#pragma unroll
      for (int k = 0; k < r; k++) acc = add(x[k], acc);
      __builtin_nontemporal_store(acc, a.out[r] + i);
    }
  } else {  // the MST tree at root 0 for P = 4: (x1 + x0) and (x3 + x2), then combined
    v4u acc;
    if constexpr (P == 4) acc = add(add(x[3], x[2]), add(x[1], x[0]));
    else {
      acc = x[0];
#pragma unroll
      for (int k = 1; k < P; k++) acc = add(x[k], acc);
    }
    __builtin_nontemporal_store(acc, a.out[0] + i);
  }
}

template <int P, bool SCAN>
__global__ __launch_bounds__(TH) void ks(Args a) {
  const long b = blockIdx.x;
  const long per = a.ntile / a.R;
  tile<P, SCAN>(a, a.t0 + (b % a.R) * per + b / a.R);
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
  Shape* sh;
  std::string name;
  int split, R;
  std::vector<double> us;
  int lib = 0;  // 1: the library's k_pway (launch_one, the streaming instantiation it picks for this shape)
};

template <int P, bool SCAN>
static void launch(const Args& a, unsigned g, hipStream_t s) { ks<P, SCAN><<<g, TH, 0, s>>>(a); }

static void run_lib(const Var& v, const Args& base, hipStream_t s) {
  mpjx::PwayArgs a{};
  const int P = v.sh->P, Q = v.sh->scan ? P : 1;
  for (int p = 0; p < P; p++) a.in[p] = base.in[p];
  for (int q = 0; q < Q; q++) a.out[q] = base.out[q];
  a.n = v.sh->bytes / 8;
  a.root = 0;
  a.nrep = 1;
  using F = mpjx::Sum<double>;
  if (v.sh->scan) mpjx::launch_one<F, 8, mpjx::K_SCAN, 2, 1024, 1, 4>(a, s);
  else if (P == 4) mpjx::launch_one<F, 4, mpjx::K_MST, 2, 1024, 1, 4>(a, s);
  else mpjx::launch_one<F, 8, mpjx::K_MST, 2, 1024, 1, 4>(a, s);
}

static void run(const Var& v, const Args& base, hipStream_t s) {
  if (v.lib) return run_lib(v, base, s);
  const long nt = v.sh->bytes / 16 / TH;
  const long per = nt / v.split;
  for (int k = 0; k < v.split; k++) {
    Args a = base;
    a.t0 = k * per;
    a.ntile = per;
    a.R = v.R;
    const unsigned g = (unsigned)per;
    if (v.sh->scan) launch<8, true>(a, g, s);
    else if (v.sh->P == 4) launch<4, false>(a, g, s);
    else launch<8, false>(a, g, s);
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  const long skew = argc > 2 ? atol(argv[2]) : 4096;
  std::vector<Shape*> shapes;
  for (long mib : {16L, 32L, 48L, 64L, 96L, 128L}) {
    char nm[64];
    snprintf(nm, sizeof nm, "MST P4 %ldMiB", mib);
    shapes.push_back(new Shape{nm, 4, false, mib << 20, {}});
  }
  shapes.push_back(new Shape{"SCAN P8 32MiB", 8, true, 32L << 20, {}});
  shapes.push_back(new Shape{"MST P8 32MiB", 8, false, 32L << 20, {}});
  unsigned long long seed = 1;
  for (auto* sh : shapes) {
    const long set_bytes = (sh->bytes + skew) * (sh->P + (sh->scan ? sh->P : 1));
    const int R = (int)std::max(3L, (1536L << 20) / set_bytes + 1);
    for (int r = 0; r < R; r++) {
      char* base;
      CK(hipMalloc(&base, set_bytes));
      Args a{};
      for (int p = 0; p < sh->P; p++) {
        a.in[p] = (const v4u*)(base + p * (sh->bytes + skew));
        k_fill<<<4096, 256>>>((unsigned long long*)a.in[p], sh->bytes / 8, seed++);
      }
      for (int q = 0; q < (sh->scan ? sh->P : 1); q++) a.out[q] = (v4u*)(base + (sh->P + q) * (sh->bytes + skew));
      sh->sets.push_back(a);
    }
  }
  CK(hipDeviceSynchronize());
  std::vector<Var> V;
  for (auto* sh : shapes) {
    V.push_back({sh, "split1 region1", 1, 1, {}});
    if (sh->bytes == (64L << 20) || sh->P == 8) {
      V.push_back({sh, "library k_pway", 1, 1, {}, 1});
      for (int k : {2, 4}) V.push_back({sh, "split" + std::to_string(k) + " region1", k, 1, {}});
      for (int r : {2, 4}) V.push_back({sh, "split1 region" + std::to_string(r), 1, r, {}});
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
      const auto& sets = v.sh->sets;
      CK(hipEventRecord(e0, s));
      for (int l = 0; l < kLaunches; l++) run(v, sets[l % sets.size()], s);
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
    printf("{\"shape\": \"%s\", \"variant\": \"%s\", \"sets\": %zu, \"us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f}\n",
           v.sh->name.c_str(), v.name.c_str(), v.sh->sets.size(), med, v.us[0], bytes / (med * 1e-6) / 8e12);
  }
  return 0;
}
