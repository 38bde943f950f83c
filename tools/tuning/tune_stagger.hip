// tune_stagger.hip — round 3, VERDICT r2 item 6: does the issue pattern of a lane's P operand loads
// matter? tune_split's harness kernel for K_MST P=4 on 64 MiB slices ran 53.6 us (0.78) against 55.5 us
// (0.75) for the library's k_pway on the same layout, and its ISA issues three loads, waits for them,
// then the fourth (the compiler's choice for that add tree), where k_pway issues all four, then waits.
// Here every variant has the library's body (1024 lanes, one 16-B vector per operand per lane, operand 0
// default policy at P >= 3 and non-temporal at P <= 2, the other operands and the stores non-temporal)
// and differs only in how many loads a lane issues before it waits for them: groups of G operands,
// each group drained (s_waitcnt vmcnt(0) between scheduler barriers) before the next group issues.
// G = P is the library's pattern.
// Cold: R sets cycled (>= 1.5 GiB between two uses of a set); operands in ONE allocation per set at
// slice + 4 KiB (the engines' layout). The library's own k_pway runs beside them on the same sets.
// Median of rounds, 20 launches per event pair, variants interleaved. One JSON line per variant.
// Run: tune_stagger [rounds=7] [skew=4096] [output skew=skew]
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include tools/tuning/tune_stagger.hip -o tools/tuning/tune_stagger
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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
  x = y + x;
  v4u r;
  __builtin_memcpy(&r, &x, 16);
  return r;
}

constexpr int TH = 1024;

struct Args {
  const v4u* in[8];
  v4u* out[8];
};

// MST tree at root 0 (PureIntracomm.java:1943-1992): acc of [L..R] = acc[M+1..R] (op) acc[L..M]
template <int L, int R, int P>
__device__ __forceinline__ v4u mst(const v4u (&x)[P]) {
  if constexpr (L == R) return x[L];
  else {
    constexpr int M = (L + R) / 2;
    return add(mst<M + 1, R>(x), mst<L, M>(x));
  }
}

// s_waitcnt vmcnt(0) with expcnt/lgkmcnt left at their maxima (gfx9 encoding)
constexpr unsigned kWaitVm0 = (7u << 4) | (15u << 8);

template <int P, int KIND, int G>
__global__ __launch_bounds__(TH) void kst(Args a) {
  const long i = (long)blockIdx.x * TH + threadIdx.x;
  v4u x[P];
  // The scheduler barriers pin the issue order: groups of G loads, each group drained (vmcnt 0)
  // before the next issues. Without them the compiler reorders loads around the adds by itself
  // (an MST P=4 tree came out as 3 loads, wait, 1 load).
#pragma unroll
  for (int p = 0; p < P; p++) {
    if (p == 0 && P > 2) x[0] = a.in[0][i];
    else x[p] = __builtin_nontemporal_load(a.in[p] + i);
    if ((p + 1) % G == 0 && p + 1 < P) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(kWaitVm0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (KIND == mpjx::K_SCAN) {
#pragma unroll
    for (int r = 0; r < P; r++) {
      v4u acc = x[r];
#pragma unroll
      for (int k = 0; k < r; k++) acc = add(x[k], acc);
      __builtin_nontemporal_store(acc, a.out[r] + i);
    }
  } else if constexpr (KIND == mpjx::K_MST) {
    __builtin_nontemporal_store(mst<0, P - 1>(x), a.out[0] + i);
  } else {
    v4u acc = x[0];
#pragma unroll
    for (int k = 1; k < P; k++) acc = add(x[k], acc);
    __builtin_nontemporal_store(acc, a.out[0] + i);
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
  int P, kind;
  long bytes;      // per slice
  bool in_place;   // out[0] = in[0] (the 2-operand fold of configs[1])
  std::vector<Args> sets;
  int Q() const { return kind == mpjx::K_SCAN ? P : 1; }
};

using Launch = void (*)(const Args&, const Shape&, hipStream_t);

template <int P, int KIND, int G>
static void launch_st(const Args& a, const Shape& sh, hipStream_t s) {
  kst<P, KIND, G><<<(unsigned)(sh.bytes / 16 / TH), TH, 0, s>>>(a);
}

template <int P, int KIND, int G = mpjx::LoadGroup<P, KIND, (P <= 2 ? 1 : 4)>::value>
static void launch_lib(const Args& b, const Shape& sh, hipStream_t s) {
  mpjx::PwayArgs a{};
  for (int p = 0; p < P; p++) a.in[p] = b.in[p];
  for (int q = 0; q < sh.Q(); q++) a.out[q] = b.out[q];
  a.n = sh.bytes / 8;
  a.root = 0;
  a.nrep = 1;
  (void)mpjx::launch_one<mpjx::Sum<double>, P, KIND, 2, 1024, 1, (P <= 2 ? 1 : 4), G>(a, s);
}

struct Var {
  Shape* sh;
  std::string name;
  Launch f;
  std::vector<double> us;
};

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  const long skew = argc > 2 ? atol(argv[2]) : 4096;
  const long oskew = argc > 3 ? atol(argv[3]) : skew;  // output-slot skew (the engines always skew outputs)
  std::vector<Shape*> shapes = {new Shape{"MST P4 64MiB", 4, mpjx::K_MST, 64L << 20, false, {}},
                                new Shape{"SCAN P8 32MiB", 8, mpjx::K_SCAN, 32L << 20, false, {}},
                                new Shape{"MST P8 32MiB", 8, mpjx::K_MST, 32L << 20, false, {}},
                                new Shape{"SCAN P4 64MiB", 4, mpjx::K_SCAN, 64L << 20, false, {}},
                                new Shape{"FOLD P2 256MiB in-place", 2, mpjx::K_FOLD, 256L << 20, true, {}}};
  unsigned long long seed = 1;
  for (auto* sh : shapes) {
    const int slots = sh->P + (sh->in_place ? 0 : sh->Q());
    const long set_bytes = (sh->bytes + std::max(skew, oskew)) * slots;
    const int R = (int)std::max(3L, (1536L << 20) / set_bytes + 1);
    for (int r = 0; r < R; r++) {
      char* base;
      CK(hipMalloc(&base, set_bytes));
      Args a{};
      for (int p = 0; p < sh->P; p++) {
        a.in[p] = (const v4u*)(base + p * (sh->bytes + skew));
        k_fill<<<4096, 256>>>((unsigned long long*)a.in[p], sh->bytes / 8, seed++);
      }
      if (sh->in_place) a.out[0] = (v4u*)a.in[0];
      else
        for (int q = 0; q < sh->Q(); q++)
          a.out[q] = (v4u*)(base + sh->P * (sh->bytes + skew) + q * (sh->bytes + oskew));
      sh->sets.push_back(a);
    }
  }
  CK(hipDeviceSynchronize());
  std::vector<Var> V;
  for (auto* sh : shapes) {
    auto add = [&](const char* n, Launch f) { V.push_back({sh, n, f, {}}); };
    if (sh->P == 4 && sh->kind == mpjx::K_MST) {
      add("library k_pway (default G)", launch_lib<4, mpjx::K_MST>);
      add("library k_pway G4", launch_lib<4, mpjx::K_MST, 4>);
      add("library k_pway G3", launch_lib<4, mpjx::K_MST, 3>);
      add("library k_pway G2", launch_lib<4, mpjx::K_MST, 2>);
      add("library k_pway G1", launch_lib<4, mpjx::K_MST, 1>);
      add("G4 (all, then wait)", launch_st<4, mpjx::K_MST, 4>);
      add("G3 (3, wait, 1)", launch_st<4, mpjx::K_MST, 3>);
      add("G2 (2, wait, 2)", launch_st<4, mpjx::K_MST, 2>);
      add("G1 (one at a time)", launch_st<4, mpjx::K_MST, 1>);
    } else if (sh->P == 4) {
      add("library k_pway (default G)", launch_lib<4, mpjx::K_SCAN>);
      add("library k_pway G4", launch_lib<4, mpjx::K_SCAN, 4>);
      add("library k_pway G2", launch_lib<4, mpjx::K_SCAN, 2>);
      add("library k_pway G3", launch_lib<4, mpjx::K_SCAN, 3>);
      add("G4 (all, then wait)", launch_st<4, mpjx::K_SCAN, 4>);
      add("G3 (3, wait, 1)", launch_st<4, mpjx::K_SCAN, 3>);
      add("G2 (2, wait, 2)", launch_st<4, mpjx::K_SCAN, 2>);
    } else if (sh->P == 8 && sh->kind == mpjx::K_SCAN) {
      add("library k_pway (default G)", launch_lib<8, mpjx::K_SCAN>);
      add("library k_pway G6", launch_lib<8, mpjx::K_SCAN, 6>);
      add("library k_pway G4", launch_lib<8, mpjx::K_SCAN, 4>);
      add("library k_pway G3", launch_lib<8, mpjx::K_SCAN, 3>);
      add("library k_pway G2", launch_lib<8, mpjx::K_SCAN, 2>);
      add("G8 (all, then wait)", launch_st<8, mpjx::K_SCAN, 8>);
      add("G6 (6, wait, 2)", launch_st<8, mpjx::K_SCAN, 6>);
      add("G4 (4, wait, 4)", launch_st<8, mpjx::K_SCAN, 4>);
      add("G2 (2 at a time)", launch_st<8, mpjx::K_SCAN, 2>);
    } else if (sh->P == 8) {
      add("library k_pway (default G)", launch_lib<8, mpjx::K_MST>);
      add("library k_pway G8", launch_lib<8, mpjx::K_MST, 8>);
      add("library k_pway G6", launch_lib<8, mpjx::K_MST, 6>);
      add("library k_pway G4", launch_lib<8, mpjx::K_MST, 4>);
      add("library k_pway G2", launch_lib<8, mpjx::K_MST, 2>);
      add("G8 (all, then wait)", launch_st<8, mpjx::K_MST, 8>);
      add("G6 (6, wait, 2)", launch_st<8, mpjx::K_MST, 6>);
      add("G4 (4, wait, 4)", launch_st<8, mpjx::K_MST, 4>);
      add("G2 (2 at a time)", launch_st<8, mpjx::K_MST, 2>);
    } else {
      add("library k_pway (default G)", launch_lib<2, mpjx::K_FOLD>);
      add("library k_pway G1", launch_lib<2, mpjx::K_FOLD, 1>);
      add("G2 (both, then wait)", launch_st<2, mpjx::K_FOLD, 2>);
      add("G1 (one at a time)", launch_st<2, mpjx::K_FOLD, 1>);
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
      for (int l = 0; l < kLaunches; l++) v.f(sets[l % sets.size()], *v.sh, s);
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
    const double bytes = (double)v.sh->bytes * (v.sh->P + v.sh->Q());
    printf("{\"shape\": \"%s\", \"variant\": \"%s\", \"sets\": %zu, \"us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f}\n",
           v.sh->name.c_str(), v.name.c_str(), v.sh->sets.size(), med, v.us[0], bytes / (med * 1e-6) / 8e12);
  }
  return 0;
}
