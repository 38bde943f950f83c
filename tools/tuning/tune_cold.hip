// tune_cold.hip — cache-policy and tile-shape variants of the path's streaming kernels, timed COLD:
// every launch works on the next of R independent buffer sets (R sets of >= 512 MiB between two uses
// of a line), so no launch finds its operands in the 256 MiB Infinity Cache from an earlier launch —
// what a reduction over fresh message data sees. The same variants are also timed WARM (R = 1: the
// same buffers every launch, the round-2 tuning method), to show how much of a warm figure is cache.
// 20 launches between one event pair, variants interleaved over rounds, median reported.
//
// Shapes: in-place fold (configs[1]: inout = in + inout, 2 x 256 MiB double), out-of-place 2-way fold
// (256 MiB), copy (256 MiB: Reduce's arraycopy at P = 1), 8-way sum of 32 MiB slices (the N=8 K_MST
// block), copy of 32 MiB (the IPC push blocks).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune_cold.hip -o tools/tune_cold
// Run:   tools/tune_cold [rounds=7] [cold_sets=4] [sweep=1..5]
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

struct Args {
  const v4u* in[8];
  v4u* out;
  long nv;
};

// P operands (P = 1: copy) summed in list order into out; NT0 = policy of operand 0 (the accumulator
// of an in-place fold), NTR = the others, NTS = stores. One tile of T lanes x U vectors per block.
template <int P, int T, int U, bool NT0, bool NTR, bool NTS>
__global__ __launch_bounds__(T) void k(Args a) {
  const long base = (long)blockIdx.x * T * U;
  v4u x[U][P];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < a.nv) {
      x[u][0] = ld<NT0>(a.in[0] + i);
#pragma unroll
      for (int p = 1; p < P; p++) x[u][p] = ld<NTR>(a.in[p] + i);
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < a.nv) {
      v4u r = x[u][0];
#pragma unroll
      for (int p = 1; p < P; p++) r = add(x[u][p], r);
      st<NTS>(a.out + i, r);
    }
  }
}

// per-operand policy: bit p of MASK set = operand p loaded non-temporally (sweep 3)
template <int P, int T, int U, int MASK, bool NTS>
__global__ __launch_bounds__(T) void km(Args a) {
  const long base = (long)blockIdx.x * T * U;
  v4u x[U][P];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < a.nv) {
#pragma unroll
      for (int p = 0; p < P; p++) {
        if ((MASK >> p) & 1) x[u][p] = __builtin_nontemporal_load(a.in[p] + i);
        else x[u][p] = a.in[p][i];
      }
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < a.nv) {
      v4u r = x[u][0];
#pragma unroll
      for (int p = 1; p < P; p++) r = add(x[u][p], r);
      st<NTS>(a.out + i, r);
    }
  }
}

// Scan (sweep 5): Q = P outputs, out[r] = in[r-1] + (... + (in[0] + in[r])); outputs at a.out + r*nv
template <int P, int T, int MASK, bool NTS>
__global__ __launch_bounds__(T) void kscan(Args a) {
  const long i = (long)blockIdx.x * T + threadIdx.x;
  if (i >= a.nv) return;
  v4u x[P];
#pragma unroll
  for (int p = 0; p < P; p++) {
    if ((MASK >> p) & 1) x[p] = __builtin_nontemporal_load(a.in[p] + i);
    else x[p] = a.in[p][i];
  }
#pragma unroll
  for (int r = 0; r < P; r++) {
    v4u acc = x[r];
#pragma unroll
    for (int k = 0; k < r; k++) acc = add(x[k], acc);
    st<NTS>(a.out + (long)r * a.nv + i, acc);
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
  int P;          // operands
  bool inplace;   // out == in[0]
  long bytes;     // per operand
  std::vector<Args> sets;  // sets[0] = the warm set; cold cycles over all
};

struct Var {
  std::string shape, name;
  int T, U;
  std::function<void(const Args&, unsigned, hipStream_t)> f;
  const Shape* sh;
  std::vector<double> warm, cold;
};

template <int P, int T, int U, bool A, bool B, bool C>
static void add_var(std::vector<Var>& V, const Shape& sh) {
  char nm[96];
  snprintf(nm, sizeof nm, "T%-4d U%d  acc %-5s in %-5s st %-5s", T, U, A ? "NT" : "plain", B ? "NT" : "plain",
           C ? "NT" : "plain");
  V.push_back({sh.name, nm, T, U,
               [](const Args& a, unsigned g, hipStream_t s) { k<P, T, U, A, B, C><<<g, T, 0, s>>>(a); }, &sh,
               {}, {}});
}

// every load/store policy combination (P = 1: the operand-0 policy is the copy's load policy)
template <int P, int T, int U>
static void add_pols(std::vector<Var>& V, const Shape& sh) {
  add_var<P, T, U, true, true, true>(V, sh);
  add_var<P, T, U, false, false, true>(V, sh);
  add_var<P, T, U, false, false, false>(V, sh);
  add_var<P, T, U, true, true, false>(V, sh);
  if constexpr (P > 1) {
    add_var<P, T, U, true, false, true>(V, sh);
    add_var<P, T, U, false, true, true>(V, sh);
  }
}

template <int P, int T, int MASK, int U = 1>
static void add_mask(std::vector<Var>& V, const Shape& sh) {
  char nm[96];
  snprintf(nm, sizeof nm, "T%-4d U%d  nt-mask 0x%02x st NT", T, U, MASK);
  V.push_back({sh.name, nm, T, U, [](const Args& a, unsigned g, hipStream_t s) { km<P, T, U, MASK, true><<<g, T, 0, s>>>(a); },
               &sh, {}, {}});
}

template <int P, int T, int MASK, bool NTS>
static void add_scan(std::vector<Var>& V, const Shape& sh) {
  char nm[96];
  snprintf(nm, sizeof nm, "scan T%-4d nt-mask 0x%02x st %s", T, MASK, NTS ? "NT" : "plain");
  V.push_back({sh.name, nm, T, 1, [](const Args& a, unsigned g, hipStream_t s) { kscan<P, T, MASK, NTS><<<g, T, 0, s>>>(a); },
               &sh, {}, {}});
}

// the policies that led a first sweep (profiles/r02/cold/tune_cold_sweep1.txt) for a second, shape-only one
template <int P, int T, int U>
static void add_lead(std::vector<Var>& V, const Shape& sh) {
  add_var<P, T, U, true, true, true>(V, sh);
  add_var<P, T, U, false, false, true>(V, sh);
  if constexpr (P > 1) {
    add_var<P, T, U, true, false, true>(V, sh);
    add_var<P, T, U, false, true, true>(V, sh);
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  const int R = argc > 2 ? atoi(argv[2]) : 4;
  const int sweep = argc > 3 ? atoi(argv[3]) : 1;
  std::vector<Shape> shapes = {{"inplace P2 256MiB", 2, true, 256L << 20, {}},
                               {"fold P2 256MiB -> out", 2, false, 256L << 20, {}},
                               {"copy 256MiB", 1, false, 256L << 20, {}},
                               {"sum P8 32MiB -> out", 8, false, 32L << 20, {}},
                               {"copy 32MiB", 1, false, 32L << 20, {}}};
  if (sweep == 5)  // Scan shapes: P outputs (the set's out holds P slices)
    shapes = {{"scan P8 32MiB -> 8 outs", 8, false, 32L << 20, {}}, {"scan P2 32MiB -> 2 outs", 2, false, 32L << 20, {}}};
  if (sweep == 4)  // tile shapes at the N = 2 / 4 combine shapes
    shapes = {{"fold P2 128MiB -> out", 2, false, 128L << 20, {}}, {"sum P4 64MiB -> out", 4, false, 64L << 20, {}}};
  if (sweep == 3)  // per-operand policy masks at the N = 2 / 4 / 8 combine shapes
    shapes = {{"fold P2 128MiB -> out", 2, false, 128L << 20, {}},
              {"sum P4 64MiB -> out", 4, false, 64L << 20, {}},
              {"sum P8 32MiB -> out", 8, false, 32L << 20, {}},
              {"sum P8 8MiB -> out", 8, false, 8L << 20, {}}};
  unsigned long long seed = 1;
  for (auto& sh : shapes) {
    const long n = sh.bytes / 8;
    for (int r = 0; r < R; r++) {
      Args a{};
      a.nv = sh.bytes / 16;
      for (int p = 0; p < sh.P; p++) {
        v4u* b;
        CK(hipMalloc(&b, sh.bytes));
        k_fill<<<4096, 256>>>((unsigned long long*)b, n, seed++);
        a.in[p] = b;
      }
      if (sh.inplace) {
        a.out = const_cast<v4u*>(a.in[0]);
      } else {
        CK(hipMalloc(&a.out, sh.bytes * (sweep == 5 ? sh.P : 1)));
      }
      sh.sets.push_back(a);
    }
  }
  CK(hipDeviceSynchronize());
  const bool shapes_only = sweep == 2;  // 1: every policy; 2: tile shapes; 3: per-operand masks
  std::vector<Var> V;
  for (auto& sh : shapes) {
    if (sweep == 5) {
      if (sh.P == 8) {
        add_scan<8, 1024, 0xFF, true>(V, sh);
        add_scan<8, 1024, 0xFE, true>(V, sh);
        add_scan<8, 1024, 0x00, true>(V, sh);
        add_scan<8, 1024, 0xFF, false>(V, sh);
        add_scan<8, 1024, 0x00, false>(V, sh);
        add_scan<8, 512, 0xFE, true>(V, sh);
        add_scan<8, 256, 0xFE, true>(V, sh);
      } else {
        add_scan<2, 1024, 0x3, true>(V, sh);
        add_scan<2, 1024, 0x2, true>(V, sh);
        add_scan<2, 1024, 0x0, true>(V, sh);
        add_scan<2, 1024, 0x3, false>(V, sh);
        add_scan<2, 256, 0x3, true>(V, sh);
      }
    } else if (sweep == 4) {
      if (sh.P == 2) {
        add_mask<2, 1024, 0x3>(V, sh);
        add_mask<2, 512, 0x3>(V, sh);
        add_mask<2, 512, 0x3, 2>(V, sh);
        add_mask<2, 256, 0x3, 2>(V, sh);
        add_mask<2, 256, 0x3, 4>(V, sh);
      } else {
        add_mask<4, 1024, 0xF>(V, sh);
        add_mask<4, 1024, 0xE>(V, sh);
        add_mask<4, 512, 0xF>(V, sh);
        add_mask<4, 512, 0xE>(V, sh);
        add_mask<4, 512, 0xF, 2>(V, sh);
        add_mask<4, 512, 0xE, 2>(V, sh);
        add_mask<4, 256, 0xF, 2>(V, sh);
        add_mask<4, 256, 0xE, 2>(V, sh);
        add_mask<4, 256, 0xF, 4>(V, sh);
        add_mask<4, 1024, 0xF, 2>(V, sh);
      }
    } else if (sweep == 3) {
      if (sh.P == 2) {
        add_mask<2, 1024, 0x3>(V, sh);
        add_mask<2, 1024, 0x2>(V, sh);
        add_mask<2, 1024, 0x1>(V, sh);
        add_mask<2, 1024, 0x0>(V, sh);
      } else if (sh.P == 4) {
        add_mask<4, 1024, 0xF>(V, sh);
        add_mask<4, 1024, 0xE>(V, sh);
        add_mask<4, 1024, 0xC>(V, sh);
        add_mask<4, 1024, 0xA>(V, sh);
        add_mask<4, 1024, 0x7>(V, sh);
        add_mask<4, 1024, 0x0>(V, sh);
      } else {
        add_mask<8, 1024, 0xFF>(V, sh);
        add_mask<8, 1024, 0xFE>(V, sh);
        add_mask<8, 1024, 0xFC>(V, sh);
        add_mask<8, 1024, 0xF0>(V, sh);
        add_mask<8, 1024, 0xAA>(V, sh);
        add_mask<8, 1024, 0x7F>(V, sh);
        add_mask<8, 1024, 0xEE>(V, sh);
        add_mask<8, 1024, 0x00>(V, sh);
      }
    } else if (shapes_only) {
      if (sh.P == 2) {
        add_lead<2, 1024, 1>(V, sh);
        add_lead<2, 512, 1>(V, sh);
        add_lead<2, 256, 1>(V, sh);
        add_lead<2, 1024, 2>(V, sh);
        add_lead<2, 512, 4>(V, sh);
      } else if (sh.P == 1) {
        add_lead<1, 1024, 1>(V, sh);
        add_lead<1, 512, 1>(V, sh);
        add_lead<1, 1024, 2>(V, sh);
        add_lead<1, 512, 2>(V, sh);
        add_lead<1, 256, 2>(V, sh);
        add_lead<1, 1024, 4>(V, sh);
      } else {
        add_lead<8, 1024, 1>(V, sh);
        add_lead<8, 512, 1>(V, sh);
        add_lead<8, 256, 1>(V, sh);
        add_lead<8, 512, 2>(V, sh);
      }
    } else if (sh.P == 2) {
      add_pols<2, 256, 4>(V, sh);
      add_pols<2, 256, 2>(V, sh);
      add_pols<2, 512, 2>(V, sh);
      add_pols<2, 1024, 1>(V, sh);
    } else if (sh.P == 1) {
      add_pols<1, 256, 4>(V, sh);
      add_pols<1, 256, 2>(V, sh);
      add_pols<1, 512, 2>(V, sh);
      add_pols<1, 256, 8>(V, sh);
    } else {
      add_pols<8, 256, 1>(V, sh);
      add_pols<8, 256, 2>(V, sh);
      add_pols<8, 512, 1>(V, sh);
    }
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int K = 20;
  for (int r = 0; r < rounds; r++)
    for (auto& v : V)
      for (int cold = 0; cold < 2; cold++) {
        const auto& sets = v.sh->sets;
        const unsigned g = (unsigned)((sets[0].nv + (long)v.T * v.U - 1) / ((long)v.T * v.U));
        auto set = [&](int i) -> const Args& { return cold ? sets[i % sets.size()] : sets[0]; };
        for (int w = 0; w < 3; w++) v.f(set(w), g, s);
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < K; i++) v.f(set(i + 3), g, s);
        CK(hipEventRecord(e1, s));
        CK(hipStreamSynchronize(s));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        (cold ? v.cold : v.warm).push_back(ms / K * 1e3);
      }
  printf("cold = %d buffer sets cycled per launch; warm = the same set every launch\n", R);
  printf("%-24s %-38s %9s %7s %9s %7s\n", "shape", "variant", "cold_us", "frac", "warm_us", "frac");
  for (auto& v : V) {
    std::sort(v.cold.begin(), v.cold.end());
    std::sort(v.warm.begin(), v.warm.end());
    const double c = v.cold[v.cold.size() / 2], w = v.warm[v.warm.size() / 2];
    const double bytes = (double)v.sh->bytes * (v.sh->P + (sweep == 5 ? v.sh->P : 1));
    printf("%-24s %-38s %9.1f %7.3f %9.1f %7.3f\n", v.shape.c_str(), v.name.c_str(), c, bytes / (c * 1e-6) / 8e12, w,
           bytes / (w * 1e-6) / 8e12);
  }
}
