// tune_policy2.hip — per-operand load policy of the P-way fold (double SUM, out = fold of P slices),
// sustained: 20 back-to-back launches between one event pair, variants interleaved over rounds.
// tune_policy found, for the 2-operand combine, non-temporal loads of one operand and default-policy
// loads of the other 12 % faster than non-temporal loads of both. Which operands to load
// non-temporally at P > 2? mask bit p set = operand p loaded non-temporally; stores non-temporal.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune_policy2.hip -o tools/tune_policy2
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
  v4u* out;
  long nv;
};

template <int P, unsigned MASK, int U>
__global__ __launch_bounds__(256) void k(Args a) {
  constexpr int T = 256;
  const long base = (long)blockIdx.x * T * U;
  v4u x[U][P];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < a.nv) {
#pragma unroll
      for (int p = 0; p < P; p++)
        x[u][p] = ((MASK >> p) & 1u) ? __builtin_nontemporal_load(a.in[p] + i) : a.in[p][i];
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const long i = base + u * T + threadIdx.x;
    if (i < a.nv) {
      d2 acc;
      __builtin_memcpy(&acc, &x[u][0], 16);
#pragma unroll
      for (int p = 1; p < P; p++) {
        d2 v;
        __builtin_memcpy(&v, &x[u][p], 16);
        acc = v + acc;
      }
      v4u r;
      __builtin_memcpy(&r, &acc, 16);
      __builtin_nontemporal_store(r, a.out + i);
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

template <int P, unsigned MASK, int U>
static Var make(const char* tag, Args a) {
  const unsigned grid = (unsigned)((a.nv + 256L * U - 1) / (256L * U));
  char name[96];
  snprintf(name, sizeof name, "P=%d %-10s mask=0x%02x U%d", P, tag, MASK, U);
  return {name, [=](hipStream_t st) { k<P, MASK, U><<<grid, 256, 0, st>>>(a); }, (double)(P + 1) * a.nv * 16, {}};
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  const long big = 256L << 20, small = 32L << 20;
  char* pool;
  const size_t cap = 9 * big;
  CK(hipMalloc(&pool, cap));
  k_fill<<<4096, 256>>>((unsigned long long*)pool, (long)(cap / 8), 11);
  CK(hipDeviceSynchronize());
  auto args = [&](int P, long slice) {
    Args a{};
    for (int p = 0; p < P; p++) a.in[p] = (const v4u*)(pool + p * slice);
    a.out = (v4u*)(pool + P * slice);
    a.nv = slice / 16;
    return a;
  };
  std::vector<Var> V;
  const bool sweep = argc > 2 && std::string(argv[2]) == "sweep";  // footprint sweep, slices 8..256 MiB
  const bool unroll = argc > 2 && std::string(argv[2]) == "unroll";  // U per P at 32 / 256 MiB slices
  if (unroll) {
    Args a4s = args(4, small), a8s = args(8, small), a4b = args(4, big), a8b = args(8, big);
    V.push_back(make<4, 0x0, 2>("plain32 U2", a4s));
    V.push_back(make<4, 0x0, 4>("plain32 U4", a4s));
    V.push_back(make<8, 0x00, 1>("plain32 U1", a8s));
    V.push_back(make<8, 0x00, 2>("plain32 U2", a8s));
    V.push_back(make<4, 0xF, 2>("NT256 U2", a4b));
    V.push_back(make<4, 0xF, 4>("NT256 U4", a4b));
    V.push_back(make<8, 0xFF, 1>("NT256 U1", a8b));
    V.push_back(make<8, 0xFF, 2>("NT256 U2", a8b));
  } else if (sweep) {
    static char names[64][32];
    int k = 0;
    for (long mib : {8L, 16L, 32L, 64L, 128L, 256L}) {
      const long slice = mib << 20;
      Args a2 = args(2, slice), a4 = args(4, slice), a8 = args(8, slice);
      snprintf(names[k], 32, "NT %ldMiB", mib);
      snprintf(names[k + 1], 32, "plain %ldMiB", mib);
      V.push_back(make<2, 0x3, 4>(names[k], a2));
      V.push_back(make<2, 0x0, 4>(names[k + 1], a2));
      V.push_back(make<4, 0xF, 2>(names[k], a4));
      V.push_back(make<4, 0x0, 2>(names[k + 1], a4));
      V.push_back(make<8, 0xFF, 1>(names[k], a8));
      V.push_back(make<8, 0x00, 1>(names[k + 1], a8));
      k += 2;
    }
  } else {
    Args a = args(2, big);  // the configs[1] shape as a fold into a third buffer
    V.push_back(make<2, 0x3, 4>("allNT", a));
    V.push_back(make<2, 0x1, 4>("p0NT", a));
    V.push_back(make<2, 0x2, 4>("p1NT", a));
  }
  for (long slice : {small, big}) {
    if (sweep || unroll) break;
    Args a3 = args(3, slice), a4 = args(4, slice), a8 = args(8, slice);
    const char* sz = slice == small ? "32MiB" : "256MiB";
    char t[8][32];
    snprintf(t[0], 32, "allNT %s", sz);
    snprintf(t[1], 32, "p0NT %s", sz);
    snprintf(t[2], 32, "alt %s", sz);
    snprintf(t[3], 32, "half %s", sz);
    snprintf(t[4], 32, "plain %s", sz);
    V.push_back(make<3, 0x7, 2>(t[0], a3));
    V.push_back(make<3, 0x1, 2>(t[1], a3));
    V.push_back(make<3, 0x5, 2>(t[2], a3));
    V.push_back(make<4, 0xF, 2>(t[0], a4));
    V.push_back(make<4, 0x1, 2>(t[1], a4));
    V.push_back(make<4, 0x5, 2>(t[2], a4));
    V.push_back(make<4, 0x3, 2>(t[3], a4));
    V.push_back(make<8, 0xFF, 1>(t[0], a8));
    V.push_back(make<8, 0x01, 1>(t[1], a8));
    V.push_back(make<8, 0x55, 1>(t[2], a8));
    V.push_back(make<8, 0x0F, 1>(t[3], a8));
    V.push_back(make<8, 0x00, 1>(t[4], a8));
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
  printf("%-40s %9s %9s %9s %7s\n", "variant (20 b2b launches, 1 event pair)", "med_us", "min_us", "GB/s", "frac");
  for (auto& v : V) {
    std::sort(v.us.begin(), v.us.end());
    const double med = v.us[v.us.size() / 2];
    printf("%-40s %9.1f %9.1f %9.1f %7.3f\n", v.name.c_str(), med, v.us[0], v.bytes / (med * 1e-6) / 1e9,
           v.bytes / (med * 1e-6) / 8e12);
  }
}
