// tune_short.hip — round 4, VERDICT r3 item 3: the configs[3] combine launches are short (8-32 MiB
// int32 slices, 13-26 us) and ran at 0.65-0.74 of the spec in the RCCL engine's layout, against
// 0.79-0.82 for the >= 256 MiB launches. Which launch structure suits a launch that is ~10x the
// kernel boundary? Every variant runs the library's own k_pway template (mpjx_kernels.hpp) with an
// explicit tile (lanes TH x U vectors), cache policy, load group and grid (one tile per block, or a
// persistent grid of k blocks per CU that grid-strides), beside the library's own launch choice
// ("lib": launch_pw), on the same operands: inputs contiguous in ONE allocation (the RCCL engine's
// exchange #1 slots), Scan's P outputs 4 KiB apart, cold (R sets cycled, >= 1 GiB between two uses
// of a set). Median of rounds, ITERS launches per event pair, variants interleaved; one JSON line per
// (shape, variant). Every variant's result is checked against the library's.
// Run: tune_short [rounds=7] [iters=20]   (SHAPES=1,2,... selects shapes)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude tools/tuning/tune_short.hip mpjexpress_amd/csrc/mpjx_k_util.hip -o tools/tuning/tune_short
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../mpjexpress_amd/csrc/mpjx_kernels.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

size_t mpjx::nt_min_bytes() { return mpjx::kStreamBytes; }
size_t mpjx::short_max_bytes() {  // as the library (mpjx_core.hip): MPJX_SHORT_MAX_MIB, default kShortBytes
  const char* e = getenv("MPJX_SHORT_MAX_MIB");
  return e && *e ? (size_t)atol(e) << 20 : mpjx::kShortBytes;
}
int mpjx::cu_count() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 256;
  return n;
}

using namespace mpjx;

struct Set {
  char* in;   // P slots, contiguous
  char* out;  // Q slots, 4 KiB apart
};

struct Shape {
  const char* name;
  int P, kind;
  size_t slice;  // bytes
};

using Launch = std::function<void(const PwayArgs&, hipStream_t)>;

template <class F, int P, int KIND, int TH, int U, int POL, int G>
Launch fixed(int blocks_per_cu) {  // 0 = one tile per block
  return [=](const PwayArgs& a, hipStream_t s) {
    constexpr int W = 16 / sizeof(typename F::T);
    const int64_t nv = a.n / W;
    int64_t blocks = (nv + (int64_t)TH * U - 1) / ((int64_t)TH * U);
    if (blocks_per_cu > 0) blocks = std::min<int64_t>(blocks, 256 * blocks_per_cu);
    hipLaunchKernelGGL((k_pway<F, P, KIND, W, TH, U, POL, G, false>), dim3((unsigned)blocks), dim3(TH), 0, s, a);
  };
}

// Sweep c (round 4, after sweeps a and b = profiles/r04/tuning/tune_short_{a,b}.jsonl: K_SCAN gained
// with more loads in flight per lane — 256 x 8 at P = 4/8 — and the MST/fold shapes with one persistent
// 1024-lane block per CU): those forms and their neighbours, with SKEW = input-slot skew in bytes.
template <class F, int P, int KIND>
std::vector<std::pair<std::string, Launch>> variants() {
  constexpr int PH = P <= 2 ? 1 : 4;  // the streaming form's policy
  std::vector<std::pair<std::string, Launch>> v;
  v.push_back({"lib", [](const PwayArgs& a, hipStream_t s) { CK((launch_pw<F, P, KIND>(a, s, true))); }});
  v.push_back({"1024x1 persist1", fixed<F, P, KIND, 1024, 1, PH, P>(1)});
  if constexpr (P >= 4) {
    v.push_back({"1024x1 persist1 G=2", fixed<F, P, KIND, 1024, 1, PH, 2>(1)});
    v.push_back({"1024x1 persist1 G=4", fixed<F, P, KIND, 1024, 1, PH, 4>(1)});
  }
  v.push_back({"1024x2 persist1", fixed<F, P, KIND, 1024, 2, PH, P>(1)});
  v.push_back({"512x4", fixed<F, P, KIND, 512, 4, PH, P>(0)});
  v.push_back({"512x8", fixed<F, P, KIND, 512, 8, PH, P>(0)});
  v.push_back({"256x8", fixed<F, P, KIND, 256, 8, PH, P>(0)});
  v.push_back({"256x8 pol1", fixed<F, P, KIND, 256, 8, 1, P>(0)});
  v.push_back({"256x8 persist2", fixed<F, P, KIND, 256, 8, PH, P>(2)});
  v.push_back({"256x16", fixed<F, P, KIND, 256, 16, PH, P>(0)});
  v.push_back({"128x16", fixed<F, P, KIND, 128, 16, PH, P>(0)});
  v.push_back({"64x16", fixed<F, P, KIND, 64, 16, PH, P>(0)});
  // sweep d: every load non-temporal, the stores with the default policy (POL 6) — tools/tuning/
  // tune_streams.hip "stores" found plain stores 5 % faster than non-temporal ones for a read-8-write-1
  // launch on 8 MiB slices (the written 8 MiB stay in the L2s / Infinity Cache and drain after the launch)
  v.push_back({"1024x1 persist1 pol6", fixed<F, P, KIND, 1024, 1, 6, P>(1)});
  v.push_back({"1024x1 pol6", fixed<F, P, KIND, 1024, 1, 6, P>(0)});
  if constexpr (P >= 4) v.push_back({"1024x1 persist1 pol6 G=2", fixed<F, P, KIND, 1024, 1, 6, 2>(1)});
  v.push_back({"256x8 pol6", fixed<F, P, KIND, 256, 8, 6, P>(0)});
  return v;
}

template <class F, int P, int KIND>
void run_shape(const char* name, size_t slice, int rounds, int iters) {
  constexpr int Q = KIND == K_SCAN ? P : 1;
  const size_t oslot = slice + 4096;
  const size_t iskew = getenv("SKEW") ? (size_t)atol(getenv("SKEW")) : 0;  // input-slot skew (bytes)
  const size_t islot = slice + iskew;
  const size_t set_bytes = (P + Q) * slice;
  const int R = std::max<int>(2, (int)(((size_t)1 << 30) / set_bytes) + 2);
  std::vector<Set> sets(R);
  using T = typename F::T;
  const int64_t n = slice / sizeof(T);
  for (auto& st : sets) {
    CK(hipMalloc(&st.in, P * islot));
    CK(hipMalloc(&st.out, Q * oslot));
    std::vector<uint32_t> h(P * slice / 4);
    uint64_t x = (uint64_t)(uintptr_t)st.in;
    for (auto& w : h) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      w = (uint32_t)(x >> 32) | (uint32_t)(x >> 40);  // ~5/8 of the bits set (f64: finite, any sign)
      if (sizeof(T) == 8 && (&w - h.data()) % 2) w &= 0xBFFFFFFFu;
    }
    for (int p = 0; p < P; p++)
      CK(hipMemcpy(st.in + p * islot, h.data() + p * slice / 4, slice, hipMemcpyHostToDevice));
  }
  auto args = [&](const Set& st) {
    PwayArgs a{};
    for (int p = 0; p < P; p++) a.in[p] = st.in + p * islot;
    for (int q = 0; q < Q; q++) a.out[q] = st.out + q * oslot;
    a.n = n;
    a.root = 0;
    a.nrep = 1;
    return a;
  };
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto vs = variants<F, P, KIND>();
  // reference result of set 0 from the library launch
  std::vector<uint32_t> ref(Q * slice / 4), got(Q * slice / 4);
  vs[0].second(args(sets[0]), s);
  CK(hipStreamSynchronize(s));
  const size_t wq = slice / 4;  // 32-bit words per output slot
  for (int q = 0; q < Q; q++) CK(hipMemcpy(ref.data() + q * wq, sets[0].out + q * oslot, slice, hipMemcpyDeviceToHost));
  std::vector<std::vector<float>> t(vs.size());
  std::vector<bool> ok(vs.size(), true);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int k = 0;
  for (int r = 0; r < rounds; r++) {
    for (size_t v = 0; v < vs.size(); v++) {
      for (int i = 0; i < R; i++) vs[v].second(args(sets[(k + i) % R]), s);  // warm the code path, flush
      k += R;
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < iters; i++) vs[v].second(args(sets[(k + i) % R]), s);
      CK(hipEventRecord(e1, s));
      k += iters;
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms * 1e3f / iters);
      if (r == 0) {  // check every variant once against the library's result
        CK(hipMemsetAsync(sets[0].out, 0, Q * oslot, s));
        vs[v].second(args(sets[0]), s);
        CK(hipStreamSynchronize(s));
        for (int q = 0; q < Q; q++)
          CK(hipMemcpy(got.data() + q * wq, sets[0].out + q * oslot, slice, hipMemcpyDeviceToHost));
        ok[v] = memcmp(got.data(), ref.data(), got.size() * 4) == 0;
      }
    }
  }
  const double alg = (double)(P + Q) * slice;
  for (size_t v = 0; v < vs.size(); v++) {
    auto w = t[v];
    std::sort(w.begin(), w.end());
    const double med = w[w.size() / 2];
    printf("{\"shape\": \"%s\", \"variant\": \"%s\", \"in_skew\": %zu, \"us_median\": %.2f, \"us_min\": %.2f, "
           "\"frac\": %.4f, \"sets\": %d, \"exact\": %s}\n",
           name, vs[v].first.c_str(), iskew, med, w[0], alg / (med * 1e-6) / 8e12, R, ok[v] ? "true" : "false");
  }
  fflush(stdout);
  for (auto& st : sets) {
    CK(hipFree(st.in));
    CK(hipFree(st.out));
  }
  CK(hipStreamDestroy(s));
}

// ---- the P = 1 Allreduce's copy (the N = 1 headline: recv = send, 256 MiB) ---------------------------
// The library's k_copies<true> is 512 lanes x one 16-B vector per lane, non-temporal loads and stores
// (mpjx_k_util.hip). Variants: tile shape, store / load policy, persistent grids.
template <int TH, int U, bool LNT, bool SNT>
__global__ __launch_bounds__(TH) void k_copy(const v4u* __restrict__ src, v4u* __restrict__ dst, int64_t nv) {
  for (int64_t t = (int64_t)blockIdx.x * TH * U; t < nv; t += (int64_t)gridDim.x * TH * U) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t i = t + u * TH + threadIdx.x;
      if (i < nv) v[u] = LNT ? __builtin_nontemporal_load(src + i) : src[i];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t i = t + u * TH + threadIdx.x;
      if (i < nv) {
        if (SNT) __builtin_nontemporal_store(v[u], dst + i);
        else dst[i] = v[u];
      }
    }
  }
}

using CopyLaunch = std::function<void(const char*, char*, int64_t, hipStream_t)>;

template <int TH, int U, bool LNT, bool SNT>
CopyLaunch copyv(int blocks_per_cu) {
  return [=](const char* src, char* dst, int64_t bytes, hipStream_t s) {
    const int64_t nv = bytes / 16;
    int64_t blocks = (nv + (int64_t)TH * U - 1) / ((int64_t)TH * U);
    if (blocks_per_cu > 0) blocks = std::min<int64_t>(blocks, 256 * blocks_per_cu);
    hipLaunchKernelGGL((k_copy<TH, U, LNT, SNT>), dim3((unsigned)blocks), dim3(TH), 0, s, (const v4u*)src, (v4u*)dst, nv);
  };
}

void run_copy(size_t bytes, int rounds, int iters) {
  std::vector<std::pair<std::string, CopyLaunch>> vs;
  vs.push_back({"lib k_copies", [](const char* src, char* dst, int64_t b, hipStream_t s) {
                  CopyList l;
                  l.add(dst, src, b);
                  CK(launch_copies(l, s));
                }});
  vs.push_back({"512x1 nt/nt", copyv<512, 1, true, true>(0)});
  vs.push_back({"1024x1 nt/nt", copyv<1024, 1, true, true>(0)});
  vs.push_back({"256x1 nt/nt", copyv<256, 1, true, true>(0)});
  vs.push_back({"256x2 nt/nt", copyv<256, 2, true, true>(0)});
  vs.push_back({"256x4 nt/nt", copyv<256, 4, true, true>(0)});
  vs.push_back({"512x1 nt/default", copyv<512, 1, true, false>(0)});
  vs.push_back({"512x1 default/nt", copyv<512, 1, false, true>(0)});
  vs.push_back({"512x1 default/default", copyv<512, 1, false, false>(0)});
  vs.push_back({"512x2 nt/nt persist4", copyv<512, 2, true, true>(4)});
  vs.push_back({"1024x1 nt/nt persist2", copyv<1024, 1, true, true>(2)});
  vs.push_back({"256x4 nt/nt persist8", copyv<256, 4, true, true>(8)});
  vs.push_back({"1024x4 nt/nt persist1", copyv<1024, 4, true, true>(1)});
  const int R = std::max<int>(2, (int)(((size_t)1 << 30) / (2 * bytes)) + 2);
  std::vector<char*> src(R), dst(R);
  for (int k = 0; k < R; k++) {
    CK(hipMalloc(&src[k], bytes));
    CK(hipMalloc(&dst[k], bytes));
    CK(hipMemset(src[k], k + 1, bytes));
  }
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> t(vs.size());
  std::vector<bool> ok(vs.size(), true);
  std::vector<unsigned char> h(bytes);
  int k = 0;
  for (int r = 0; r < rounds; r++)
    for (size_t v = 0; v < vs.size(); v++) {
      for (int i = 0; i < R; i++) vs[v].second(src[(k + i) % R], dst[(k + i) % R], bytes, s);
      k += R;
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < iters; i++) vs[v].second(src[(k + i) % R], dst[(k + i) % R], bytes, s);
      CK(hipEventRecord(e1, s));
      k += iters;
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms * 1e3f / iters);
      if (r == 0) {
        CK(hipMemsetAsync(dst[0], 0, bytes, s));
        vs[v].second(src[0], dst[0], bytes, s);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h.data(), dst[0], bytes, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < bytes && ok[v]; i += 4093) ok[v] = h[i] == 1;
      }
    }
  for (size_t v = 0; v < vs.size(); v++) {
    auto w = t[v];
    std::sort(w.begin(), w.end());
    const double med = w[w.size() / 2];
    printf("{\"shape\": \"copy %zu MiB (Allreduce P=1)\", \"variant\": \"%s\", \"us_median\": %.2f, \"us_min\": %.2f, "
           "\"frac\": %.4f, \"sets\": %d, \"exact\": %s}\n",
           bytes >> 20, vs[v].first.c_str(), med, w[0], 2.0 * bytes / (med * 1e-6) / 8e12, R, ok[v] ? "true" : "false");
  }
  fflush(stdout);
  for (int i = 0; i < R; i++) {
    CK(hipFree(src[i]));
    CK(hipFree(dst[i]));
  }
  CK(hipStreamDestroy(s));
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7, iters = argc > 2 ? atoi(argv[2]) : 20;
  const char* only = getenv("SHAPES");  // optional comma list of shape numbers
  auto want = [&](int i) {  // SHAPES: comma list of shape numbers (all when unset)
    if (!only) return true;
    const std::string l = std::string(",") + only + ",";
    return l.find("," + std::to_string(i) + ",") != std::string::npos;
  };
  if (want(1)) run_shape<Band<uint32_t>, 8, K_MST>("RS BAND int32 N=8 (K_MST P=8, 8 MiB)", 8 << 20, rounds, iters);
  if (want(2)) run_shape<Bxor<uint32_t>, 8, K_SCAN>("Scan BXOR int32 N=8 (K_SCAN P=8, 8 MiB)", 8 << 20, rounds, iters);
  if (want(3)) run_shape<Band<uint32_t>, 4, K_MST>("RS BAND int32 N=4 (K_MST P=4, 16 MiB)", 16 << 20, rounds, iters);
  if (want(4)) run_shape<Bxor<uint32_t>, 4, K_SCAN>("Scan BXOR int32 N=4 (K_SCAN P=4, 16 MiB)", 16 << 20, rounds, iters);
  if (want(5)) run_shape<Band<uint32_t>, 2, K_FOLD>("RS BAND int32 N=2 (K_FOLD P=2, 32 MiB)", 32 << 20, rounds, iters);
  if (want(6)) run_shape<Bxor<uint32_t>, 2, K_SCAN>("Scan BXOR int32 N=2 (K_SCAN P=2, 32 MiB)", 32 << 20, rounds, iters);
  // guards: the f64 shapes the engines run at N = 8 (a short-launch form must not slow them)
  if (want(7)) run_shape<Sum<double>, 8, K_MST>("Allreduce SUM f64 N=8 (K_MST P=8, 32 MiB)", 32 << 20, rounds, iters);
  if (want(8)) run_shape<Sum<double>, 8, K_SCAN>("Scan SUM f64 N=8 (K_SCAN P=8, 32 MiB)", 32 << 20, rounds, iters);
  if (want(9)) run_copy((size_t)256 << 20, rounds, iters);
  // the short-launch forms on other element widths (f64 Allreduce / Scan of 64 MiB at N = 8; byte types
  // take the 512-lane tile at P = 8)
  if (want(10)) run_shape<Sum<double>, 8, K_MST>("Allreduce SUM f64 64 MiB N=8 (K_MST P=8, 8 MiB)", 8 << 20, rounds, iters);
  if (want(11)) run_shape<Sum<double>, 8, K_SCAN>("Scan SUM f64 64 MiB N=8 (K_SCAN P=8, 8 MiB)", 8 << 20, rounds, iters);
  if (want(12)) run_shape<Band<uint8_t>, 8, K_MST>("RS BAND byte N=8 (K_MST P=8, 8 MiB)", 8 << 20, rounds, iters);
  return 0;
}
