// tune_streams.hip — round 4: where does a read-dominated P-way combine lose against the read-only
// stream? The K_MST P=8 combine reads 8 operand streams and writes 1 (8:1) at 6.3-6.4 TB/s (0.79-0.80 of
// the spec), while one read-only stream reaches 7.4-7.5 TB/s (tools/hbm_probe.hip). Same total bytes,
// cold (sets cycled, >= 1 GiB between two uses), 1024 lanes x one 16-B vector per stream per lane:
//   read S streams, no stores        (S = 1, 2, 4, 8; the lane's XOR is kept live with one store per block)
//   read S streams, write 1 stream   (the combine's traffic shape, S = 1 (copy), 2, 4, 8)
//   read 8 streams in pairs (load groups) and 8 streams with the slots 4 KiB apart
// Median of rounds; one JSON line per variant. Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tuning/tune_streams.hip -o tools/tuning/tune_streams
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

using v4u = unsigned int __attribute__((ext_vector_type(4)));

struct Args {
  const v4u* in[8];
  v4u* out;
  int64_t nv;  // vectors per stream
};

template <int S, bool WRITE, int G>
__global__ __launch_bounds__(1024) void k_streams(Args a) {
  const int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
  if (i >= a.nv) return;
  v4u x[S];
#pragma unroll
  for (int p = 0; p < S; p++) {
    x[p] = __builtin_nontemporal_load(a.in[p] + i);
    if constexpr (G < S) {
      if ((p + 1) % G == 0 && p + 1 < S) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt((7u << 4) | (15u << 8));
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  v4u r = x[0];
#pragma unroll
  for (int p = 1; p < S; p++) r ^= x[p];
  if constexpr (WRITE) {
    __builtin_nontemporal_store(r, a.out + i);
  } else {
    // keep the loads live: one lane per block stores (negligible traffic), the rest fold into it
    if ((r.x ^ r.y ^ r.z ^ r.w) == 0x9E3779B9u) a.out[blockIdx.x] = r;
  }
}

// The same read-8-write-1 body with the result store's cache policy as a parameter (round 4, the fixed
// cost of short launches): 0 = __builtin_nontemporal_store (the library's streaming stores), 1 = plain,
// else a buffer store with aux = STP - 2 cache bits (16 = sc1 write-through, 17 = sc0 sc1, 2 = nt,
// 18 = sc1 nt). Plain / sc0 / nt keep the written line in the XCD's L2, sc1 drops it (MI355X_MICROARCH.md
// "stores of each flavour"): does that change what the end of the launch costs?
template <int STP>
__global__ __launch_bounds__(1024) void k_r8w1(Args a) {
  const int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
  if (i >= a.nv) return;
  v4u x[8];
#pragma unroll
  for (int p = 0; p < 8; p++) x[p] = __builtin_nontemporal_load(a.in[p] + i);
  v4u r = x[0];
#pragma unroll
  for (int p = 1; p < 8; p++) r ^= x[p];
  if constexpr (STP == 0) {
    __builtin_nontemporal_store(r, a.out + i);
  } else if constexpr (STP == 1) {
    a.out[i] = r;
  } else {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, (int)(a.nv * 16 > 0x7fffffff ? 0x7fffffff : a.nv * 16),
                                                        0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(r, rsrc, (int)(i * 16), 0, STP - 2);
  }
}

static int stores_main(int rounds, int iters) {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct P {
    const char* name;
    void (*k)(Args);
  };
  const P pols[] = {{"nt (library)", k_r8w1<0>}, {"plain", k_r8w1<1>}, {"sc1", k_r8w1<2 + 16>},
                    {"sc0 sc1", k_r8w1<2 + 17>}, {"nt (buffer)", k_r8w1<2 + 2>}, {"sc1 nt", k_r8w1<2 + 18>}};
  for (size_t slice_mib : {8, 16, 32}) {
    const size_t slice = slice_mib << 20, set = 8 * (slice + 4096) + slice;
    const int R = (int)std::max<size_t>(3, ((size_t)3 << 30) / set + 1);  // >= 3 GiB between two uses
    std::vector<char*> bufs(R);
    for (int k = 0; k < R; k++) {
      CK(hipMalloc(&bufs[k], set));
      CK(hipMemset(bufs[k], k + 1, set));
    }
    auto args = [&](int k) {
      Args a{};
      for (int p = 0; p < 8; p++) a.in[p] = (const v4u*)(bufs[k] + p * (slice + 4096));
      a.out = (v4u*)(bufs[k] + 8 * (slice + 4096));
      a.nv = (int64_t)(slice / 16);
      return a;
    };
    std::vector<std::vector<float>> t(sizeof pols / sizeof pols[0]);
    int c = 0;
    for (int r = 0; r < rounds; r++)
      for (size_t v = 0; v < t.size(); v++) {
        auto go = [&](int k) {
          const Args a = args(k);
          hipLaunchKernelGGL(pols[v].k, dim3((unsigned)((a.nv + 1023) / 1024)), dim3(1024), 0, st, a);
        };
        for (int i = 0; i < R; i++) go((c + i) % R);
        c += R;
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < iters; i++) go((c + i) % R);
        CK(hipEventRecord(e1, st));
        c += iters;
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[v].push_back(ms * 1e3f / iters);
      }
    for (size_t v = 0; v < t.size(); v++) {
      auto w = t[v];
      std::sort(w.begin(), w.end());
      const double med = w[w.size() / 2], bytes = 9.0 * slice;
      printf("{\"mode\": \"stores\", \"store\": \"%s\", \"slice_MiB\": %zu, \"bytes\": %.0f, \"us_median\": %.2f, "
             "\"us_min\": %.2f, \"frac\": %.4f}\n", pols[v].name, slice_mib, bytes, med, w[0], bytes / med / 1e6 / 8.0);
      fflush(stdout);
    }
    for (char* b : bufs) CK(hipFree(b));
  }
  return 0;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7, iters = argc > 2 ? atoi(argv[2]) : 20;
  if (argc > 3 && std::string(argv[3]) == "stores") return stores_main(rounds, iters);
  const size_t total = (size_t)256 << 20;  // bytes READ per launch, split over the streams
  struct V {
    std::string name;
    int S;
    bool write;
    size_t skew;
    std::function<void(const Args&, hipStream_t)> go;
  };
  auto mk = [](auto kern) {
    return [kern](const Args& a, hipStream_t s) {
      hipLaunchKernelGGL(kern, dim3((unsigned)((a.nv + 1023) / 1024)), dim3(1024), 0, s, a);
    };
  };
  // the copy with the destination offset from the source's alignment by `skew` bytes (dst = out + skew):
  // do reads and writes that run at the same offsets meet in the same HBM channels?
  std::vector<V> vs = {
      {"copy, dst +0", 1, true, 0, mk(k_streams<1, true, 1>)},
      {"copy, dst +4 KiB", 1, true, 4096, mk(k_streams<1, true, 1>)},
      {"copy, dst +64 KiB", 1, true, 65536, mk(k_streams<1, true, 1>)},
      {"copy, dst +1 MiB", 1, true, 1 << 20, mk(k_streams<1, true, 1>)},
      {"copy, dst +2 MiB+4 KiB", 1, true, (2 << 20) + 4096, mk(k_streams<1, true, 1>)},
      {"read 1 stream", 1, false, 0, mk(k_streams<1, false, 1>)},
      {"read 2 streams", 2, false, 0, mk(k_streams<2, false, 2>)},
      {"read 4 streams", 4, false, 0, mk(k_streams<4, false, 4>)},
      {"read 8 streams", 8, false, 0, mk(k_streams<8, false, 8>)},
      {"read 8 streams, 4 KiB skew", 8, false, 4096, mk(k_streams<8, false, 8>)},
      {"read 8 streams G=2", 8, false, 0, mk(k_streams<8, false, 2>)},
      {"copy: read 1 write 1", 1, true, 0, mk(k_streams<1, true, 1>)},
      {"read 2 write 1", 2, true, 0, mk(k_streams<2, true, 2>)},
      {"read 4 write 1", 4, true, 0, mk(k_streams<4, true, 4>)},
      {"read 8 write 1", 8, true, 0, mk(k_streams<8, true, 8>)},
      {"read 8 write 1, 4 KiB skew", 8, true, 4096, mk(k_streams<8, true, 8>)},
      {"read 8 write 1 G=2", 8, true, 0, mk(k_streams<8, true, 2>)},
  };
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int R = 6;  // sets of (256 MiB read + up to 256 MiB written): >= 2.5 GiB between two uses
  std::vector<char*> inb(R), outb(R);
  for (int k = 0; k < R; k++) {
    CK(hipMalloc(&inb[k], total + 8 * 4096));
    CK(hipMalloc(&outb[k], total + (4 << 20)));
    CK(hipMemset(inb[k], k + 1, total + 8 * 4096));
  }
  std::vector<std::vector<float>> t(vs.size());
  int c = 0;
  for (int r = 0; r < rounds; r++)
    for (size_t v = 0; v < vs.size(); v++) {
      const V& x = vs[v];
      const size_t per = total / x.S;  // bytes per stream
      auto args = [&](int k) {
        Args a{};
        const bool dst_skew = x.S == 1 && x.write;  // the copy rows: skew the destination instead
        for (int p = 0; p < x.S; p++) a.in[p] = (const v4u*)(inb[k] + p * (per + (dst_skew ? 0 : x.skew)));
        a.out = (v4u*)(outb[k] + (dst_skew ? x.skew : 0));
        a.nv = (int64_t)(per / 16);
        return a;
      };
      for (int i = 0; i < R; i++) x.go(args((c + i) % R), st);
      c += R;
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < iters; i++) x.go(args((c + i) % R), st);
      CK(hipEventRecord(e1, st));
      c += iters;
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms * 1e3f / iters);
    }
  for (size_t v = 0; v < vs.size(); v++) {
    auto w = t[v];
    std::sort(w.begin(), w.end());
    const double med = w[w.size() / 2];
    const double bytes = (double)total + (vs[v].write ? (double)total / vs[v].S : 0.0);
    printf("{\"variant\": \"%s\", \"streams\": %d, \"write\": %s, \"bytes\": %.0f, \"us_median\": %.2f, \"TBps\": %.3f, "
           "\"frac\": %.4f}\n",
           vs[v].name.c_str(), vs[v].S, vs[v].write ? "true" : "false", bytes, med, bytes / med / 1e6,
           bytes / med / 1e6 / 8.0);
  }
  return 0;
}
