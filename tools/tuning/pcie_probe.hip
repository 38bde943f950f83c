// pcie_probe.hip — round 4: what bounds the host-resident path (mpjx_*_host, north_star's end-to-end
// rate)? The chunk pipeline overlaps H2D of chunk c+1, the collective on chunk c and D2H of chunk c-1, and
// reaches 38-40 GB/s of S/t at P = 1, while one direction alone runs 45-57 GB/s. Is the ceiling the host
// link's duplex, the DMA engines, or the pageable staging? Measured here, 256 MiB per direction:
//   dma   hipMemcpyAsync between pinned host and device, one direction, then both at once on two streams
//   kern  a copy kernel whose lanes read (H2D) or write (D2H) the pinned host buffer through its device
//         mapping, one direction, both at once, and mixed with DMA in the other direction
//   cpu   memcpy pageable -> pinned with T host threads (the staging step a pageable call needs)
// Round 5 adds the chain with alternating copy streams. Median of rounds; one JSON line per variant. Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tuning/pcie_probe.hip -o tools/tuning/pcie_probe -lpthread
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

using v4u = unsigned int __attribute__((ext_vector_type(4)));

// grid-stride copy, 16 B per lane per step
__global__ __launch_bounds__(256) void k_copy(v4u* __restrict__ dst, const v4u* __restrict__ src, int64_t nv) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += stride) dst[i] = src[i];
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 5;
  const size_t S = (size_t)256 << 20;
  const int64_t nv = (int64_t)(S / 16);
  char *dA, *dB, *hA, *hB;
  CK(hipMalloc(&dA, S));
  CK(hipMalloc(&dB, S));
  CK(hipHostMalloc((void**)&hA, S, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&hB, S, hipHostMallocDefault));
  memset(hA, 1, S);
  memset(hB, 2, S);
  CK(hipMemset(dA, 3, S));
  CK(hipMemset(dB, 4, S));
  void *hAd, *hBd;  // device views of the pinned host buffers
  CK(hipHostGetDevicePointer(&hAd, hA, 0));
  CK(hipHostGetDevicePointer(&hBd, hB, 0));
  std::vector<char> pg(S), pg2(S);  // pageable
  memset(pg.data(), 5, S);
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  auto kh2d = [&](int g, hipStream_t s) { hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, s, (v4u*)dA, (const v4u*)hAd, nv); };
  auto kd2h = [&](int g, hipStream_t s) { hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, s, (v4u*)hBd, (const v4u*)dB, nv); };
  auto dh2d = [&](hipStream_t s) { CK(hipMemcpyAsync(dA, hA, S, hipMemcpyHostToDevice, s)); };
  auto dd2h = [&](hipStream_t s) { CK(hipMemcpyAsync(hB, dB, S, hipMemcpyDeviceToHost, s)); };
  auto sync = [&] { CK(hipStreamSynchronize(s1)); CK(hipStreamSynchronize(s2)); };
  struct V {
    std::string name;
    int dirs;  // bytes moved = dirs x S
    std::function<void()> go;
  };
  std::vector<V> vs = {
      {"dma h2d", 1, [&] { dh2d(s1); sync(); }},
      {"dma d2h", 1, [&] { dd2h(s1); sync(); }},
      {"dma h2d + dma d2h (two streams)", 2, [&] { dh2d(s1); dd2h(s2); sync(); }},
  };
  for (int g : {64, 256, 1024}) {
    const std::string gs = " grid " + std::to_string(g);
    vs.push_back({"kern h2d" + gs, 1, [&, g] { kh2d(g, s1); sync(); }});
    vs.push_back({"kern d2h" + gs, 1, [&, g] { kd2h(g, s1); sync(); }});
    vs.push_back({"kern h2d + kern d2h" + gs, 2, [&, g] { kh2d(g, s1); kd2h(g, s2); sync(); }});
    vs.push_back({"dma h2d + kern d2h" + gs, 2, [&, g] { dh2d(s1); kd2h(g, s2); sync(); }});
    vs.push_back({"kern h2d + dma d2h" + gs, 2, [&, g] { kh2d(g, s1); dd2h(s2); sync(); }});
  }
  for (int T : {1, 2, 4, 8}) {
    vs.push_back({"cpu pageable->pinned threads " + std::to_string(T), 1, [&, T] {
                     std::vector<std::thread> th;
                     const size_t per = S / T;
                     for (int t = 0; t < T; t++) th.emplace_back([&, t] { memcpy(hA + t * per, pg.data() + t * per, per); });
                     for (auto& x : th) x.join();
                   }});
    vs.push_back({"cpu pinned->pageable threads " + std::to_string(T), 1, [&, T] {
                     std::vector<std::thread> th;
                     const size_t per = S / T;
                     for (int t = 0; t < T; t++) th.emplace_back([&, t] { memcpy(pg2.data() + t * per, hB + t * per, per); });
                     for (auto& x : th) x.join();
                   }});
  }
  vs.push_back({"dma h2d pageable", 1, [&] { CK(hipMemcpyAsync(dA, pg.data(), S, hipMemcpyHostToDevice, s1)); sync(); }});
  vs.push_back({"dma d2h pageable", 1, [&] { CK(hipMemcpyAsync(pg2.data(), dB, S, hipMemcpyDeviceToHost, s1)); sync(); }});
  vs.push_back({"dma h2d + d2h pageable (two streams)", 2, [&] {
                   CK(hipMemcpyAsync(dA, pg.data(), S, hipMemcpyHostToDevice, s1));
                   CK(hipMemcpyAsync(pg2.data(), dB, S, hipMemcpyDeviceToHost, s2));
                   sync();
                 }});
  // the host pipeline's shape: per chunk, H2D on s1 -> a device copy (the collective's stand-in) on s3
  // -> D2H on s2, chained by events; transfers by DMA or by copy kernels; bytes = S (the e2e S/t)
  hipStream_t s3;
  CK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(2 * 256);
  for (auto& x : ev) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  for (int kern = 0; kern < 2; kern++)
    for (size_t cmib : {4, 8, 16, 32}) {
      const std::string nm = std::string("pipeline ") + (kern ? "kern" : "dma") + " chunk " + std::to_string(cmib) + " MiB";
      vs.push_back({nm, 1, [&, kern, cmib] {
                      const size_t cb = cmib << 20, nch = S / cb;
                      for (size_t c = 0; c < nch; c++) {
                        const size_t o = c * cb;
                        if (kern)
                          hipLaunchKernelGGL(k_copy, dim3(256), dim3(256), 0, s1, (v4u*)(dA + o), (const v4u*)((char*)hAd + o),
                                             (int64_t)(cb / 16));
                        else
                          CK(hipMemcpyAsync(dA + o, hA + o, cb, hipMemcpyHostToDevice, s1));
                        CK(hipEventRecord(ev[2 * c], s1));
                        CK(hipStreamWaitEvent(s3, ev[2 * c], 0));
                        hipLaunchKernelGGL(k_copy, dim3(1024), dim3(256), 0, s3, (v4u*)(dB + o), (const v4u*)(dA + o),
                                           (int64_t)(cb / 16));
                        CK(hipEventRecord(ev[2 * c + 1], s3));
                        CK(hipStreamWaitEvent(s2, ev[2 * c + 1], 0));
                        if (kern)
                          hipLaunchKernelGGL(k_copy, dim3(256), dim3(256), 0, s2, (v4u*)((char*)hBd + o), (const v4u*)(dB + o),
                                             (int64_t)(cb / 16));
                        else
                          CK(hipMemcpyAsync(hB + o, dB + o, cb, hipMemcpyDeviceToHost, s2));
                      }
                      sync();
                      CK(hipStreamSynchronize(s3));
                    }});
    }
  // the same chain with the H2D event recorded only every E chunks: the device copies of a group wait
  // for the group's last H2D (does the per-chunk event cost the H2D engine its idle gap?)
  for (int E : {2, 4})
    for (size_t cmib : {8, 16}) {
      const std::string nm = "pipeline dma chunk " + std::to_string(cmib) + " MiB, H2D event every " + std::to_string(E);
      vs.push_back({nm, 1, [&, E, cmib] {
                      const size_t cb = cmib << 20, nch = S / cb;
                      for (size_t g = 0; g < nch; g += E) {
                        const size_t ge = std::min(nch, g + E);
                        for (size_t c = g; c < ge; c++) CK(hipMemcpyAsync(dA + c * cb, hA + c * cb, cb, hipMemcpyHostToDevice, s1));
                        CK(hipEventRecord(ev[2 * g], s1));
                        CK(hipStreamWaitEvent(s3, ev[2 * g], 0));
                        for (size_t c = g; c < ge; c++) {
                          const size_t o = c * cb;
                          hipLaunchKernelGGL(k_copy, dim3(1024), dim3(256), 0, s3, (v4u*)(dB + o), (const v4u*)(dA + o),
                                             (int64_t)(cb / 16));
                          CK(hipEventRecord(ev[2 * c + 1], s3));
                          CK(hipStreamWaitEvent(s2, ev[2 * c + 1], 0));
                          CK(hipMemcpyAsync(hB + o, dB + o, cb, hipMemcpyDeviceToHost, s2));
                        }
                      }
                      sync();
                      CK(hipStreamSynchronize(s3));
                    }});
    }
  // round 5: the chain with the copies of consecutive chunks on alternating streams (two H2D, two D2H),
  // so one engine's wait on its event chain can overlap the other stream's copy
  hipStream_t s4, s5;
  CK(hipStreamCreateWithFlags(&s4, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s5, hipStreamNonBlocking));
  for (int split : {1, 2})  // 1: two H2D streams only; 2: two H2D and two D2H streams
    for (size_t cmib : {8, 16, 32}) {
      const std::string nm = "pipeline dma chunk " + std::to_string(cmib) + " MiB, alternating " +
                             (split == 1 ? "H2D streams" : "H2D and D2H streams");
      vs.push_back({nm, 1, [&, split, cmib] {
                      const size_t cb = cmib << 20, nch = S / cb;
                      for (size_t c = 0; c < nch; c++) {
                        const size_t o = c * cb;
                        hipStream_t hs = (c & 1) ? s4 : s1, ds = (split == 2 && (c & 1)) ? s5 : s2;
                        CK(hipMemcpyAsync(dA + o, hA + o, cb, hipMemcpyHostToDevice, hs));
                        CK(hipEventRecord(ev[2 * c], hs));
                        CK(hipStreamWaitEvent(s3, ev[2 * c], 0));
                        hipLaunchKernelGGL(k_copy, dim3(1024), dim3(256), 0, s3, (v4u*)(dB + o), (const v4u*)(dA + o),
                                           (int64_t)(cb / 16));
                        CK(hipEventRecord(ev[2 * c + 1], s3));
                        CK(hipStreamWaitEvent(ds, ev[2 * c + 1], 0));
                        CK(hipMemcpyAsync(hB + o, dB + o, cb, hipMemcpyDeviceToHost, ds));
                      }
                      sync();
                      CK(hipStreamSynchronize(s3));
                      CK(hipStreamSynchronize(s4));
                      CK(hipStreamSynchronize(s5));
                    }});
    }
  std::vector<std::vector<double>> t(vs.size());
  for (auto& v : vs) v.go();  // warm: page-in, first-touch mappings
  for (int r = 0; r < rounds; r++)
    for (size_t i = 0; i < vs.size(); i++) {
      const double t0 = now();
      vs[i].go();
      t[i].push_back(now() - t0);
    }
  for (size_t i = 0; i < vs.size(); i++) {
    auto w = t[i];
    std::sort(w.begin(), w.end());
    const double med = w[w.size() / 2];
    printf("{\"variant\": \"%s\", \"bytes\": %zu, \"ms_median\": %.3f, \"GBps_total\": %.2f, \"GBps_each_dir\": %.2f}\n",
           vs[i].name.c_str(), vs[i].dirs * S, med * 1e3, vs[i].dirs * S / med / 1e9, S / med / 1e9);
  }
  return 0;
}
