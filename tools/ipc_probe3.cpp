// ipc_probe3 — large exported allocations: hipMalloc(S), hipIpcGetMemHandle, then a D2D copy of
// S/2 into it, for S = 512 MiB .. 4 GiB; prints the time of each step (one process, one device).
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/ipc_probe3 tools/ipc_probe3.cpp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main(int argc, char** argv) {
  const int exportit = argc > 1 ? atoi(argv[1]) : 1;
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (size_t mib = 512; mib <= 4096; mib *= 2) {
    const size_t S = mib << 20;
    char *src = nullptr, *dst = nullptr;
    auto t = std::chrono::steady_clock::now();
    CK(hipMalloc(&src, S / 2));
    CK(hipMalloc(&dst, S));
    double t_alloc = ms_since(t);
    t = std::chrono::steady_clock::now();
    hipIpcMemHandle_t h;
    if (exportit) CK(hipIpcGetMemHandle(&h, dst));
    double t_exp = ms_since(t);
    t = std::chrono::steady_clock::now();
    CK(hipMemcpyAsync(dst, src, S / 2, hipMemcpyDeviceToDevice, s));
    CK(hipStreamSynchronize(s));
    double t_cp = ms_since(t);
    t = std::chrono::steady_clock::now();
    CK(hipMemcpyAsync(dst + S / 2, src, S / 2, hipMemcpyDeviceToDevice, s));
    CK(hipStreamSynchronize(s));
    double t_cp2 = ms_since(t);
    printf("S=%5zu MiB export=%d: alloc %.2f ms, export %.2f ms, copy S/2 %.2f ms, again (upper half) %.2f ms\n", mib,
           exportit, t_alloc, t_exp, t_cp, t_cp2);
    fflush(stdout);
    CK(hipFree(src));
    CK(hipFree(dst));
  }
  return 0;
}
