// ipc_probe4 — cross-process hipIpcOpenMemHandle of large allocations (two processes, one device):
// the owner exports regions of 512 MiB .. 4 GiB, the importer opens (and closes) each, timed.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/ipc_probe4 tools/ipc_probe4.cpp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

int main() {
  int p2c[2], c2p[2];
  if (pipe(p2c) || pipe(c2p)) return 1;
  const size_t sizes[] = {512ull << 20, 1ull << 30, 1536ull << 20, 2ull << 30, 4ull << 30};
  pid_t pid = fork();
  if (pid == 0) {
    CK(hipSetDevice(0));
    for (size_t S : sizes) {
      hipIpcMemHandle_t h;
      if (read(p2c[0], &h, sizeof h) != sizeof h) return 2;
      alarm(20);
      auto t = std::chrono::steady_clock::now();
      void* p = nullptr;
      hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
      unsigned long long v = 0;
      if (e == hipSuccess) CK(hipMemcpy(&v, (char*)p + S - 8, 8, hipMemcpyDeviceToHost));
      printf("importer: %5zu MiB open %s in %.2f ms, last word %llx\n", S >> 20, hipGetErrorString(e), ms, v);
      fflush(stdout);
      if (e == hipSuccess) CK(hipIpcCloseMemHandle(p));
      alarm(0);
      char ok = 1;
      if (write(c2p[1], &ok, 1) != 1) return 3;
    }
    return 0;
  }
  CK(hipSetDevice(0));
  for (size_t S : sizes) {
    char* a = nullptr;
    CK(hipMalloc(&a, S));
    unsigned long long v = S;
    CK(hipMemcpy(a + S - 8, &v, 8, hipMemcpyHostToDevice));
    hipIpcMemHandle_t h;
    CK(hipIpcGetMemHandle(&h, a));
    if (write(p2c[1], &h, sizeof h) != sizeof h) return 4;
    char ok;
    if (read(c2p[0], &ok, 1) != 1) { printf("owner: importer died at %zu MiB\n", S >> 20); break; }
    CK(hipFree(a));
  }
  int st = 0;
  waitpid(pid, &st, 0);
  printf("importer exit status %d (signal %d)\n", WIFEXITED(st) ? WEXITSTATUS(st) : -1,
         WIFSIGNALED(st) ? WTERMSIG(st) : 0);
  return 0;
}
