// ipc_probe2 — what hipIpcOpenMemHandle returns when the exporter frees an allocation and a new one
// lands at the same virtual address (two processes, one device; fork before any HIP call):
//   step 1: owner allocates A, writes 1; importer opens A's handle and reads
//   step 2: owner frees A, allocates B (same size), writes 2; importer opens B's handle WITHOUT
//           closing A's mapping, reads                  -> stale (1) or fresh (2)?
//   step 3: importer closes every mapping, opens B's handle again, reads -> expect 2
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/ipc_probe2 tools/ipc_probe2.cpp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

static unsigned long long fnv(const void* p, size_t n) {
  unsigned long long h = 1469598103934665603ull;
  for (size_t i = 0; i < n; i++) h = (h ^ ((const unsigned char*)p)[i]) * 1099511628211ull;
  return h;
}

int main() {
  int p2c[2], c2p[2];
  if (pipe(p2c) || pipe(c2p)) return 1;
  const size_t sz = 8 << 20;
  pid_t pid = fork();
  if (pid == 0) {
    CK(hipSetDevice(0));
    hipIpcMemHandle_t h;
    char ok = 1;
    void *ma = nullptr, *mb = nullptr, *mc = nullptr;
    unsigned long long v = 0;
    if (read(p2c[0], &h, sizeof h) != sizeof h) return 2;
    CK(hipIpcOpenMemHandle(&ma, h, hipIpcMemLazyEnablePeerAccess));
    CK(hipMemcpy(&v, ma, 8, hipMemcpyDeviceToHost));
    printf("step1: open A -> %p reads %llu (expect 1)\n", ma, v);
    if (write(c2p[1], &ok, 1) != 1) return 3;
    if (read(p2c[0], &h, sizeof h) != sizeof h) return 4;
    hipError_t e = hipIpcOpenMemHandle(&mb, h, hipIpcMemLazyEnablePeerAccess);
    v = 0;
    if (e == hipSuccess) CK(hipMemcpy(&v, mb, 8, hipMemcpyDeviceToHost));
    printf("step2: open B (A still open) -> %s %p reads %llu (expect 2; 1 = stale) same VA as A: %s\n",
           hipGetErrorString(e), mb, v, mb == ma ? "yes" : "no");
    CK(hipIpcCloseMemHandle(ma));
    if (e == hipSuccess && mb != ma) (void)hipIpcCloseMemHandle(mb);
    hipError_t e3 = hipIpcOpenMemHandle(&mc, h, hipIpcMemLazyEnablePeerAccess);
    v = 0;
    if (e3 == hipSuccess) CK(hipMemcpy(&v, mc, 8, hipMemcpyDeviceToHost));
    printf("step3: close all, open B -> %s %p reads %llu (expect 2)\n", hipGetErrorString(e3), mc, v);
    if (e3 == hipSuccess) (void)hipIpcCloseMemHandle(mc);
    if (write(c2p[1], &ok, 1) != 1) return 5;
    return 0;
  }
  CK(hipSetDevice(0));
  char* a = nullptr;
  CK(hipMalloc(&a, sz));
  unsigned long long one = 1, two = 2;
  CK(hipMemcpy(a, &one, 8, hipMemcpyHostToDevice));
  hipIpcMemHandle_t ha, hb;
  CK(hipIpcGetMemHandle(&ha, a));
  if (write(p2c[1], &ha, sizeof ha) != sizeof ha) return 6;
  char ok;
  if (read(c2p[0], &ok, 1) != 1) return 7;
  CK(hipFree(a));
  char* b = nullptr;
  CK(hipMalloc(&b, sz));
  CK(hipMemcpy(b, &two, 8, hipMemcpyHostToDevice));
  CK(hipIpcGetMemHandle(&hb, b));
  printf("owner: A %p handle %016llx; B %p handle %016llx (%s VA, %s handle)\n", (void*)a, fnv(&ha, sizeof ha),
         (void*)b, fnv(&hb, sizeof hb), a == b ? "same" : "different",
         memcmp(&ha, &hb, sizeof ha) == 0 ? "same" : "different");
  fflush(stdout);
  if (write(p2c[1], &hb, sizeof hb) != sizeof hb) return 8;
  if (read(c2p[0], &ok, 1) != 1) return 9;
  int st = 0;
  waitpid(pid, &st, 0);
  CK(hipFree(b));
  return WEXITSTATUS(st);
}
