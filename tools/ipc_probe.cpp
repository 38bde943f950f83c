// ipc_probe — checks the HIP IPC facilities a cross-process direct engine would rely on, with two
// processes on one device (fork before any HIP call):
//   * HIP_POINTER_ATTRIBUTE_BUFFER_ID is unique per allocation (free + re-malloc at the same VA gives
//     a new id), so a peer-side mapping cache keyed by it cannot go stale;
//   * hipIpcGetMemHandle of an interior pointer vs. the allocation base (offset semantics);
//   * hipIpcOpenMemHandle in the other process: data written by one is read by the other;
//   * cost of get/open.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/ipc_probe tools/ipc_probe.cpp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Msg {
  hipIpcMemHandle_t h_base, h_inner;
  size_t inner_off;
};

int main() {
  int p2c[2], c2p[2];
  if (pipe(p2c) || pipe(c2p)) return 1;
  pid_t pid = fork();
  if (pid == 0) {  // child: opens the parent's memory
    Msg m;
    if (read(p2c[0], &m, sizeof m) != (ssize_t)sizeof m) return 2;
    CK(hipSetDevice(0));
    void *pb = nullptr, *pi = nullptr;
    double t0 = now_us();
    CK(hipIpcOpenMemHandle(&pb, m.h_base, hipIpcMemLazyEnablePeerAccess));
    double t1 = now_us();
    hipError_t e2 = hipIpcOpenMemHandle(&pi, m.h_inner, hipIpcMemLazyEnablePeerAccess);
    printf("child: open(base) %.1f us -> %p; open(inner) -> %s %p (diff %td, parent offset %zu)\n", t1 - t0, pb,
           hipGetErrorString(e2), pi, (char*)pi - (char*)pb, m.inner_off);
    unsigned long long first = 0, at_off = 0;
    CK(hipMemcpy(&first, pb, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&at_off, (char*)pb + m.inner_off, 8, hipMemcpyDeviceToHost));
    printf("child: base[0]=%llx base[off]=%llx\n", first, at_off);
    unsigned long long v = 0xC0FFEEull;
    CK(hipMemcpy((char*)pb + 8, &v, 8, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    char ok = 1;
    if (write(c2p[1], &ok, 1) != 1) return 3;
    if (read(p2c[0], &ok, 1) != 1) return 4;  // parent done checking
    CK(hipIpcCloseMemHandle(pb));
    if (e2 == hipSuccess) (void)hipIpcCloseMemHandle(pi);
    return 0;
  }
  CK(hipSetDevice(0));
  const size_t sz = 64 << 20;
  char* a = nullptr;
  CK(hipMalloc(&a, sz));
  unsigned long long id1 = 0, id2 = 0, id3 = 0;
  hipError_t ea = hipPointerGetAttribute(&id1, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)a);
  hipError_t eb = hipPointerGetAttribute(&id2, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)(a + 4096));
  printf("parent: BUFFER_ID base %s %llu, interior %s %llu\n", hipGetErrorString(ea), id1, hipGetErrorString(eb), id2);
  hipDeviceptr_t base = nullptr;
  size_t bsz = 0;
  CK(hipMemGetAddressRange(&base, &bsz, (hipDeviceptr_t)(a + 12345)));
  printf("parent: address range of a+12345: base %p (a %p) size %zu\n", (void*)base, (void*)a, bsz);
  unsigned long long pat[2] = {0x1111ull, 0x2222ull};
  CK(hipMemcpy(a, &pat[0], 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(a + (1 << 20), &pat[1], 8, hipMemcpyHostToDevice));
  Msg m;
  double t0 = now_us();
  CK(hipIpcGetMemHandle(&m.h_base, a));
  double t1 = now_us();
  CK(hipIpcGetMemHandle(&m.h_base, a));
  double t2 = now_us();
  hipError_t ei = hipIpcGetMemHandle(&m.h_inner, a + (1 << 20));
  printf("parent: get handle %.1f us, again %.1f us; interior handle: %s\n", t1 - t0, t2 - t1, hipGetErrorString(ei));
  m.inner_off = 1 << 20;
  if (write(p2c[1], &m, sizeof m) != (ssize_t)sizeof m) return 5;
  char ok = 0;
  if (read(c2p[0], &ok, 1) != 1) return 6;
  unsigned long long back = 0;
  CK(hipMemcpy(&back, a + 8, 8, hipMemcpyDeviceToHost));
  printf("parent: child's write seen: %llx (%s)\n", back, back == 0xC0FFEEull ? "ok" : "WRONG");
  if (write(p2c[1], &ok, 1) != 1) return 7;
  int st = 0;
  waitpid(pid, &st, 0);
  CK(hipFree(a));
  char* b = nullptr;
  CK(hipMalloc(&b, sz));
  CK(hipPointerGetAttribute(&id3, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)b));
  printf("parent: re-malloc same size: %p (old %p) BUFFER_ID %llu (old %llu) -> %s\n", (void*)b, (void*)a, id3, id1,
         id3 != id1 ? "unique" : "REUSED");
  CK(hipFree(b));
  printf("child exit %d\n", WEXITSTATUS(st));
  return WEXITSTATUS(st);
}
