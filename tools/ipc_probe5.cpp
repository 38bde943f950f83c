// ipc_probe5 — two processes on one device export a region each and open each other's AT THE SAME
// TIME (the IPC engine's pattern), for a sequence of sizes, without closing earlier mappings.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/ipc_probe5 tools/ipc_probe5.cpp
#include <hip/hip_runtime.h>
#include <signal.h>
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

static void side(int me, int rfd, int wfd, int nsz, const size_t* sizes) {
  CK(hipSetDevice(0));
  for (int i = 0; i < nsz; i++) {
    const size_t S = sizes[i];
    char* a = nullptr;
    CK(hipMalloc(&a, S));
    hipIpcMemHandle_t mine, theirs;
    CK(hipIpcGetMemHandle(&mine, a));
    if (write(wfd, &mine, sizeof mine) != sizeof mine) exit(2);
    if (read(rfd, &theirs, sizeof theirs) != sizeof theirs) exit(3);
    alarm(20);
    auto t = std::chrono::steady_clock::now();
    void* p = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&p, theirs, hipIpcMemLazyEnablePeerAccess);
    double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    alarm(0);
    printf("side %d: %5zu MiB mutual open %s in %.2f ms\n", me, S >> 20, hipGetErrorString(e), ms);
    fflush(stdout);
    char ok = 1;  // step barrier
    if (write(wfd, &ok, 1) != 1) exit(4);
    if (read(rfd, &ok, 1) != 1) exit(5);
  }
}

int main(int argc, char** argv) {
  int a2b[2], b2a[2];
  if (pipe(a2b) || pipe(b2a)) return 1;
  const size_t sizes[] = {512ull << 20, 1ull << 30, 2ull << 30, 4ull << 30};
  const int nsz = 4;
  pid_t pid = fork();
  if (pid == 0) {
    side(1, a2b[0], b2a[1], nsz, sizes);
    return 0;
  }
  side(0, b2a[0], a2b[1], nsz, sizes);
  int st = 0;
  waitpid(pid, &st, 0);
  printf("side 1 exit %d signal %d\n", WIFEXITED(st) ? WEXITSTATUS(st) : -1, WIFSIGNALED(st) ? WTERMSIG(st) : 0);
  return 0;
}
