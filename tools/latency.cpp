// latency.cpp — multicore-mode (ranks as threads, one process) Allreduce(SUM, double) latency and
// bandwidth sweep through the C++ mirror (include/mpjx.hpp), without Python in the loop. Each rank
// calls the blocking Allreduce `iters` times per size; the per-call time is the max over ranks of
// the median of its calls; every element of the last result is checked (rank r sends r + 1). Engines: direct (default), and the exchange engine (MPJX_SMP_COPY=1)
// with and without the one-shot small-vector path.
//   build: make -C mpjexpress_amd tools     run: tools/latency [P] [max_MiB]
// `tools/latency ipc P [max_MiB]`: P rank PROCESSES (forked before any HIP call) over the HIP-IPC
// direct engine, push and pull modes; the max over ranks comes from an Allreduce(MAX) of the medians.
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "mpjx.hpp"

using mpi::MPI;
using clk = std::chrono::steady_clock;

// Rank r sends r + 1 in every element, so every element of every result must be P(P+1)/2 exactly
// (small integers: any summation order gives the same double); a mismatch fails the run.
static double run(std::vector<mpi::Intracomm>& w, size_t n, int iters) {
  const int P = (int)w.size();
  std::vector<double> med(P);
  std::vector<int> bad(P, 0);
  std::vector<std::thread> th;
  for (int r = 0; r < P; r++) {
    th.emplace_back([&, r] {
      (void)hipSetDevice(0);
      const size_t m = std::max<size_t>(n, 1);
      double *s = nullptr, *d = nullptr;
      (void)hipMalloc(&s, m * 8);
      (void)hipMalloc(&d, m * 8);
      std::vector<double> h(m, r + 1.0);
      (void)hipMemcpy(s, h.data(), m * 8, hipMemcpyHostToDevice);
      (void)hipMemset(d, 0, m * 8);
      (void)hipDeviceSynchronize();
      std::vector<double> t;
      for (int i = 0; i < iters + 3; i++) {
        w[r].Barrier();
        auto t0 = clk::now();
        w[r].Allreduce(s, 0, d, 0, (int)n, MPI::DOUBLE, MPI::SUM);
        auto t1 = clk::now();
        if (i >= 3) t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      }
      (void)hipMemcpy(h.data(), d, n * 8, hipMemcpyDeviceToHost);
      const double want = P * (P + 1) / 2.0;
      for (size_t i = 0; i < n; i++) bad[r] += h[i] != want;
      std::sort(t.begin(), t.end());
      med[r] = t[t.size() / 2];
      (void)hipFree(s);
      (void)hipFree(d);
    });
  }
  for (auto& x : th) x.join();
  for (int r = 0; r < P; r++)
    if (bad[r]) {
      fprintf(stderr, "latency: rank %d: %d of %zu result elements wrong\n", r, bad[r], n);
      exit(3);
    }
  return *std::max_element(med.begin(), med.end());
}

// Floor for comparison: one thread, one 8-byte mpjx_combine launch + hipStreamSynchronize.
static double launch_sync_floor() {
  (void)hipSetDevice(0);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  double *a = nullptr, *b = nullptr;
  (void)hipMalloc(&a, 256);
  (void)hipMalloc(&b, 256);
  (void)hipMemset(a, 0, 256);
  (void)hipMemset(b, 0, 256);
  (void)hipDeviceSynchronize();
  std::vector<double> t;
  for (int i = 0; i < 203; i++) {
    auto t0 = clk::now();
    mpi::check(mpjx_combine(MPJX_SUM, MPJX_DOUBLE, a, b, 1, s), "combine");
    (void)hipStreamSynchronize(s);
    auto t1 = clk::now();
    if (i >= 3) t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  std::sort(t.begin(), t.end());
  (void)hipFree(a);
  (void)hipFree(b);
  (void)hipStreamDestroy(s);
  return t[t.size() / 2];
}

static double run_ipc_rank(mpi::Intracomm& c, size_t n, int iters) {
  const size_t m = std::max<size_t>(n, 1);
  double *s = nullptr, *d = nullptr;
  (void)hipMalloc(&s, m * 8);
  (void)hipMalloc(&d, m * 8);
  std::vector<double> h(m, c.Rank() + 1.0);  // every result element must be P(P+1)/2 (as run())
  (void)hipMemcpy(s, h.data(), m * 8, hipMemcpyHostToDevice);
  (void)hipDeviceSynchronize();
  std::vector<double> t;
  for (int i = 0; i < iters + 3; i++) {
    c.Barrier();
    auto t0 = clk::now();
    c.Allreduce(s, 0, d, 0, (int)n, MPI::DOUBLE, MPI::SUM);
    auto t1 = clk::now();
    if (i >= 3) t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  std::sort(t.begin(), t.end());
  (void)hipMemcpy(h.data(), d, n * 8, hipMemcpyDeviceToHost);
  const double want = c.Size() * (c.Size() + 1) / 2.0;
  for (size_t i = 0; i < n; i++)
    if (h[i] != want) {
      fprintf(stderr, "latency ipc: rank %d: element %zu = %g, want %g\n", c.Rank(), i, h[i], want);
      _exit(3);
    }
  (void)hipFree(s);
  (void)hipFree(d);
  std::vector<double> med{t[t.size() / 2]}, mx(1);
  c.Allreduce(med, 0, mx, 0, 1, MPI::DOUBLE, MPI::MAX);
  return mx[0];
}

static int ipc_main(int P, size_t max_mib) {
  mpjx_unique_id id;
  FILE* f = fopen("/dev/urandom", "rb");
  if (!f || fread(&id, sizeof id, 1, f) != 1) return 2;
  fclose(f);
  std::vector<pid_t> kids;
  for (int r = 0; r < P; r++) {
    pid_t pid = fork();
    if (pid == 0) {  // no HIP call happened in the parent
      (void)hipSetDevice(0);
      setenv("MPJX_IPC_OVERSUBSCRIBE", "1", 1);  // ranks share one GPU; buffers allocated once
      setenv("MPJX_IPC_MODE", "push", 1);  // read at init: one world per mode
      mpi::Intracomm c = mpi::InitIPC(r, P, 0, id);
      mpjx_unique_id id2 = id;
      id2.internal[0] ^= 0x5a;
      setenv("MPJX_IPC_MODE", "pull", 1);
      mpi::Intracomm cp = mpi::InitIPC(r, P, 0, id2);
      if (r == 0)
        printf("{\"P\": %d, \"engine\": \"ipc (rank processes, one device)\", \"op\": \"SUM\", \"type\": "
               "\"DOUBLE\", \"unit\": \"us per call (max over ranks of median)\", \"rows\": [\n", P);
      bool first = true;
      std::vector<size_t> sizes;  // 8 B x 8^k, plus configs[0]'s 1 MiB vector
      for (size_t bytes = 8; bytes <= (max_mib << 20); bytes *= 8) sizes.push_back(bytes);
      if (max_mib >= 1) sizes.push_back((size_t)1 << 20);
      std::sort(sizes.begin(), sizes.end());
      for (size_t bytes : sizes) {
        const size_t n = bytes / 8;
        const int iters = bytes <= (1 << 20) ? 200 : bytes <= (64 << 20) ? 30 : 10;
        const double push = run_ipc_rank(c, n, iters);
        const double pull = run_ipc_rank(cp, n, iters);
        if (r == 0) {
          printf("%s  {\"bytes\": %zu, \"push_us\": %.2f, \"pull_us\": %.2f, \"push_algbw_GBps\": %.2f}",
                 first ? "" : ",\n", bytes, push, pull, bytes / push / 1e3);
          fflush(stdout);
        }
        first = false;
      }
      if (r == 0) printf("\n]}\n");
      fflush(stdout);
      _exit(0);
    }
    kids.push_back(pid);
  }
  int bad = 0;
  for (pid_t k : kids) {
    int st = 0;
    waitpid(k, &st, 0);
    bad += !WIFEXITED(st) || WEXITSTATUS(st) != 0;
  }
  return bad ? 1 : 0;
}

int main(int argc, char** argv) {
  if (argc > 2 && std::string(argv[1]) == "ipc") return ipc_main(atoi(argv[2]), argc > 3 ? (size_t)atol(argv[3]) : 256);
  const int P = argc > 1 ? atoi(argv[1]) : 4;
  const size_t max_mib = argc > 2 ? (size_t)atol(argv[2]) : 256;
  const double floor_us = launch_sync_floor();
  auto w = mpi::smp_world(P, std::vector<int>(P, 0));
  printf("{\"P\": %d, \"op\": \"SUM\", \"type\": \"DOUBLE\", \"unit\": \"us per call (max over ranks of median)\", "
         "\"single_thread_launch_sync_floor_us\": %.2f, \"rows\": [\n", P, floor_us);
  bool first = true;
  std::vector<size_t> sizes;  // 8 B x 8^k, plus configs[0]'s 1 MiB vector
  for (size_t bytes = 8; bytes <= (max_mib << 20); bytes *= 8) sizes.push_back(bytes);
  if (max_mib >= 1) sizes.push_back((size_t)1 << 20);
  std::sort(sizes.begin(), sizes.end());
  for (size_t bytes : sizes) {
    const size_t n = bytes / 8;
    const int iters = bytes <= (1 << 20) ? 200 : bytes <= (64 << 20) ? 30 : 10;
    unsetenv("MPJX_SMP_COPY");
    unsetenv("MPJX_ONESHOT_KIB");
    const double direct = run(w, n, iters);
    setenv("MPJX_SMP_COPY", "1", 1);
    setenv("MPJX_ONESHOT_KIB", "0", 1);
    const double two = run(w, n, iters);
    setenv("MPJX_ONESHOT_KIB", "1048576", 1);
    const double one = run(w, n, iters);
    unsetenv("MPJX_SMP_COPY");
    unsetenv("MPJX_ONESHOT_KIB");
    printf("%s  {\"bytes\": %zu, \"direct_us\": %.2f, \"exchange_us\": %.2f, \"oneshot_us\": %.2f, "
           "\"direct_algbw_GBps\": %.2f}",
           first ? "" : ",\n", bytes, direct, two, one, bytes / direct / 1e3);
    first = false;
    fflush(stdout);
  }
  printf("\n]}\n");
  return 0;
}
