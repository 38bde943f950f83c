// va_alias_probe.cpp — does a kernel of one process ever read memory it did not write: another
// process's data, or its own earlier data, when processes share one GPU?
//
// Context (profiles/r01/pytest_gpu_reentry_failure.txt): the one wrong IPC result had
// rank 0's reduce_scatter block computed with rank 0's own send block 0 in place of rank 2's block 0.
// Rank 2's push copy reads offset 0 of ITS send buffer, which the test allocated right after freeing
// every buffer of the previous case (torch.cuda.empty_cache() in every rank process). If a kernel
// can be served a freed page's old translation after the physical page went to another process,
// that copy reads whatever the other process put there — e.g. rank 0's new send buffer.
//
// Two modes, run by N processes at once on GPU 0 (tools/va_alias_probe.sh):
//   steady  buffers allocated once; fill (kernel) -> copy (kernel) -> check (kernel), four streams,
//           each stream with its own buffers (four hardware queues per process)
//   churn   every iteration hipMalloc a buffer, fill it from the host (hipMemcpy H2D, as torch's
//           tensor.cuda() does), check it with a kernel, hipFree it — the pattern of the test workers
// Every word is stamped (rank << 24 | iteration & 0xffffff). The check counts words that differ,
// words stamped by another rank, and words of this rank from another iteration (stale). No IPC, no
// libmpjx: a foreign or stale word is a platform fault independent of the engine.
//   usage: va_alias_probe <rank> <seconds> <steady|churn>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__global__ void k_fill(unsigned* p, size_t n, unsigned v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

__global__ void k_copy(unsigned* d, const unsigned* s, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}

// c[0] = words != want, c[1] = stamped by another rank, c[2] = this rank, another iteration;
// c[3] = the first bad word seen
__global__ void k_check(const unsigned* d, size_t n, unsigned want, unsigned long long* c) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const unsigned w = d[i];
    if (w != want) {
      if (atomicAdd(c, 1ull) == 0) atomicExch(c + 3, (unsigned long long)w);
      atomicAdd(c + ((w >> 24) != (want >> 24) ? 1 : 2), 1ull);
    }
  }
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "probe: %s: %s\n", #x, hipGetErrorString(e_));            \
      return 3;                                                                 \
    }                                                                           \
  } while (0)

static unsigned grid(size_t n) { return (unsigned)((n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024); }

int main(int argc, char** argv) {
  if (argc != 4) {
    fprintf(stderr, "usage: va_alias_probe rank seconds steady|churn\n");
    return 2;
  }
  const unsigned rank = (unsigned)atoi(argv[1]);
  const double secs = atof(argv[2]);
  const bool churn = strncmp(argv[3], "churn", 5) == 0;
  const bool sync_after_fill = strcmp(argv[3], "churn_sync") == 0;  // hipDeviceSynchronize after the H2D fill
  char ev[4096] = "";
  int nev = 0;
  unsigned long long bad_iters = 0;
  CK(hipSetDevice(0));
  const size_t sizes[4] = {4096, (size_t)64 << 10, (size_t)1 << 20, (size_t)16 << 20};  // bytes
  unsigned long long* cnt;
  CK(hipMalloc(&cnt, 4 * sizeof(unsigned long long)));
  CK(hipMemset(cnt, 0, 4 * sizeof(unsigned long long)));
  unsigned long long* one;  // per-iteration counters (churn modes)
  CK(hipMalloc(&one, 4 * sizeof(unsigned long long)));
  hipStream_t st[4];
  for (int i = 0; i < 4; i++) CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
  unsigned *src[4] = {}, *dst[4] = {};
  if (!churn)
    for (int b = 0; b < 4; b++) {
      CK(hipMalloc(&src[b], sizes[b]));
      CK(hipMalloc(&dst[b], sizes[b]));
    }
  std::vector<unsigned> host(sizes[3] / 4);
  CK(hipDeviceSynchronize());
  const auto t0 = std::chrono::steady_clock::now();
  unsigned long long it = 0, launches = 0;
  for (;; it++) {
    if ((it & 15) == 0 && std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > secs) break;
    const int b = (int)(it % 4);  // buffer b lives on stream b
    hipStream_t s = st[b];
    const size_t n = sizes[b] / 4;
    const unsigned v = (rank << 24) | (unsigned)(it & 0xffffff);
    if (churn) {
      unsigned* p = nullptr;
      CK(hipMalloc(&p, sizes[b]));
      for (size_t i = 0; i < n; i++) host[i] = v;
      CK(hipMemcpy(p, host.data(), sizes[b], hipMemcpyHostToDevice));
      if (sync_after_fill) CK(hipDeviceSynchronize());
      CK(hipMemsetAsync(one, 0, 4 * sizeof(unsigned long long), s));
      hipLaunchKernelGGL(k_check, dim3(grid(n)), dim3(256), 0, s, p, n, v, one);
      unsigned long long h1[4];
      CK(hipMemcpyAsync(h1, one, sizeof h1, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      launches += 1;
      if (h1[0]) {  // this iteration saw words it did not write: look again, from the device and the host
        bad_iters++;
        CK(hipMemsetAsync(one, 0, 4 * sizeof(unsigned long long), s));
        hipLaunchKernelGGL(k_check, dim3(grid(n)), dim3(256), 0, s, p, n, v, one);
        unsigned long long h2[4];
        CK(hipMemcpyAsync(h2, one, sizeof h2, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        std::vector<unsigned> back(n);
        CK(hipMemcpy(back.data(), p, sizes[b], hipMemcpyDeviceToHost));
        size_t hb = 0;
        for (size_t i = 0; i < n; i++) hb += back[i] != v;
        if (nev < 6)
          nev += snprintf(ev + strlen(ev), sizeof ev - strlen(ev),
                          "%s{\"it\": %llu, \"bytes\": %zu, \"va\": \"%p\", \"first_check_bad\": %llu, "
                          "\"first_bad_word\": \"0x%08llx\", \"recheck_bad\": %llu, \"host_readback_bad\": %zu}",
                          nev ? ", " : "", it, sizes[b], (void*)p, h1[0], h1[3], h2[0], hb) > 0;
      }
      CK(hipFree(p));
    } else {
      hipLaunchKernelGGL(k_fill, dim3(grid(n)), dim3(256), 0, s, src[b], n, v);
      hipLaunchKernelGGL(k_copy, dim3(grid(n)), dim3(256), 0, s, dst[b], src[b], n);
      hipLaunchKernelGGL(k_check, dim3(grid(n)), dim3(256), 0, s, dst[b], n, v, cnt);
      launches += 3;
      if ((it & 7) == 7) CK(hipStreamSynchronize(s));  // host round trips, as the engine's calls have
    }
  }
  CK(hipDeviceSynchronize());
  unsigned long long hc[4];
  CK(hipMemcpy(hc, cnt, sizeof hc, hipMemcpyDeviceToHost));
  if (churn) {
    printf("{\"rank\": %u, \"mode\": \"%s\", \"iterations\": %llu, \"bad_iterations\": %llu, \"events\": [%s]}\n",
           rank, argv[3], it, bad_iters, ev);
    return bad_iters ? 5 : 0;
  }
  printf("{\"rank\": %u, \"mode\": \"%s\", \"iterations\": %llu, \"launches\": %llu, \"bad_words\": %llu, "
         "\"foreign_rank_words\": %llu, \"stale_own_words\": %llu, \"first_bad\": \"0x%08llx\"}\n",
         rank, argv[3], it, launches, hc[0], hc[1], hc[2], hc[0] ? hc[3] : 0ull);
  return hc[0] ? 5 : 0;
}
