// ipc_stress.cpp — one rank of a HIP-IPC world that runs many Allreduce / ragged Reduce_scatter calls
// back to back with new data and a new block layout every call, and checks every element of every
// result. It looks for results read stale across calls: a staging slot another rank rewrote through
// its IPC mapping while this rank's L2 still holds the previous call's lines.
//   usage: ipc_stress <rank> <nranks> <device> <world id, 256 hex chars> <iterations>
// Environment: MPJX_IPC_MODE push|pull, MPJX_IPC_STAGE_ALLOC (see mpjx_ipc.hip). Exit 0 = no mismatch.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mpjx.h"

static int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

static unsigned long long mix(unsigned long long x) {  // splitmix64: the same layout on every rank
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// x_r[i] = (i*7 + it) mod 4096 + 4096 r: integer partial sums below 2^53, exact in any order
static double val(size_t i, int r, int it) { return (double)((i * 7 + (size_t)it) % 4096) + 4096.0 * r; }

int main(int argc, char** argv) {
  if (argc != 6 || strlen(argv[4]) != 2 * sizeof(mpjx_unique_id)) {
    fprintf(stderr, "usage: ipc_stress rank nranks device id_hex iterations\n");
    return 2;
  }
  const int rank = atoi(argv[1]), P = atoi(argv[2]), dev = atoi(argv[3]), iters = atoi(argv[5]);
  mpjx_unique_id id;
  for (size_t i = 0; i < sizeof id; i++) {
    const int hi = hexval(argv[4][2 * i]), lo = hexval(argv[4][2 * i + 1]);
    if (hi < 0 || lo < 0) return 2;
    id.internal[i] = (char)(hi * 16 + lo);
  }
  if (hipSetDevice(dev) != hipSuccess) return 3;
  mpjx_comm_t c = nullptr;
  if (mpjx_comm_init_ipc(&c, P, &id, rank, dev) != 0) {
    fprintf(stderr, "stress r%d: init: %s\n", rank, mpjx_last_error());
    return 4;
  }
  const size_t nmax = 1 << 17;  // 1 MiB of doubles
  double *s = nullptr, *d = nullptr;
  if (hipMalloc(&s, nmax * 8) != hipSuccess || hipMalloc(&d, nmax * 8) != hipSuccess) return 3;
  std::vector<double> h(nmax), g(nmax);
  long bad_calls = 0, bad_elems = 0;
  // MPJX_STRESS_REALLOC=1: free and reallocate both buffers every call (the same virtual addresses
  // come back in every rank process, as a caching allocator's do after empty_cache())
  const char* ra = getenv("MPJX_STRESS_REALLOC");
  const bool realloc_each = ra && *ra == '1';
  for (int it = 0; it < iters; it++) {
    if (realloc_each && it) {
      (void)hipFree(s);
      (void)hipFree(d);
      s = d = nullptr;
      if (hipMalloc(&s, nmax * 8) != hipSuccess || hipMalloc(&d, nmax * 8) != hipSuccess) return 3;
    }
    const unsigned long long k = mix(0x5354524553ull + (unsigned long long)it);
    const bool rs = (k & 1) != 0;
    size_t n = 1 + (size_t)(mix(k) % nmax);
    std::vector<int64_t> rc(P);
    size_t lo = 0, m = n;
    if (rs) {  // ragged recvcounts, one block empty
      n = 0;
      for (int j = 0; j < P; j++) {
        rc[j] = (int64_t)(mix(k + 17 + (unsigned long long)j) % (nmax / P));
        if (j == (int)((k >> 8) % (unsigned long long)P)) rc[j] = 0;
        if (j < rank) lo += (size_t)rc[j];
        n += (size_t)rc[j];
      }
      m = (size_t)rc[rank];
    }
    for (size_t i = 0; i < n; i++) h[i] = val(i, rank, it);
    if (hipMemcpy(s, h.data(), n * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(d, 0xff, nmax * 8) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
      return 3;
    int e = rs ? mpjx_reduce_scatter(c, s, d, rc.data(), MPJX_DOUBLE, MPJX_SUM, 0, nullptr)
               : mpjx_allreduce(c, s, d, (int64_t)n, MPJX_DOUBLE, MPJX_SUM, 0, nullptr);
    if (e == 0) e = mpjx_comm_synchronize(c);
    if (e != 0) {
      fprintf(stderr, "stress r%d it %d: %s\n", rank, it, mpjx_last_error());
      return 4;
    }
    if (m && hipMemcpy(g.data(), d, m * 8, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    long b = 0;
    size_t first = 0;
    double delta = 0;
    for (size_t i = 0; i < m; i++) {
      double want = 0;
      for (int r = 0; r < P; r++) want += val(lo + i, r, it);
      if (g[i] != want && b++ == 0) first = i, delta = g[i] - want;
    }
    if (b) {
      // one rank's contribution replaced by rank q's at the same index shows as 4096 (q - j)
      if (bad_calls < 8)
        fprintf(stderr, "stress r%d it %d %s n=%zu m=%zu: %ld bad, first at %zu, off by %.17g (%.3f x 4096) %p\n",
                rank, it, rs ? "reduce_scatter" : "allreduce", n, m, b, first, delta, delta / 4096, (void*)s);
      bad_calls++;
      bad_elems += b;
    }
  }
  (void)hipFree(s);
  (void)hipFree(d);
  if (mpjx_comm_destroy(c) != 0) return 4;
  printf("rank %d: %d calls, %ld bad calls, %ld bad elements\n", rank, iters, bad_calls, bad_elems);
  return bad_calls ? 5 : 0;
}
