// combine_bench.cpp — the N=1 bench's configs[1] combine (mpjx_combine SUM double, 2 x 256 MiB,
// R operand pairs cycled per launch so no launch reuses the Infinity Cache) from a native process
// with no torch: libmpjx binds /opt/rocm's HIP runtime and RCCL here, as under a JVM, instead of the
// ones torch loads into a Python process. Prints one JSON line with the runtime versions it bound.
// Build: make -C mpjexpress_amd tools      Run: tools/combine_bench [steps=20] [warmup=5] [sets=4]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mpjx.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
#define MK(x) do { int rc_ = (x); if (rc_ != MPJX_SUCCESS) { fprintf(stderr, "%s: %s (%s)\n", #x, mpjx_strerror(rc_), mpjx_last_error()); return 1; } } while (0)

__global__ void k_fill(double* p, long n, unsigned long long seed) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (i + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    p[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
  }
}

int main(int argc, char** argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 20, warmup = argc > 2 ? atoi(argv[2]) : 5;
  const int R = argc > 3 ? atoi(argv[3]) : 4;
  const long n = 256L * (1 << 20) / 8;
  std::vector<double*> io(R), in(R);
  for (int r = 0; r < R; r++) {
    CK(hipMalloc(&io[r], n * 8));
    CK(hipMalloc(&in[r], n * 8));
    k_fill<<<4096, 256>>>(io[r], n, 2 * r + 1);
    k_fill<<<4096, 256>>>(in[r], n, 2 * r + 2);
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(hipDeviceSynchronize());
  for (int i = 0; i < warmup; i++) MK(mpjx_combine(3, 8, io[i % R], in[i % R], n, s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < steps; i++) MK(mpjx_combine(3, 8, io[(warmup + i) % R], in[(warmup + i) % R], n, s));
  CK(hipEventRecord(e1, s));
  CK(hipStreamSynchronize(s));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / steps, alg = 3.0 * n * 8;
  int hv = 0, rv = 0;
  MK(mpjx_runtime_versions(&hv, &rv));
  printf("{\"kernel_us\": %.2f, \"achieved_GBps\": %.1f, \"frac\": %.4f, \"sets\": %d, \"steps\": %d, "
         "\"runtime\": {\"hip_runtime\": %d, \"rccl\": %d}, \"process\": \"native (no torch)\"}\n",
         us, alg / (us * 1e-6) / 1e9, alg / (us * 1e-6) / 8e12, R, steps, hv, rv);
  return 0;
}
