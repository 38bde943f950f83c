// ipc_preflight.cpp — one rank of a throw-away HIP-IPC world, run as a CHILD process by bench.py
// before its own ranks touch the GPU. It maps the peers' staging regions (cross-device when each
// rank sits on its own GPU), runs Allreduce(SUM, DOUBLE) in a push-mode and a pull-mode world and
// over two staging windows, with different data every call (a result read stale from a cache across calls shows),
// and checks every element. Exit 0 = the cross-process direct engine works on this node; anything
// else (error, wrong value, a fault that kills this process) makes the bench skip the IPC engine
// instead of losing the run with it. Then the same in a device-synchronised world (stdout verdict).
//   usage: ipc_preflight <rank> <nranks> <device> <128-byte world id as 256 hex chars>
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

// send_r[i] = (i mod 1000) + 1000 r + 1e6 salt: every partial sum is an integer below 2^53, so the
// result is exact in any combine order and the check needs no order model
static int run(mpjx_comm_t c, int rank, int P, size_t n, const char* mode, int salt) {
  std::vector<double> h(n);
  for (size_t i = 0; i < n; i++) h[i] = (double)(i % 1000) + 1000.0 * rank + 1e6 * salt;
  double *s = nullptr, *d = nullptr;
  if (hipMalloc(&s, n * 8) != hipSuccess || hipMalloc(&d, n * 8) != hipSuccess) {
    fprintf(stderr, "preflight r%d: hipMalloc %zu B failed\n", rank, n * 8);
    return 3;
  }
  if (hipMemcpy(s, h.data(), n * 8, hipMemcpyHostToDevice) != hipSuccess || hipMemset(d, 0, n * 8) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess)
    return 3;
  int rc = mpjx_allreduce(c, s, d, (int64_t)n, MPJX_DOUBLE, MPJX_SUM, 0, nullptr);
  if (rc == 0) rc = mpjx_comm_synchronize(c);
  if (rc != 0) {
    fprintf(stderr, "preflight r%d: allreduce %s n=%zu: %s\n", rank, mode, n, mpjx_last_error());
    return 4;
  }
  if (hipMemcpy(h.data(), d, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  (void)hipFree(s);
  (void)hipFree(d);
  const double base = 1000.0 * P * (P - 1) / 2 + 1e6 * P * salt;
  for (size_t i = 0; i < n; i++)
    if (h[i] != (double)P * (double)(i % 1000) + base) {
      fprintf(stderr, "preflight r%d: allreduce %s n=%zu: element %zu = %.17g\n", rank, mode, n, i, h[i]);
      return 5;
    }
  return 0;
}

int main(int argc, char** argv) {
  if (argc != 5 || strlen(argv[4]) != 2 * sizeof(mpjx_unique_id)) {
    fprintf(stderr, "usage: ipc_preflight rank nranks device id_hex\n");
    return 2;
  }
  const int rank = atoi(argv[1]), P = atoi(argv[2]), dev = atoi(argv[3]);
  mpjx_unique_id id;
  for (size_t i = 0; i < sizeof id; i++) {
    const int hi = hexval(argv[4][2 * i]), lo = hexval(argv[4][2 * i + 1]);
    if (hi < 0 || lo < 0) return 2;
    id.internal[i] = (char)(hi * 16 + lo);
  }
  if (hipSetDevice(dev) != hipSuccess) return 3;
  const char* e = getenv("MPJX_IPC_STAGE_MIB");
  const size_t stage = (size_t)(e && atol(e) > 0 ? atol(e) : 256) << 20;
  // one world per mode (MPJX_IPC_MODE is read at init): push, with a call over two staging windows,
  // then pull
  mpjx_comm_t c = nullptr;
  int rc = 0;
  for (int m = 0; m < 2 && rc == 0; m++) {
    const char* mode = m == 0 ? "push" : "pull";
    setenv("MPJX_IPC_MODE", mode, 1);
    id.internal[1] ^= (char)(m + 1);
    if (mpjx_comm_init_ipc(&c, P, &id, rank, dev) != 0) {
      fprintf(stderr, "preflight r%d: init (%s): %s\n", rank, mode, mpjx_last_error());
      return 4;
    }
    rc = run(c, rank, P, 4099, mode, 3 * m);
    if (rc == 0) rc = run(c, rank, P, 4099, mode, 3 * m + 1);
    if (rc == 0 && m == 0) rc = run(c, rank, P, (stage + (1 << 20)) / 8, mode, 3 * m + 2);  // two windows
    if (mpjx_comm_destroy(c) != 0 && rc == 0) rc = 4;
  }
  if (rc == 0 && rank == 0) printf("ipc preflight ok: P=%d\n", P);
  // The device-synchronised mode (MPJX_IPC_SYNC=device) in a third world: its verdict is printed
  // ("dsync ok" / "dsync failed") and does not change the exit status, so a failure here only drops
  // the bench's ipc_dsync engine. Short wait limit: a flag that never arrives costs seconds.
  if (rc == 0) {
    id.internal[0] ^= 0x5a;
    setenv("MPJX_IPC_MODE", "push", 1);
    setenv("MPJX_IPC_SYNC", "device", 1);
    setenv("MPJX_IPC_TIMEOUT_S", "5", 1);
    c = nullptr;
    int d = mpjx_comm_init_ipc(&c, P, &id, rank, dev) != 0 ? 4 : 0;
    if (d == 0) d = run(c, rank, P, 4099, "push", 5);
    if (d == 0) d = run(c, rank, P, 4099, "push", 6);
    if (d == 0) d = run(c, rank, P, (size_t)1 << 17, "push", 7);
    if (c && d != 4 && mpjx_comm_destroy(c) != 0 && d == 0) d = 4;
    if (d == 0) printf("dsync ok\n");
    else printf("dsync failed: %s\n", mpjx_last_error());
  }
  return rc;
}
