// rccl_preflight.cpp — one rank of a throw-away RCCL world, run as a CHILD process by bench.py before
// its own ranks touch the GPU (one world per engine variant, so a fault, hang or wrong result in one
// variant costs that variant only). The first P > 1 RCCL execution of libmpjx's exchange engine —
// ncclAllToAll(v) / ncclAllGather / grouped ncclSend/ncclRecv standing in for the edges of
// MST_Reduce (src/mpi/PureIntracomm.java:1966-1985) — then happens here, not in the measuring ranks.
//
// Per variant: Allreduce(SUM, DOUBLE) on an equal-block vector and a ragged one (for the chunk
// pipelines: two full chunks plus a ragged tail), twice each with new data, every element checked
// against the MST(0) grouping recomputed on the host from every rank's input; Reduce_scatter(BAND,
// INT) with equal and ragged recvcounts and Scan(BXOR, INT), every element checked. Exit 0 = the
// variant works on this node; rank 0 prints "rccl preflight ok: <variant> P=<P>".
//
//   usage: rccl_preflight <rank> <nranks> <device> <variant> <uid file>
//   variant: rccl | rccl_skew | rccl_p2p | rccl_pipe32 | rccl_pipe64 | rccl_native (the bench's engine names)
// Rank 0 creates the RCCL unique id and publishes it atomically as <uid file> (same node: the bench
// runs one process per GPU of ONE node); the other ranks wait for it. MPJX_PREFLIGHT_FAIL=<variant>[,...]
// makes the child fail that variant before touching the GPU (tests of the skip path).
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mpjx.h"

namespace {

uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
// element i of rank r's input for call `salt`: U[-1, 1) doubles (53 random bits), order-sensitive sums
double gen_d(int salt, int r, uint64_t i) {
  const uint64_t b = splitmix(((uint64_t)salt << 48) ^ ((uint64_t)r << 40) ^ i);
  return (double)(b >> 11) * 0x1.0p-52 - 1.0;
}
uint32_t gen_u(int salt, int r, uint64_t i) { return (uint32_t)splitmix(((uint64_t)salt << 48) ^ ((uint64_t)r << 40) ^ i); }

// MST_Reduce grouping (PureIntracomm.java:1943-1992): the half holding `root` is the accumulator, the
// other half's sub-root result is folded in as acc = recv + acc
double mst(const double* v, int l, int r, int root) {
  if (l == r) return v[l];
  const int mid = (l + r) / 2;
  if (root <= mid) {
    const double own = mst(v, l, mid, root), other = mst(v, mid + 1, r, r);
    return other + own;
  }
  const double own = mst(v, mid + 1, r, root), other = mst(v, l, mid, l);
  return other + own;
}

int g_rank = 0;

int bad(const char* what, const char* detail) {
  fprintf(stderr, "rccl preflight r%d: %s: %s\n", g_rank, what, detail);
  return 4;
}

int allreduce_check(mpjx_comm_t c, int P, size_t n, int salt) {
  std::vector<double> h(n), got(n);
  for (size_t i = 0; i < n; i++) h[i] = gen_d(salt, g_rank, i);
  double *s = nullptr, *d = nullptr;
  if (hipMalloc(&s, n * 8) != hipSuccess || hipMalloc(&d, n * 8) != hipSuccess) return bad("hipMalloc", "failed");
  int rc = 0;
  if (hipMemcpy(s, h.data(), n * 8, hipMemcpyHostToDevice) != hipSuccess || hipMemset(d, 0, n * 8) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess)
    rc = bad("staging", "hip copy failed");
  if (rc == 0 && (mpjx_allreduce(c, s, d, (int64_t)n, MPJX_DOUBLE, MPJX_SUM, 0, nullptr) != 0 ||
                  mpjx_comm_synchronize(c) != 0))
    rc = bad("allreduce", mpjx_last_error());
  if (rc == 0 && hipMemcpy(got.data(), d, n * 8, hipMemcpyDeviceToHost) != hipSuccess) rc = bad("read-back", "failed");
  (void)hipFree(s);
  (void)hipFree(d);
  if (rc) return rc;
  std::vector<double> v(P);
  for (size_t i = 0; i < n; i++) {
    for (int r = 0; r < P; r++) v[r] = gen_d(salt, r, i);
    const double e = mst(v.data(), 0, P - 1, 0);
    if (memcmp(&e, &got[i], 8) != 0) {
      char m[160];
      snprintf(m, sizeof m, "n=%zu salt=%d element %zu = %.17g, MST(0) = %.17g", n, salt, i, got[i], e);
      return bad("allreduce mismatch", m);
    }
  }
  return 0;
}

// Allreduce(SUM, LONG) of random 64-bit words: Java's wrap-around sum, any order (the rccl_native
// variant's integer path: one ncclAllReduce at every P)
int allreduce_long_check(mpjx_comm_t c, int P, size_t n, int salt) {
  std::vector<int64_t> h(n), got(n);
  for (size_t i = 0; i < n; i++) h[i] = (int64_t)splitmix(((uint64_t)salt << 48) ^ ((uint64_t)g_rank << 40) ^ i);
  int64_t *s = nullptr, *d = nullptr;
  if (hipMalloc(&s, n * 8) != hipSuccess || hipMalloc(&d, n * 8) != hipSuccess) return bad("hipMalloc", "failed");
  int rc = 0;
  if (hipMemcpy(s, h.data(), n * 8, hipMemcpyHostToDevice) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    rc = bad("staging", "hip copy failed");
  if (rc == 0 && (mpjx_allreduce(c, s, d, (int64_t)n, MPJX_LONG, MPJX_SUM, 0, nullptr) != 0 ||
                  mpjx_comm_synchronize(c) != 0))
    rc = bad("allreduce long", mpjx_last_error());
  if (rc == 0 && hipMemcpy(got.data(), d, n * 8, hipMemcpyDeviceToHost) != hipSuccess) rc = bad("read-back", "failed");
  (void)hipFree(s);
  (void)hipFree(d);
  if (rc) return rc;
  for (size_t i = 0; i < n; i++) {
    uint64_t e = 0;
    for (int r = 0; r < P; r++) e += splitmix(((uint64_t)salt << 48) ^ ((uint64_t)r << 40) ^ i);
    if ((uint64_t)got[i] != e) {
      char m[128];
      snprintf(m, sizeof m, "n=%zu element %zu = %016llx, expected %016llx", n, i, (unsigned long long)got[i],
               (unsigned long long)e);
      return bad("allreduce long mismatch", m);
    }
  }
  return 0;
}

int reduce_scatter_check(mpjx_comm_t c, int P, int64_t per, int salt) {
  std::vector<int64_t> rc(P, per);
  const int64_t total = per * P;
  std::vector<uint32_t> h(total), got(per);
  for (int64_t i = 0; i < total; i++) h[i] = gen_u(salt, g_rank, i) | gen_u(salt + 1, g_rank, i);  // p(bit)=3/4
  uint32_t *s = nullptr, *d = nullptr;
  if (hipMalloc(&s, total * 4) != hipSuccess || hipMalloc(&d, per * 4 + 4) != hipSuccess) return bad("hipMalloc", "failed");
  int e = 0;
  if (hipMemcpy(s, h.data(), total * 4, hipMemcpyHostToDevice) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    e = bad("staging", "hip copy failed");
  if (e == 0 && (mpjx_reduce_scatter(c, s, d, rc.data(), MPJX_INT, MPJX_BAND, 0, nullptr) != 0 ||
                 mpjx_comm_synchronize(c) != 0))
    e = bad("reduce_scatter", mpjx_last_error());
  if (e == 0 && hipMemcpy(got.data(), d, per * 4, hipMemcpyDeviceToHost) != hipSuccess) e = bad("read-back", "failed");
  (void)hipFree(s);
  (void)hipFree(d);
  if (e) return e;
  for (int64_t i = 0; i < per; i++) {
    const int64_t g = (int64_t)g_rank * per + i;
    uint32_t x = ~0u;
    for (int r = 0; r < P; r++) x &= gen_u(salt, r, g) | gen_u(salt + 1, r, g);
    if (x != got[i]) {
      char m[128];
      snprintf(m, sizeof m, "per=%lld element %lld = %08x, expected %08x", (long long)per, (long long)i, got[i], x);
      return bad("reduce_scatter mismatch", m);
    }
  }
  return 0;
}

int scan_check(mpjx_comm_t c, size_t n, int salt) {
  std::vector<uint32_t> h(n), got(n);
  for (size_t i = 0; i < n; i++) h[i] = gen_u(salt, g_rank, i);
  uint32_t *s = nullptr, *d = nullptr;
  if (hipMalloc(&s, n * 4) != hipSuccess || hipMalloc(&d, n * 4) != hipSuccess) return bad("hipMalloc", "failed");
  int e = 0;
  if (hipMemcpy(s, h.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    e = bad("staging", "hip copy failed");
  if (e == 0 && (mpjx_scan(c, s, d, (int64_t)n, MPJX_INT, MPJX_BXOR, 0, nullptr) != 0 || mpjx_comm_synchronize(c) != 0))
    e = bad("scan", mpjx_last_error());
  if (e == 0 && hipMemcpy(got.data(), d, n * 4, hipMemcpyDeviceToHost) != hipSuccess) e = bad("read-back", "failed");
  (void)hipFree(s);
  (void)hipFree(d);
  if (e) return e;
  for (size_t i = 0; i < n; i++) {
    uint32_t x = 0;
    for (int r = 0; r <= g_rank; r++) x ^= gen_u(salt, r, i);
    if (x != got[i]) {
      char m[128];
      snprintf(m, sizeof m, "n=%zu element %zu = %08x, expected %08x", n, i, got[i], x);
      return bad("scan mismatch", m);
    }
  }
  return 0;
}

bool forced_fail(const std::string& variant) {
  const char* e = getenv("MPJX_PREFLIGHT_FAIL");
  if (!e) return false;
  const std::string l = std::string(",") + e + ",";
  return l.find("," + variant + ",") != std::string::npos || l.find(",all,") != std::string::npos;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 6) {
    fprintf(stderr, "usage: rccl_preflight rank nranks device variant uid_file\n");
    return 2;
  }
  const int rank = atoi(argv[1]), P = atoi(argv[2]), dev = atoi(argv[3]);
  const std::string variant = argv[4], uid_path = argv[5];
  g_rank = rank;
  if (forced_fail(variant)) {
    fprintf(stderr, "rccl preflight r%d: %s: forced failure (MPJX_PREFLIGHT_FAIL)\n", rank, variant.c_str());
    return 7;
  }
  size_t chunk = 0;  // the engine variant's per-call settings, as bench.py passes them to the library
  if (variant == "rccl_skew") {
    setenv("MPJX_SLOT_SKEW", "4096", 1);
  } else if (variant == "rccl_p2p") {
    setenv("MPJX_RCCL_P2P", "1", 1);
  } else if (variant.rfind("rccl_pipe", 0) == 0) {
    chunk = (size_t)atoi(variant.c_str() + 9) << 20;
    if (!chunk) return bad("variant", variant.c_str());
    setenv("MPJX_PIPE_CHUNK_MIB", variant.c_str() + 9, 1);
  } else if (variant == "rccl_native") {
    setenv("MPJX_RCCL_NATIVE", "1", 1);  // one ncclAllReduce where the result is order-free (P <= 2 for doubles)
  } else if (variant != "rccl") {
    return bad("unknown variant", variant.c_str());
  }
  if (P == 1) setenv("MPJX_P1_EXCHANGE", "1", 1);  // world size 1: still run the transport's calls
  if (!getenv("MPJX_RCCL_TIMEOUT_S")) setenv("MPJX_RCCL_TIMEOUT_S", "30", 1);
  if (hipSetDevice(dev) != hipSuccess) return bad("hipSetDevice", "failed");

  mpjx_unique_id id;
  if (rank == 0) {
    if (mpjx_get_unique_id(&id) != 0) return bad("mpjx_get_unique_id", mpjx_last_error());
    const std::string tmp = uid_path + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f || fwrite(&id, sizeof id, 1, f) != 1 || fclose(f) != 0 || rename(tmp.c_str(), uid_path.c_str()) != 0)
      return bad("uid file", uid_path.c_str());
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      FILE* f = fopen(uid_path.c_str(), "rb");
      if (f) {
        const size_t k = fread(&id, sizeof id, 1, f);
        fclose(f);
        if (k == 1) break;
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) return bad("uid file", "not published in 60 s");
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
  }
  mpjx_comm_t c = nullptr;
  if (mpjx_comm_init_rank(&c, P, &id, rank, dev) != 0) return bad("mpjx_comm_init_rank", mpjx_last_error());
  // equal blocks (one ncclAllToAll + in-place ncclAllGather) and ragged (ncclAllToAllv / grouped
  // send/recv); for the pipelines two whole chunks plus a ragged third
  const size_t unit = (size_t)P * 256 / 8;
  const size_t n_eq = chunk ? 2 * chunk / 8 : ((size_t)4 << 20) / 8 / unit * unit * P;
  const size_t sizes[2] = {n_eq, n_eq + 4099};
  int rc = 0, salt = 1;
  for (size_t n : sizes)
    for (int rep = 0; rep < 2 && rc == 0; rep++) rc = allreduce_check(c, P, n, salt++);
  if (rc == 0 && variant == "rccl_native") rc = allreduce_long_check(c, P, ((size_t)1 << 20) + 5, 60);
  if (rc == 0) rc = reduce_scatter_check(c, P, 262144, 50);
  if (rc == 0) rc = reduce_scatter_check(c, P, 262147, 52);
  if (rc == 0) rc = scan_check(c, ((size_t)1 << 20) + 3, 54);
  if (mpjx_comm_destroy(c) != 0 && rc == 0) rc = bad("mpjx_comm_destroy", mpjx_last_error());
  if (rc == 0 && rank == 0) printf("rccl preflight ok: %s P=%d\n", variant.c_str(), P);
  return rc;
}
