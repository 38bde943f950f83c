// mpjx_core.hip — libmpjx entry points that need no communicator: error strings, the datatype and
// (op, datatype) validity tables, the P-way launch dispatcher and mpjx_combine / mpjx_combine_multi.
//
// Reference behaviour followed (file:line in /root/reference):
//   datatype sizes   src/mpi/BasicType.java:50-140
//   worker tables    src/mpi/<Op>Worker.java (which (op, type) pairs throw MPIException)
//   one combine      src/mpi/SumDouble.java:49-67 (createInitialBuffer + perform + getResultant)
#include "mpjx_internal.hpp"

#include <atomic>

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <thread>

using namespace mpjx;

// ---------------------------------------------------------------------------------------------
// errors

static thread_local std::string g_err;

int mpjx::fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

const char* mpjx::type_name(int t) {
  static const char* n[] = {"NULL", "BYTE", "CHAR", "SHORT", "BOOLEAN", "INT", "LONG", "FLOAT", "DOUBLE"};
  static const char* p[] = {"?", "?", "?", "SHORT2", "?", "INT2", "LONG2", "FLOAT2", "DOUBLE2"};
  if (t >= 0 && t <= 8) return n[t];
  if (t >= 0x100 && t <= 0x108) return p[t - 0x100];
  return "UNKNOWN";
}
const char* mpjx::op_name(int o) {
  static const char* n[] = {"?", "MAX", "MIN", "SUM", "PROD", "LAND", "BAND", "LOR", "BOR", "LXOR", "BXOR",
                            "MAXLOC", "MINLOC"};
  return (o >= 1 && o <= 12) ? n[o] : "UNKNOWN";
}
bool mpjx::is_pair(int t) {
  return t == MPJX_SHORT2 || t == MPJX_INT2 || t == MPJX_LONG2 || t == MPJX_FLOAT2 || t == MPJX_DOUBLE2;
}

extern "C" int mpjx_type_size(int type) {
  switch (type) {  // src/mpi/BasicType.java:50-140
    case MPJX_BYTE: case MPJX_BOOLEAN: return 1;
    case MPJX_CHAR: case MPJX_SHORT: return 2;
    case MPJX_INT: case MPJX_FLOAT: return 4;
    case MPJX_LONG: case MPJX_DOUBLE: return 8;
    case MPJX_SHORT2: return 4;
    case MPJX_INT2: case MPJX_FLOAT2: return 8;
    case MPJX_LONG2: case MPJX_DOUBLE2: return 16;
  }
  return 0;
}

extern "C" int mpjx_op_check(int op, int type) {
  if (mpjx_type_size(type) == 0) return fail(MPJX_ERR_ARG, "unknown datatype code %d", type);
  if (op == MPJX_MAXLOC || op == MPJX_MINLOC) {  // Maxloc.java / Minloc.java: pair types only
    if (!is_pair(type)) return fail(MPJX_ERR_OP_TYPE, "MPI.%s: invalid datatype MPI.%s", op_name(op), type_name(type));
    return MPJX_SUCCESS;
  }
  if (is_pair(type))  // the typed workers read a pair array as `count` scalars: not a valid reduction
    return fail(MPJX_ERR_OP_TYPE, "MPI.%s is not supported for MPI.%s", op_name(op), type_name(type));
  switch (op) {
    case MPJX_SUM: case MPJX_PROD: case MPJX_MAX: case MPJX_MIN:  // SumWorker.java:60 etc.
      if (type == MPJX_BOOLEAN)
        return fail(MPJX_ERR_OP_TYPE, "MPI.%s is invalid for MPI.BOOLEAN", op_name(op));
      return MPJX_SUCCESS;
    case MPJX_BAND: case MPJX_BOR: case MPJX_BXOR:  // BandWorker.java:44-62
      if (type == MPJX_BOOLEAN || type == MPJX_FLOAT || type == MPJX_DOUBLE)
        return fail(MPJX_ERR_OP_TYPE, "MPI.%s is not valid for MPI.%s", op_name(op), type_name(type));
      return MPJX_SUCCESS;
    case MPJX_LAND: case MPJX_LOR: case MPJX_LXOR:  // LandWorker.java:48-74
      if (type != MPJX_BOOLEAN)
        return fail(MPJX_ERR_OP_TYPE, "MPI.%s is invalid for MPI.%s", op_name(op), type_name(type));
      return MPJX_SUCCESS;
  }
  return fail(MPJX_ERR_ARG, "unknown op code %d", op);
}

extern "C" int mpjx_version(void) { return MPJX_VERSION; }

extern "C" int mpjx_runtime_versions(int* hip_runtime, int* rccl) {
  if (hip_runtime) HIPCHK(hipRuntimeGetVersion(hip_runtime));
  if (rccl) NCCLCHK(ncclGetVersion(rccl));
  return MPJX_SUCCESS;
}

extern "C" const char* mpjx_strerror(int status) {
  switch (status) {
    case MPJX_SUCCESS: return "success";
    case MPJX_ERR_ARG: return "invalid argument";
    case MPJX_ERR_OP_TYPE: return "operation invalid for datatype";
    case MPJX_ERR_HIP: return "HIP runtime error";
    case MPJX_ERR_RCCL: return "RCCL error";
    case MPJX_ERR_NO_DEVICE: return "no usable gfx950 device";
    case MPJX_ERR_UNSUPPORTED: return "unsupported";
    case MPJX_ERR_INTERNAL: return "internal error";
  }
  return "unknown status";
}

extern "C" const char* mpjx_last_error(void) { return g_err.c_str(); }

extern "C" int mpjx_device_count(int* count) {
  if (!count) return fail(MPJX_ERR_ARG, "count is NULL");
  *count = 0;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return fail(MPJX_ERR_NO_DEVICE, "hipGetDeviceCount failed");
  int ok = 0;
  for (int d = 0; d < n; d++) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, d) == hipSuccess && strncmp(p.gcnArchName, "gfx950", 6) == 0) ok++;
  }
  *count = ok;
  return MPJX_SUCCESS;
}

// ---------------------------------------------------------------------------------------------
// P-way combine dispatch

size_t mpjx::nt_min_bytes() {
  static const size_t b = [] {
    const char* e = getenv("MPJX_NT_MIN_MIB");
    return e && *e ? (size_t)std::max(0L, atol(e)) << 20 : kStreamBytes;
  }();
  return b;
}

size_t mpjx::short_max_bytes() {
  static const size_t b = [] {
    const char* e = getenv("MPJX_SHORT_MAX_MIB");  // negative values clamp to 0 (short forms off)
    return e && *e ? (size_t)std::max(0L, atol(e)) << 20 : kShortBytes;
  }();
  return b;
}

int mpjx::cu_count() {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  cache[dev].store(n, std::memory_order_relaxed);
  return n;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// One kernel launch (P <= MAXP). Chooses the 16-B vector instantiation when every pointer allows it.
int mpjx::launch_pway(int op, int type, unsigned flags, int kind, int P, const PwayArgs& a,
                       hipStream_t s) {
  const int Q = (kind == K_SCAN) ? P : a.nrep;
  bool vec = true;
  for (int p = 0; p < P; p++) vec = vec && aligned16(a.in[p]);
  for (int q = 0; q < Q; q++) vec = vec && aligned16(a.out[q]);
  hipError_t e;
  if ((flags & MPJX_FLAG_FAITHFUL) && (op == MPJX_BOR || op == MPJX_BXOR)) {
    e = launch_keep(type, kind, P, a, s, vec);
  } else {
    switch (op) {
      case MPJX_SUM: e = launch_sum(type, kind, P, a, s, vec); break;
      case MPJX_PROD: e = launch_prod(type, kind, P, a, s, vec); break;
      case MPJX_MAX: e = launch_max(type, kind, P, a, s, vec); break;
      case MPJX_MIN: e = launch_min(type, kind, P, a, s, vec); break;
      case MPJX_BAND: case MPJX_BOR: case MPJX_BXOR:
        e = launch_bitwise(op, type, kind, P, a, s, vec);
        break;
      case MPJX_LAND: case MPJX_LOR: case MPJX_LXOR: e = launch_logical(op, kind, P, a, s, vec); break;
      case MPJX_MAXLOC: case MPJX_MINLOC: e = launch_loc(op, type, kind, P, a, s, vec); break;
      default: return fail(MPJX_ERR_ARG, "unknown op code %d", op);
    }
  }
  if (e == hipErrorNoBinaryForGpu || e == hipErrorInvalidDeviceFunction)
    return fail(MPJX_ERR_NO_DEVICE, "no gfx950 kernel image for this device: %s", hipGetErrorString(e));
  if (e != hipSuccess) return fail(MPJX_ERR_HIP, "kernel launch (op %s, type %s, kind %d, P %d): %s",
                                   op_name(op), type_name(type), kind, P, hipGetErrorString(e));
  return MPJX_SUCCESS;
}

// Kernels must never dereference memory the GPU cannot reach (a pageable host pointer faults the
// device): every user buffer handed to a device entry point is looked up first.
int mpjx::check_dev_ptr(const void* p, const char* what) {
  if (!p) return MPJX_SUCCESS;  // NULL is the callers' business (allowed where not significant)
  hipPointerAttribute_t at{};
  const hipError_t e = hipPointerGetAttributes(&at, p);
  if (e != hipSuccess || at.type == hipMemoryTypeUnregistered) {  // pageable host memory (ROCm 7.2: type 0)
    (void)hipGetLastError();
    return fail(MPJX_ERR_ARG, "%s %p is not GPU-accessible memory (use the *_host entry points for host arrays)",
                what, p);
  }
  if (at.type == hipMemoryTypeHost && at.devicePointer != p)  // hipHostRegister'd: the device alias differs
    return fail(MPJX_ERR_ARG, "%s %p is registered host memory: pass its device pointer %p", what, p,
                at.devicePointer);
  return MPJX_SUCCESS;
}

extern "C" int mpjx_combine(int op, int type, void* inout, const void* in, int64_t count, void* stream) {
  CHK(mpjx_op_check(op, type));
  if (count < 0) return fail(MPJX_ERR_ARG, "negative count");
  if (count == 0) return MPJX_SUCCESS;
  if (!inout || !in) return fail(MPJX_ERR_ARG, "NULL buffer");
  CHK(check_dev_ptr(inout, "inout"));
  CHK(check_dev_ptr(in, "in"));
  PwayArgs a{};
  a.in[0] = inout;  // acc (arr[i])
  a.in[1] = in;     // in (arr1[i])
  a.out[0] = inout;
  a.n = count;
  return launch_pway(op, type, 0, K_FOLD, 2, a, (hipStream_t)stream);
}

extern "C" int mpjx_combine_multi(int op, int type, int order, int P, const void* const* in, void* const* out,
                                  int64_t count, int root, unsigned flags, void* stream) {
  CHK(mpjx_op_check(op, type));
  if (count < 0 || P < 1 || !in || !out) return fail(MPJX_ERR_ARG, "bad arguments");
  if (order == MPJX_ORDER_MST && (root < 0 || root >= P)) return fail(MPJX_ERR_ARG, "root %d of %d", root, P);
  if (count == 0) return MPJX_SUCCESS;
  const int Q = order == MPJX_ORDER_SCAN ? P : 1;
  for (int p = 0; p < P; p++) {
    if (!in[p]) return fail(MPJX_ERR_ARG, "in[%d] is NULL", p);
    CHK(check_dev_ptr(in[p], "in[]"));
  }
  for (int q = 0; q < Q; q++) {
    if (!out[q]) return fail(MPJX_ERR_ARG, "out[%d] is NULL", q);
    CHK(check_dev_ptr(out[q], "out[]"));
  }
  const int esz = mpjx_type_size(type);
  // P > 8 compositions need temporaries: a call-local device buffer (freed after the stream drains)
  char* tbuf = nullptr;
  size_t tb = 0;
  if (P > MAXP) {
    int levels = 0;
    for (int m = P; m > MAXP; m = (m + 1) / 2) levels++;
    tb = (size_t)(2 * levels + 2) * (((size_t)count * esz + 255) & ~(size_t)255);
    HIPCHK(hipMallocAsync((void**)&tbuf, tb, (hipStream_t)stream));
  }
  TempStack ts{tbuf, tb, 0, (size_t)esz};
  Combine cb{op, type, flags, esz, (hipStream_t)stream, &ts};
  int rc;
  switch (order) {
    case MPJX_ORDER_FOLD: rc = cb.fold(P, in, out[0], count); break;
    case MPJX_ORDER_MST: rc = cb.mst(in, 0, P - 1, root, out[0], count); break;
    case MPJX_ORDER_SCAN: rc = cb.scan(P, in, out, count); break;
    default: rc = fail(MPJX_ERR_ARG, "unknown order %d", order);
  }
  if (tbuf) (void)hipFreeAsync(tbuf, (hipStream_t)stream);
  return rc;
}

extern "C" int mpjx_mpjbuf_combine(int op, int type, void* acc, const void* msg, int64_t msg_bytes, int64_t count,
                                   int* status, unsigned flags, void* stream) {
  CHK(mpjx_op_check(op, type));
  if (count < 0 || msg_bytes < 0) return fail(MPJX_ERR_ARG, "negative count or size");
  if (count == 0) return MPJX_SUCCESS;
  if (!acc || !msg || !status) return fail(MPJX_ERR_ARG, "NULL argument");
  CHK(check_dev_ptr(acc, "acc"));
  CHK(check_dev_ptr(msg, "msg"));
  CHK(check_dev_ptr(status, "status"));
  const hipError_t e = launch_mpjbuf(op, type, (flags & MPJX_FLAG_FAITHFUL) != 0, acc, msg, msg_bytes, count, status,
                                     (hipStream_t)stream);
  if (e == hipErrorNoBinaryForGpu || e == hipErrorInvalidDeviceFunction)
    return fail(MPJX_ERR_NO_DEVICE, "no gfx950 kernel image for this device: %s", hipGetErrorString(e));
  if (e != hipSuccess) return fail(MPJX_ERR_HIP, "mpjbuf combine launch: %s", hipGetErrorString(e));
  return MPJX_SUCCESS;
}
