// mpjx_transport.hip — the byte transports under the collectives (RCCL over xGMI for one process
// per GPU; host-rendezvous device pulls / direct access for multicore ranks) and the communicator
// lifecycle. Multicore mode follows src/runtime/starter/MulticoreStarter.java:309-322 (ranks are
// threads of one process); one process per GPU stands in for MPJDev.init + COMM_WORLD
// (src/mpi/MPI.java:298-305).
#include "mpjx_internal.hpp"

#include <map>
#include <mutex>
#include <string>

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <thread>

using namespace mpjx;

// ---------------------------------------------------------------------------------------------
// transports

RcclTransport::~RcclTransport() {
  second.reset();
  if (dflag) (void)hipFree(dflag);
  if (nccl) ncclCommDestroy(nccl);
}

// The chunk pipeline's second lane: a second RCCL communicator over the same ranks, so the all-gather
// of chunk k-1 and the exchange #1 of chunk k+1 can be in flight at once (RCCL serialises one
// communicator's operations whatever their streams). HAZARD: operations of two communicators in flight
// together can deadlock when their kernels cannot be co-scheduled — if a rank's two streams share one
// hardware queue, or a communicator's kernel waits for CUs the other holds, and the ranks' GPUs order
// the two communicators' kernels differently. What keeps it safe here: every rank issues the same
// host-side sequence (exchange #1 of chunk k on lane 1, then the all-gather of chunk k-1 on lane 2),
// each lane's operations in the same order on every rank, the gather lane waits only on this rank's
// combine events; and the process runs with >= 8 hardware queues (bench.py sets GPU_MAX_HW_QUEUES=8;
// a JVM launcher must too), so the two lanes never share a queue. The pipeline is off
// by default (MPJX_PIPE_CHUNK_MIB), and bench.py runs every pipelined variant first in child processes
// (tools/rccl_preflight) before timing it, so a deadlock there costs the variant, not the run; an
// RCCL wait that does not finish within MPJX_RCCL_TIMEOUT_S aborts both communicators.
Transport* RcclTransport::lane2() {
  if (usable() != MPJX_SUCCESS) return nullptr;
  if (!second) {
    int rank = 0;
    if (ncclCommUserRank(nccl, &rank) != ncclSuccess) return nullptr;
    auto t = std::make_unique<RcclTransport>();
    t->p2p_only = p2p_only;  // the parent's agreed routing
    t->native = native;
    t->nranks = nranks;
    t->parent = this;
    // collective over the communicator: every rank reaches it in the same pipelined call
    const ncclResult_t r = ncclCommSplit(nccl, 0, rank, &t->nccl, nullptr);
    if (r != ncclSuccess || !t->nccl) {
      t->nccl = nullptr;
      failed_call("ncclCommSplit (the pipeline's second lane)", r != ncclSuccess ? r : ncclInternalError);
      return nullptr;
    }
    second = std::move(t);
  }
  return second.get();
}

int Transport::wait(hipStream_t s) {
  HIPCHK(hipStreamSynchronize(s));
  return MPJX_SUCCESS;
}

void RcclTransport::abort_comms() {
  if (parent) return parent->abort_comms();
  if (second) {
    if (second->nccl) (void)ncclCommAbort(second->nccl);
    second->nccl = nullptr;
    second->aborted = true;
  }
  if (nccl) (void)ncclCommAbort(nccl);
  nccl = nullptr;
  aborted = true;
}

void RcclTransport::abort_world() {
  if (nranks > 1) abort_comms();
}

int RcclTransport::failed_call(const char* what, ncclResult_t r) {
  abort_comms();
  return fail(MPJX_ERR_RCCL, "%s: %s (communicator aborted; destroy and re-create it)", what, ncclGetErrorString(r));
}

// An RCCL call of an RcclTransport member: a failure aborts the communicator (failed_call).
#define RCCL_CALL(expr)                                 \
  do {                                                  \
    ncclResult_t r_ = (expr);                           \
    if (r_ != ncclSuccess) return failed_call(#expr, r_); \
  } while (0)

int RcclTransport::usable() const {
  return aborted ? fail(MPJX_ERR_RCCL, "RCCL communicator was aborted after an earlier failure; destroy and "
                                       "re-create it") : MPJX_SUCCESS;
}

static double rccl_timeout_s() {
  const char* e = getenv("MPJX_RCCL_TIMEOUT_S");  // read per wait; unset or <= 0: no limit
  const double t = e ? atof(e) : 0.0;
  return t > 0 ? t : 0.0;
}

int RcclTransport::wait(hipStream_t s) {
  CHK(usable());
  const double lim = rccl_timeout_s();
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned it = 0;; it++) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return MPJX_SUCCESS;
    if (q != hipErrorNotReady) return fail(MPJX_ERR_HIP, "stream: %s", hipGetErrorString(q));
    ncclResult_t ar = ncclSuccess;
    bool async_err = ncclCommGetAsyncError(nccl, &ar) == ncclSuccess && ar != ncclSuccess && ar != ncclInProgress;
    if (!async_err && second && second->nccl)  // the pipeline's second lane feeds the same streams
      async_err = ncclCommGetAsyncError(second->nccl, &ar) == ncclSuccess && ar != ncclSuccess && ar != ncclInProgress;
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (async_err || (lim > 0 && el > lim)) {
      abort_comms();  // releases this rank's RCCL kernels; the peers see the failure
      if (async_err) return fail(MPJX_ERR_RCCL, "asynchronous RCCL error: %s (communicator aborted)", ncclGetErrorString(ar));
      return fail(MPJX_ERR_RCCL, "RCCL call not complete after %.3g s (MPJX_RCCL_TIMEOUT_S): communicator aborted", lim);
    }
    if (it < 4096) __builtin_ia32_pause();
    else if (it < 8192) sched_yield();
    else usleep(20);
  }
}

int RcclTransport::exchange(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s) {
  CHK(usable());
  if (sends.empty() && recvs.empty()) return MPJX_SUCCESS;
  RCCL_CALL(ncclGroupStart());
  // the group is closed whatever happens inside it (an open group would swallow this thread's next call)
  ncclResult_t r = ncclSuccess;
  for (const Xfer& x : sends)
    if (r == ncclSuccess) r = ncclSend(x.ptr, x.bytes, ncclUint8, x.peer, nccl, s);
  for (const Xfer& x : recvs)
    if (r == ncclSuccess) r = ncclRecv(x.ptr, x.bytes, ncclUint8, x.peer, nccl, s);
  const ncclResult_t e = ncclGroupEnd();
  if (r != ncclSuccess) return failed_call("ncclSend/ncclRecv in a group", r);
  if (e != ncclSuccess) return failed_call("ncclGroupEnd", e);
  return MPJX_SUCCESS;
}

int RcclTransport::barrier(hipStream_t s) {
  CHK(usable());
  if (!dflag) HIPCHK(hipMalloc(&dflag, 4 * sizeof(int)));
  RCCL_CALL(ncclAllReduce(dflag, dflag, 1, ncclInt32, ncclSum, nccl, s));
  return wait(s);
}

static bool env_on(const char* name) {
  const char* e = getenv(name);
  return e && *e && strcmp(e, "0") != 0;
}

int RcclTransport::agree(hipStream_t s) {
  CHK(usable());
  p2p_only = env_on("MPJX_RCCL_P2P");
  native = env_on("MPJX_RCCL_NATIVE") ? 1 : env_on("MPJX_RCCL_NATIVE_P2") ? 2 : 0;
  if (!dflag) HIPCHK(hipMalloc(&dflag, 4 * sizeof(int)));
  int v[4] = {p2p_only ? 1 : 0, native, p2p_only ? -1 : 0, -native};
  HIPCHK(hipMemcpyAsync(dflag, v, sizeof v, hipMemcpyHostToDevice, s));
  RCCL_CALL(ncclAllReduce(dflag, dflag, 4, ncclInt32, ncclMax, nccl, s));
  HIPCHK(hipMemcpyAsync(v, dflag, sizeof v, hipMemcpyDeviceToHost, s));
  CHK(wait(s));
  // max(x) == -max(-x) == min(x) exactly when every rank holds the same x
  if (v[0] != -v[2] || v[1] != -v[3])
    return fail(MPJX_ERR_ARG, "ranks disagree on the RCCL routing read at init: MPJX_RCCL_P2P %s, MPJX_RCCL_NATIVE(_P2) "
                "%s (set the same on every rank)", v[0] != -v[2] ? "differs" : "agrees",
                v[1] != -v[3] ? "differs" : "agrees");
  return MPJX_SUCCESS;
}

int Transport::alltoallv(int me, const char* send, const std::vector<size_t>& scount,
                         const std::vector<size_t>& sdispl, char* recv, const std::vector<size_t>& rcount,
                         const std::vector<size_t>& rdispl, hipStream_t s) {
  std::vector<Xfer> sends, recvs;
  const int P = (int)scount.size();
  for (int j = 0; j < P; j++) {
    if (j == me) {
      if (scount[j]) HIPCHK(hipMemcpyAsync(recv + rdispl[j], send + sdispl[j], scount[j], hipMemcpyDeviceToDevice, s));
      continue;
    }
    if (scount[j]) sends.push_back({j, (void*)(send + sdispl[j]), scount[j]});
    if (rcount[j]) recvs.push_back({j, recv + rdispl[j], rcount[j]});
  }
  return exchange(sends, recvs, s);
}

int Transport::allgather_equal(int me, int P, char* buf, size_t bytes, hipStream_t s) {
  std::vector<Xfer> sends, recvs;
  if (bytes == 0) return MPJX_SUCCESS;
  for (int j = 0; j < P; j++) {
    if (j == me) continue;
    sends.push_back({j, buf + (size_t)me * bytes, bytes});
    recvs.push_back({j, buf + (size_t)j * bytes, bytes});
  }
  return exchange(sends, recvs, s);
}

int RcclTransport::allreduce(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                             hipStream_t s) {
  CHK(usable());
  if (count == 0) return MPJX_SUCCESS;
  RCCL_CALL(ncclAllReduce(send, recv, count, dt, op, nccl, s));
  return MPJX_SUCCESS;
}

int RcclTransport::alltoallv(int me, const char* send, const std::vector<size_t>& scount,
                             const std::vector<size_t>& sdispl, char* recv, const std::vector<size_t>& rcount,
                             const std::vector<size_t>& rdispl, hipStream_t s) {
  CHK(usable());
  if (p2p()) return Transport::alltoallv(me, send, scount, sdispl, recv, rcount, rdispl, s);
  const int P = (int)scount.size();
  bool equal = true;
  for (int j = 0; j < P; j++)
    equal = equal && scount[j] == scount[0] && rcount[j] == scount[0] && sdispl[j] == j * scount[0] &&
            rdispl[j] == j * scount[0];
  if (equal) {
    if (scount[0] == 0) return MPJX_SUCCESS;
    RCCL_CALL(ncclAllToAll(send, recv, scount[0], ncclUint8, nccl, s));
    return MPJX_SUCCESS;
  }
  RCCL_CALL(ncclAllToAllv(send, scount.data(), sdispl.data(), recv, rcount.data(), rdispl.data(), ncclUint8, nccl, s));
  return MPJX_SUCCESS;
}

int RcclTransport::allgather_equal(int me, int P, char* buf, size_t bytes, hipStream_t s) {
  CHK(usable());
  if (p2p()) return Transport::allgather_equal(me, P, buf, bytes, s);
  if (bytes == 0) return MPJX_SUCCESS;
  RCCL_CALL(ncclAllGather(buf + (size_t)me * bytes, buf, bytes, ncclUint8, nccl, s));
  return MPJX_SUCCESS;
}

// Sense-reversing host barrier: spin briefly (ranks are threads on their own cores, and a
// collective's rendezvous is usually a few microseconds apart), then sleep on the condvar. A rank
// that left a collective early (abort()) releases every waiter with an error instead of a hang.
int SmpWorld::barrier() {
  if (failed.load(std::memory_order_acquire))
    return fail(MPJX_ERR_INTERNAL, "multicore world: another rank failed; the communicator is unusable");
  const unsigned long long g = gen.load(std::memory_order_acquire);
  if (arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == P) {
    arrived.store(0, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> lk(mu);
      gen.store(g + 1, std::memory_order_release);
    }
    cv.notify_all();
    return MPJX_SUCCESS;
  }
  auto passed = [&] { return gen.load(std::memory_order_acquire) != g || failed.load(std::memory_order_acquire); };
  for (int i = 0; i < (1 << 14) && !passed(); i++) __builtin_ia32_pause();
  if (!passed()) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, passed);
  }
  if (gen.load(std::memory_order_acquire) != g) return MPJX_SUCCESS;
  return fail(MPJX_ERR_INTERNAL, "multicore world: another rank failed; the communicator is unusable");
}

void SmpWorld::abort() {
  {
    std::lock_guard<std::mutex> lk(mu);
    failed.store(1, std::memory_order_release);
  }
  cv.notify_all();
}

SmpTransport::~SmpTransport() {
  std::lock_guard<std::mutex> lk(w->mu);
  if (--w->refs == 0) {
    for (int r = 0; r < w->P; r++) {
      (void)hipSetDevice(w->devices[r]);
      if (w->ready[r]) (void)hipEventDestroy(w->ready[r]);
      if (w->done[r]) (void)hipEventDestroy(w->done[r]);
    }
  }
}

int SmpTransport::exchange(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s) {
  // 1. publish what this rank sends, once its stream has produced it
  hipError_t e0 = hipEventRecord(w->ready[me], s);
  if (e0 != hipSuccess) {
    w->abort();
    return fail(MPJX_ERR_HIP, "hipEventRecord: %s", hipGetErrorString(e0));
  }
  w->posted[me] = sends;
  CHK(w->barrier());
  // 2. pull every block addressed to this rank from its owner
  int rc = MPJX_SUCCESS;
  for (const Xfer& r : recvs) {
    const Xfer* src = nullptr;
    for (const Xfer& x : w->posted[r.peer])
      if (x.peer == me) { src = &x; break; }
    if (!src || src->bytes != r.bytes) {
      rc = fail(MPJX_ERR_INTERNAL, "smp exchange mismatch: rank %d expects %zu B from %d, got %zu", me,
                r.bytes, r.peer, src ? src->bytes : (size_t)0);
      break;
    }
    hipError_t e = hipStreamWaitEvent(s, w->ready[r.peer], 0);
    if (e == hipSuccess) e = hipMemcpyAsync(r.ptr, src->ptr, r.bytes, hipMemcpyDefault, s);
    if (e != hipSuccess) { rc = fail(MPJX_ERR_HIP, "smp pull: %s", hipGetErrorString(e)); break; }
  }
  hipError_t e = hipEventRecord(w->done[me], s);
  if (rc == MPJX_SUCCESS && e != hipSuccess) rc = fail(MPJX_ERR_HIP, "hipEventRecord: %s", hipGetErrorString(e));
  if (rc != MPJX_SUCCESS) w->abort();
  const int brc = w->barrier();
  if (rc == MPJX_SUCCESS) rc = brc;
  // 3. a sender may not overwrite its blocks until every puller has copied them
  // No closing barrier: posted[] and the events are rewritten only after the next rendezvous's first
  // barrier, which no rank reaches before it has enqueued these waits (a stream wait binds the
  // event's current record, so re-recording afterwards is safe).
  for (const Xfer& x : sends) {
    e = hipStreamWaitEvent(s, w->done[x.peer], 0);
    if (rc == MPJX_SUCCESS && e != hipSuccess) rc = fail(MPJX_ERR_HIP, "hipStreamWaitEvent: %s", hipGetErrorString(e));
  }
  return rc;
}

int SmpTransport::share(const std::vector<const void*>& mine, hipStream_t s,
                        std::vector<std::vector<const void*>>* all, bool leader) {
  // A stream with nothing pending (the usual case: the mpiJava calls are blocking) has already
  // produced its buffers, so peers need not wait on it; otherwise publish an event at this point.
  w->idle[me] = hipStreamQuery(s) == hipSuccess;
  if (!w->idle[me] && (!leader || me != 0)) {
    const hipError_t e0 = hipEventRecord(w->ready[me], s);
    if (e0 != hipSuccess) {
      w->abort();
      return fail(MPJX_ERR_HIP, "hipEventRecord: %s", hipGetErrorString(e0));
    }
  }
  w->shared[me] = mine;
  CHK(w->barrier());
  *all = w->shared;
  int rc = MPJX_SUCCESS;
  if (!leader || me == 0) {
    for (int j = 0; j < w->P; j++) {
      if (j == me || w->idle[j]) continue;
      hipError_t e = hipStreamWaitEvent(s, w->ready[j], 0);
      if (e != hipSuccess && rc == MPJX_SUCCESS) rc = fail(MPJX_ERR_HIP, "hipStreamWaitEvent: %s", hipGetErrorString(e));
    }
  }
  // shared[me] and ready[me] are rewritten only after the matching fence()'s barrier, which every
  // rank reaches after copying the table and enqueuing these waits.
  return rc;
}

// A launching rank (every rank; with leader, rank 0 alone) marks where its stream's work of this call
// ends: an event the other ranks' streams then wait on, or — for a blocking call — the stream drained
// on the host before the rendezvous (synced[me]), after which no other rank needs a device-side wait
// on it. A rank that waits on nothing more returns as soon as the rendezvous releases it: configs[0]
// (1 MiB, P = 4 rank threads, one GPU) then costs one launch, its drain and two host rendezvous per call
// instead of a chain of cross-stream waits.
int SmpTransport::fence(hipStream_t s, bool leader, bool /*signalled*/, bool blocking) {
  if (!leader || me == 0) {
    const hipError_t e0 = blocking ? hipStreamSynchronize(s) : hipEventRecord(w->done[me], s);
    if (e0 != hipSuccess) {
      w->abort();
      return fail(MPJX_ERR_HIP, "%s: %s", blocking ? "hipStreamSynchronize" : "hipEventRecord", hipGetErrorString(e0));
    }
    w->synced[me] = blocking ? 1 : 0;
  }
  CHK(w->barrier());
  int rc = MPJX_SUCCESS;
  for (int j = 0; j < w->P; j++) {
    if (j == me || (leader && j != 0) || w->synced[j]) continue;
    hipError_t e = hipStreamWaitEvent(s, w->done[j], 0);
    if (e != hipSuccess && rc == MPJX_SUCCESS) rc = fail(MPJX_ERR_HIP, "hipStreamWaitEvent: %s", hipGetErrorString(e));
  }
  return rc;  // done[] and synced[] are rewritten only after the next rendezvous's first barrier
}

int SmpTransport::barrier(hipStream_t s) {
  const hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    w->abort();
    return fail(MPJX_ERR_HIP, "hipStreamSynchronize: %s", hipGetErrorString(e));
  }
  return w->barrier();
}

// ---------------------------------------------------------------------------------------------
// communicators

int mpjx::comm_common_init(mpjx_comm* c) {
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&c->last_ev, hipEventDisableTiming));
  return MPJX_SUCCESS;
}

int mpjx::grow_device(mpjx_comm* c, char** buf, size_t* cap, size_t need, hipStream_t s) {
  if (need <= *cap) return MPJX_SUCCESS;
  const size_t old = *cap;
  if (*buf) {
    CHK(c->tr->wait(s));  // kernels still reading the old buffer finish before it is replaced
    c->retired.push_back(*buf);
  }
  *buf = nullptr;
  *cap = 0;
  // Outgrown buffers are retired, not freed, until mpjx_comm_destroy (no device free and
  // re-allocation while a communicator lives), so growth must stay geometric for the retired total to
  // stay bounded: doubling below 64 MiB (retired total < live capacity), x1.5 from 64 MiB on (retired
  // total < 2x live capacity, where sizes creeping up by 2 MiB per call would otherwise pile up a
  // quadratic sum of dead buffers), in 2 MiB granules.
  const size_t gran = (size_t)2 << 20;
  const size_t want = std::max(need, old < ((size_t)64 << 20) ? 2 * old : old + old / 2);
  const size_t b = (want + gran - 1) / gran * gran;
  HIPCHK(hipMalloc((void**)buf, b));
  *cap = b;
  return MPJX_SUCCESS;
}

int mpjx::check_device(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(MPJX_ERR_NO_DEVICE, "no HIP device visible");
  if (device < 0 || device >= n) return fail(MPJX_ERR_ARG, "device %d out of range [0,%d)", device, n);
  return MPJX_SUCCESS;
}

extern "C" int mpjx_get_unique_id(mpjx_unique_id* id) {
  if (!id) return fail(MPJX_ERR_ARG, "id is NULL");
  static_assert(sizeof(mpjx_unique_id) == sizeof(ncclUniqueId), "unique id size");
  ncclUniqueId u;
  NCCLCHK(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof u);
  return MPJX_SUCCESS;
}

extern "C" int mpjx_comm_init_rank(mpjx_comm_t* comm, int nranks, const mpjx_unique_id* id, int rank,
                                   int device) {
  if (!comm || !id) return fail(MPJX_ERR_ARG, "NULL argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(MPJX_ERR_ARG, "rank %d of %d", rank, nranks);
  CHK(check_device(device));
  auto c = std::make_unique<mpjx_comm>();
  c->rank = rank;
  c->size = nranks;
  c->device = device;
  CHK(comm_common_init(c.get()));
  auto t = std::make_unique<RcclTransport>();
  t->nranks = nranks;
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  NCCLCHK(ncclCommInitRank(&t->nccl, nranks, u, rank));
  CHK(t->agree(c->stream));  // collective: MPJX_RCCL_P2P / MPJX_RCCL_NATIVE(_P2), equal on every rank
  c->tr = std::move(t);
  *comm = c.release();
  return MPJX_SUCCESS;
}

extern "C" int mpjx_comm_init_smp(mpjx_comm_t* comms, int nranks, const int* devices) {
  if (!comms || !devices || nranks < 1) return fail(MPJX_ERR_ARG, "bad arguments");
  for (int r = 0; r < nranks; r++) CHK(check_device(devices[r]));
  auto w = std::make_shared<SmpWorld>();
  w->P = nranks;
  w->devices.assign(devices, devices + nranks);
  w->posted.resize(nranks);
  w->shared.resize(nranks);
  w->idle.assign(nranks, 0);
  w->synced.assign(nranks, 0);
  w->host_out.assign(nranks, 0);
  w->copy_src.assign(nranks, nullptr);
  w->direct = true;
  w->single = std::all_of(devices, devices + nranks, [&](int d) { return d == devices[0]; });
  w->ready.assign(nranks, nullptr);
  w->done.assign(nranks, nullptr);
  for (int r = 0; r < nranks; r++) {
    HIPCHK(hipSetDevice(devices[r]));
    for (int q = 0; q < nranks; q++) {  // direct device-to-device pulls between distinct GPUs
      if (devices[q] == devices[r]) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, devices[r], devices[q]) == hipSuccess && can) {
        hipError_t e = hipDeviceEnablePeerAccess(devices[q], 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return fail(MPJX_ERR_HIP, "peer access");
        (void)hipGetLastError();
      } else {
        w->direct = false;  // no load/store path between these GPUs: keep the copy-based exchanges
      }
    }
    HIPCHK(hipEventCreateWithFlags(&w->ready[r], hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&w->done[r], hipEventDisableTiming));
  }
  for (int r = 0; r < nranks; r++) {
    auto c = std::make_unique<mpjx_comm>();
    c->rank = r;
    c->size = nranks;
    c->device = devices[r];
    CHK(comm_common_init(c.get()));
    auto t = std::make_unique<SmpTransport>();
    t->w = w;
    t->me = r;
    {
      std::lock_guard<std::mutex> lk(w->mu);
      w->refs++;
    }
    c->tr = std::move(t);
    comms[r] = c.release();
  }
  return MPJX_SUCCESS;
}

// Multicore worlds formed by the rank threads themselves (smpdev: every rank thread runs MPI.Init and
// creates its communicators on its own, src/runtime/starter/MulticoreStarter.java:309-322). The
// first thread to arrive with an id creates every rank's handle; each thread takes its own, and the
// entry is dropped once all have. Process-wide, so rank threads whose classes (and JNI shims) were
// loaded by different class loaders still meet here, in the one libmpjx of the process.
namespace {
struct PendingSmp {
  std::vector<mpjx_comm_t> comms;
  std::vector<int> devices;  // the first caller's devices[]; every later caller must pass the same
  std::vector<char> taken;
  int left = 0;
};
std::mutex g_smp_mu;
std::map<std::string, PendingSmp> g_smp_pending;
}  // namespace

extern "C" int mpjx_comm_init_smp_rank(mpjx_comm_t* comm, int nranks, const mpjx_unique_id* id, int rank,
                                        const int* devices) {
  if (!comm || !id || !devices || nranks < 1) return fail(MPJX_ERR_ARG, "bad arguments");
  if (rank < 0 || rank >= nranks) return fail(MPJX_ERR_ARG, "rank %d of %d", rank, nranks);
  const std::string key(id->internal, sizeof id->internal);
  std::lock_guard<std::mutex> lk(g_smp_mu);
  auto it = g_smp_pending.find(key);
  if (it == g_smp_pending.end()) {
    PendingSmp p;
    p.comms.assign(nranks, nullptr);
    p.devices.assign(devices, devices + nranks);
    p.taken.assign(nranks, 0);
    p.left = nranks;
    CHK(mpjx_comm_init_smp(p.comms.data(), nranks, devices));
    it = g_smp_pending.emplace(key, std::move(p)).first;
  }
  PendingSmp& p = it->second;
  if ((int)p.comms.size() != nranks) return fail(MPJX_ERR_ARG, "world size %d, but this id's world has %d ranks",
                                                 nranks, (int)p.comms.size());
  for (int r = 0; r < nranks; r++)
    if (devices[r] != p.devices[r])
      return fail(MPJX_ERR_ARG, "devices[%d] = %d, but this id's world put rank %d on device %d", r, devices[r], r,
                  p.devices[r]);
  if (p.taken[rank]) return fail(MPJX_ERR_ARG, "rank %d of this world was already initialised", rank);
  p.taken[rank] = 1;
  *comm = p.comms[rank];
  if (--p.left == 0) g_smp_pending.erase(it);
  return MPJX_SUCCESS;
}

extern "C" int mpjx_comm_destroy(mpjx_comm_t c) {
  if (!c) return MPJX_SUCCESS;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->last_stream) (void)hipStreamSynchronize(c->last_stream);
  c->tr.reset();
  for (void* p : c->retired) (void)hipFree(p);
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->hstage) (void)hipFree(c->hstage);
  for (hipStream_t hs : {c->h2d, c->d2h})
    if (hs) {
      (void)hipStreamSynchronize(hs);
      (void)hipStreamDestroy(hs);
    }
  for (auto* v : {&c->host_in_ev, &c->host_coll_ev})
    for (hipEvent_t e : *v) (void)hipEventDestroy(e);
  if (c->last_ev) (void)hipEventDestroy(c->last_ev);
  if (c->cstream) (void)hipStreamSynchronize(c->cstream);
  for (hipEvent_t e : c->pipe_ev) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->phase_ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->trace_ev) (void)hipEventDestroy(e);
  if (c->cstream) (void)hipStreamDestroy(c->cstream);
  if (c->gstream) (void)hipStreamSynchronize(c->gstream);
  if (c->gstream) (void)hipStreamDestroy(c->gstream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return MPJX_SUCCESS;
}

extern "C" int mpjx_comm_rank(mpjx_comm_t c, int* r) { COMM_ARG(c); if (!r) return fail(MPJX_ERR_ARG, "NULL"); *r = c->rank; return MPJX_SUCCESS; }
extern "C" int mpjx_comm_size(mpjx_comm_t c, int* s) { COMM_ARG(c); if (!s) return fail(MPJX_ERR_ARG, "NULL"); *s = c->size; return MPJX_SUCCESS; }
extern "C" int mpjx_comm_device(mpjx_comm_t c, int* d) { COMM_ARG(c); if (!d) return fail(MPJX_ERR_ARG, "NULL"); *d = c->device; return MPJX_SUCCESS; }
extern "C" int mpjx_comm_stream(mpjx_comm_t c, void** s) { COMM_ARG(c); if (!s) return fail(MPJX_ERR_ARG, "NULL"); *s = (void*)c->stream; return MPJX_SUCCESS; }

extern "C" int mpjx_comm_synchronize(mpjx_comm_t c) {
  COMM_ARG(c);
  HIPCHK(hipSetDevice(c->device));
  CHK(c->tr->wait(c->stream));
  if (c->last_stream && c->last_stream != c->stream) CHK(c->tr->wait(c->last_stream));
  return MPJX_SUCCESS;
}

extern "C" int mpjx_barrier(mpjx_comm_t c) {
  COMM_ARG(c);
  HIPCHK(hipSetDevice(c->device));
  CHK(mpjx_comm_synchronize(c));
  return c->tr->barrier(c->stream);
}
