// rccl_standin.hip — TEST INFRASTRUCTURE ONLY: a stand-in for the RCCL entry points libmpjx calls, so
// the SAME libmpjx objects (mpjexpress_amd/build/*.o, no #ifdef in csrc/) run RcclTransport at P > 1 on
// a one-GPU box: rank THREADS of one process on one device play the one-process-per-GPU ranks.
// VERDICT r5 "do this" #3. Linked into tests/rccl/libmpjx_rccl_standin.so in place of -lrccl
// (mpjexpress_amd/Makefile); compiled with -fvisibility=hidden so libmpjx's nccl* references bind to
// these definitions inside that library whatever librccl a process has already loaded (torch's).
//
// Semantics kept from RCCL where libmpjx depends on them:
//   - ncclCommInitRank blocks until every rank of the id arrived; ncclCommSplit is collective over the
//     parent and forms one world per color, ranks ordered by (key, parent rank);
//   - every data movement is enqueued on the caller's stream, in call order: a sender records an event
//     where its data is ready, the receiver's stream waits on it and copies (hipMemcpyAsync, device to
//     device), and the sender's stream then waits until the receiver's copy is done (its buffer may be
//     overwritten after the call in stream order) — the rendezvous itself is on the host, which RCCL
//     does not do; libmpjx issues the same call sequence on every rank, so it cannot deadlock here;
//   - ncclSend/ncclRecv inside ncclGroupStart/End progress together; point-to-point transfers match in
//     order per (sender, receiver) pair and by operation (a collective never matches a p2p transfer);
//   - collectives are checked for consistency: AllToAllv's sendcounts[j] on rank i must equal rank j's
//     recvcounts[i] (real RCCL would corrupt or hang silently; here the call fails with
//     ncclInvalidUsage and the log says so); AllGather's in-place form is recognised
//     (sendbuff == recvbuff + rank * count);
//   - ncclAllReduce folds the ranks' contributions in rank order (0, 1, ..., P-1) — NOT RCCL's ring or
//     tree order: a test through it pins libmpjx's routing and arguments, never RCCL's arithmetic.
// Every call is logged (rsi_log: one JSON object per call and rank) so a test can assert the exact
// counts, displacements and pointers libmpjx passed. A wait longer than RSI_TIMEOUT_S (default 60 s)
// fails the call instead of hanging. rsi_fail_next(rank, op) makes that rank's next call of that
// collective fail synchronously (ncclInternalError), as an RCCL enqueue can: failure injection.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#define RSI_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

enum Kind { K_P2P = 1, K_ALLTOALL, K_ALLTOALLV, K_ALLGATHER, K_ALLREDUCE, K_SPLIT_UNUSED };

const char* kind_name(int k) {
  switch (k) {
    case K_P2P: return "p2p";
    case K_ALLTOALL: return "AllToAll";
    case K_ALLTOALLV: return "AllToAllv";
    case K_ALLGATHER: return "AllGather";
    case K_ALLREDUCE: return "AllReduce";
    default: return "?";
  }
}

double timeout_s() {
  const char* e = getenv("RSI_TIMEOUT_S");
  const double t = e ? atof(e) : 60.0;
  return t > 0 ? t : 60.0;
}

// ---- call log ---------------------------------------------------------------------------------------
std::mutex g_log_mu;
std::vector<std::string> g_log;

void log_line(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void log_line(const char* fmt, ...) {
  char buf[4096];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  std::lock_guard<std::mutex> lk(g_log_mu);
  if (g_log.size() < 200000) g_log.emplace_back(buf);
}

std::string arr(const size_t* a, int n) {
  std::string s = "[";
  for (int i = 0; i < n; i++) s += (i ? "," : "") + std::to_string(a[i]);
  return s + "]";
}

// ---- worlds -----------------------------------------------------------------------------------------
// One transfer: posted by the sender at ncclGroupEnd / the collective call, taken by the receiver.
struct Xfer {
  int kind = 0;
  const void* ptr = nullptr;
  size_t bytes = 0;
  hipEvent_t ready = nullptr;  // sender's stream: the data is in place
  hipEvent_t done = nullptr;   // receiver's stream: the copy out of ptr is done
  bool copied = false;
  bool failed = false;
};

struct World {
  int P = 0;
  int id = 0;  // for the log: 0, 1, ... in creation order
  std::mutex mu;
  std::condition_variable cv;
  bool aborted = false;
  int joined = 0;
  int refs = 0;
  // sends[src][dst]: transfers src posted to dst, in order, not yet taken
  std::vector<std::vector<std::deque<std::shared_ptr<Xfer>>>> sends;
  std::vector<hipEvent_t> pool;  // recycled events
  // ncclCommSplit rendezvous
  int split_arrived = 0;
  unsigned long long split_gen = 0;
  std::vector<int> split_color, split_key;
  std::vector<World*> split_out;
  std::vector<int> split_rank;
};

std::atomic<int> g_world_ids{0};

struct Comm {
  World* w = nullptr;
  int rank = 0;
  int device = 0;
  char* tmp = nullptr;  // AllReduce: every rank's contribution gathered here (P * bytes)
  size_t tmp_bytes = 0;
};

std::mutex g_init_mu;
std::condition_variable g_init_cv;
std::map<std::string, World*> g_pending;  // ncclCommInitRank: id -> world being formed

bool wait_until(World* w, std::unique_lock<std::mutex>& lk, const std::function<bool()>& pred) {
  const auto lim = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s());
  while (!pred()) {
    if (w->aborted) return false;
    if (w->cv.wait_until(lk, lim) == std::cv_status::timeout && !pred()) return false;
  }
  return !w->aborted;
}

hipEvent_t get_event(World* w) {  // caller holds w->mu
  if (!w->pool.empty()) {
    hipEvent_t e = w->pool.back();
    w->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  return e;
}

struct Op {  // one side of a transfer of this rank's current step
  int peer;
  void* ptr;
  size_t bytes;
};

// The rendezvous of one step (a group's sends and receives, or a collective expanded into them): post
// the sends, take and copy the receives on `s`, then order `s` after the peers' copies of our sends.
ncclResult_t run_step(Comm* c, int kind, const std::vector<Op>& sends, const std::vector<Op>& recvs, hipStream_t s,
                      const char* what) {
  World* w = c->w;
  const int me = c->rank;
  std::vector<std::shared_ptr<Xfer>> mine;
  {
    std::unique_lock<std::mutex> lk(w->mu);
    if (w->aborted) return ncclSystemError;
    for (const Op& o : sends) {
      auto x = std::make_shared<Xfer>();
      x->kind = kind;
      x->ptr = o.ptr;
      x->bytes = o.bytes;
      x->ready = get_event(w);
      x->done = get_event(w);
      if (!x->ready || !x->done || hipEventRecord(x->ready, s) != hipSuccess) return ncclUnhandledCudaError;
      w->sends[me][o.peer].push_back(x);
      mine.push_back(x);
    }
  }
  w->cv.notify_all();
  ncclResult_t rc = ncclSuccess;
  for (const Op& o : recvs) {
    std::shared_ptr<Xfer> x;
    {
      std::unique_lock<std::mutex> lk(w->mu);
      auto& q = w->sends[o.peer][me];
      if (!wait_until(w, lk, [&] { return !q.empty(); })) {
        log_line("{\"error\": \"%s: rank %d stopped waiting for rank %d's send: %s (world %d)\"}", what, me, o.peer,
                 w->aborted ? "world aborted" : "past RSI_TIMEOUT_S", w->id);
        return ncclSystemError;
      }
      x = q.front();
      q.pop_front();
    }
    if (x->kind != kind || x->bytes != o.bytes) {
      log_line("{\"error\": \"%s: rank %d expects %zu B of %s from rank %d, which posted %zu B of %s (world %d)\"}",
               what, me, o.bytes, kind_name(kind), o.peer, x->bytes, kind_name(x->kind), w->id);
      x->failed = true;
      rc = ncclInvalidUsage;
    } else {
      hipError_t e = hipStreamWaitEvent(s, x->ready, 0);
      if (e == hipSuccess && o.bytes) e = hipMemcpyAsync(o.ptr, x->ptr, o.bytes, hipMemcpyDeviceToDevice, s);
      if (e == hipSuccess) e = hipEventRecord(x->done, s);
      if (e != hipSuccess) {
        x->failed = true;
        rc = ncclUnhandledCudaError;
      }
    }
    {
      std::lock_guard<std::mutex> lk(w->mu);
      x->copied = true;
    }
    w->cv.notify_all();
  }
  for (auto& x : mine) {
    std::unique_lock<std::mutex> lk(w->mu);
    if (!wait_until(w, lk, [&] { return x->copied; })) {
      log_line("{\"error\": \"%s: rank %d stopped waiting for its send to be taken: %s (world %d)\"}", what, me,
               w->aborted ? "world aborted" : "past RSI_TIMEOUT_S", w->id);
      return ncclSystemError;
    }
    if (x->failed) rc = rc == ncclSuccess ? ncclInvalidUsage : rc;
    if (!x->failed && hipStreamWaitEvent(s, x->done, 0) != hipSuccess) rc = ncclUnhandledCudaError;
    // both waits on these events are enqueued: they can be recorded again
    w->pool.push_back(x->ready);
    w->pool.push_back(x->done);
  }
  return rc;
}

// ---- groups -----------------------------------------------------------------------------------------
thread_local int t_group_depth = 0;
struct Pending {
  std::vector<Op> sends, recvs;
  hipStream_t s = nullptr;
};
thread_local std::vector<std::pair<Comm*, Pending>> t_group;

Pending& pending_for(Comm* c, hipStream_t s) {
  for (auto& p : t_group)
    if (p.first == c) {
      p.second.s = s;
      return p.second;
    }
  t_group.push_back({c, Pending{}});
  t_group.back().second.s = s;
  return t_group.back().second;
}

// ---- AllReduce arithmetic (rank order) --------------------------------------------------------------
template <class T, int OP>
__global__ void k_fold(const T* const* in, int P, T* out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    T acc = in[0][i];
    for (int p = 1; p < P; p++) {
      const T v = in[p][i];
      if (OP == ncclSum) acc = (T)(acc + v);
      else if (OP == ncclProd) acc = (T)(acc * v);
      else if (OP == ncclMax) acc = v > acc ? v : acc;
      else acc = v < acc ? v : acc;
    }
    out[i] = acc;
  }
}

struct PtrTable {
  const void* p[64];
};

template <class T>
hipError_t fold_t(const void** dtab, int P, void* out, size_t n, ncclRedOp_t op, hipStream_t s) {
  const unsigned blocks = (unsigned)std::min<size_t>(4096, (n + 255) / 256 + 1);
  auto in = (const T* const*)dtab;
  switch (op) {
    case ncclSum: hipLaunchKernelGGL((k_fold<T, ncclSum>), dim3(blocks), dim3(256), 0, s, in, P, (T*)out, n); break;
    case ncclProd: hipLaunchKernelGGL((k_fold<T, ncclProd>), dim3(blocks), dim3(256), 0, s, in, P, (T*)out, n); break;
    case ncclMax: hipLaunchKernelGGL((k_fold<T, ncclMax>), dim3(blocks), dim3(256), 0, s, in, P, (T*)out, n); break;
    case ncclMin: hipLaunchKernelGGL((k_fold<T, ncclMin>), dim3(blocks), dim3(256), 0, s, in, P, (T*)out, n); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

size_t type_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 1;
  }
}

Comm* as(ncclComm_t c) { return reinterpret_cast<Comm*>(c); }

// failure injection (rsi_fail_next): one armed (world rank, collective name), consumed by its first match
std::mutex g_fail_mu;
int g_fail_rank = -1;
std::string g_fail_op;

bool injected_failure(const Comm* c, const char* op) {
  std::lock_guard<std::mutex> lk(g_fail_mu);
  if (g_fail_rank != c->rank || g_fail_op != op) return false;
  g_fail_rank = -1;
  log_line("{\"op\": \"InjectedFailure\", \"world\": %d, \"rank\": %d, \"call\": \"%s\"}", c->w->id, c->rank, op);
  return true;
}

World* new_world(int P) {
  World* w = new World();
  w->P = P;
  w->id = g_world_ids.fetch_add(1);
  w->sends.assign(P, std::vector<std::deque<std::shared_ptr<Xfer>>>(P));
  w->split_color.assign(P, 0);
  w->split_key.assign(P, 0);
  w->split_out.assign(P, nullptr);
  w->split_rank.assign(P, -1);
  return w;
}

}  // namespace

// ---- the entry points libmpjx binds ----------------------------------------------------------------
extern "C" {

ncclResult_t ncclGetVersion(int* version) {
  if (!version) return ncclInvalidArgument;
  *version = 99999;  // the stand-in (mpjx_runtime_versions reports it)
  return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "no error (rccl stand-in)";
    case ncclUnhandledCudaError: return "HIP call failed (rccl stand-in)";
    case ncclSystemError: return "timeout or aborted world (rccl stand-in)";
    case ncclInvalidArgument: return "invalid argument (rccl stand-in)";
    case ncclInvalidUsage: return "invalid usage: mismatched counts or operations across ranks (rccl stand-in)";
    default: return "error (rccl stand-in)";
  }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  if (!id) return ncclInvalidArgument;
  static std::atomic<unsigned long long> ctr{0};
  memset(id, 0, sizeof *id);
  const unsigned long long v[3] = {0x52534920494430ull /* "RSI ID0" */, (unsigned long long)getpid(),
                                   ctr.fetch_add(1) ^ (unsigned long long)std::chrono::steady_clock::now()
                                                          .time_since_epoch().count()};
  memcpy(id->internal, v, sizeof v);
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  const std::string key(commId.internal, sizeof commId.internal);
  World* w = nullptr;
  {
    std::unique_lock<std::mutex> lk(g_init_mu);
    auto it = g_pending.find(key);
    if (it == g_pending.end()) it = g_pending.emplace(key, new_world(nranks)).first;
    w = it->second;
    if (w->P != nranks) return ncclInvalidArgument;
    w->joined++;
    w->refs++;
    if (w->joined == nranks) g_pending.erase(key);
    g_init_cv.notify_all();
    const auto lim = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s());
    if (!g_init_cv.wait_until(lk, lim, [&] { return w->joined == nranks; })) return ncclSystemError;
  }
  auto c = new Comm();
  c->w = w;
  c->rank = rank;
  (void)hipGetDevice(&c->device);
  *comm = reinterpret_cast<ncclComm_t>(c);
  log_line("{\"op\": \"CommInitRank\", \"world\": %d, \"rank\": %d, \"nranks\": %d}", w->id, rank, nranks);
  return ncclSuccess;
}

ncclResult_t ncclCommSplit(ncclComm_t comm, int color, int key, ncclComm_t* newcomm, ncclConfig_t* config) {
  (void)config;
  Comm* c = as(comm);
  if (!c || !newcomm) return ncclInvalidArgument;
  World* w = c->w;
  std::unique_lock<std::mutex> lk(w->mu);
  const unsigned long long g = w->split_gen;
  w->split_color[c->rank] = color;
  w->split_key[c->rank] = key;
  if (++w->split_arrived == w->P) {  // the last to arrive forms every color's world
    std::map<int, std::vector<int>> by;
    for (int r = 0; r < w->P; r++)
      if (w->split_color[r] != NCCL_SPLIT_NOCOLOR) by[w->split_color[r]].push_back(r);
    std::fill(w->split_out.begin(), w->split_out.end(), nullptr);
    for (auto& kv : by) {
      auto& v = kv.second;
      std::stable_sort(v.begin(), v.end(), [&](int a, int b) { return w->split_key[a] < w->split_key[b]; });
      World* nw = new_world((int)v.size());
      nw->joined = nw->refs = (int)v.size();
      for (size_t i = 0; i < v.size(); i++) {
        w->split_out[v[i]] = nw;
        w->split_rank[v[i]] = (int)i;
      }
    }
    w->split_arrived = 0;
    w->split_gen++;
    w->cv.notify_all();
  } else if (!wait_until(w, lk, [&] { return w->split_gen != g; })) {
    return ncclSystemError;
  }
  World* nw = w->split_out[c->rank];
  if (!nw) {
    *newcomm = nullptr;
    return ncclSuccess;
  }
  auto n = new Comm();
  n->w = nw;
  n->rank = w->split_rank[c->rank];
  n->device = c->device;
  *newcomm = reinterpret_cast<ncclComm_t>(n);
  log_line("{\"op\": \"CommSplit\", \"world\": %d, \"rank\": %d, \"color\": %d, \"key\": %d, \"new_world\": %d, "
           "\"new_rank\": %d}", w->id, c->rank, color, key, nw->id, n->rank);
  return ncclSuccess;
}

static void release(Comm* c) {
  World* w = c->w;
  if (c->tmp) (void)hipFree(c->tmp);
  bool last = false;
  {
    std::lock_guard<std::mutex> lk(w->mu);
    last = --w->refs == 0;
  }
  if (last) {
    for (hipEvent_t e : w->pool) (void)hipEventDestroy(e);
    delete w;
  }
  delete c;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (!comm) return ncclSuccess;
  (void)hipDeviceSynchronize();  // RCCL's destroy waits for the communicator's work
  release(as(comm));
  return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t comm) {
  if (!comm) return ncclSuccess;
  Comm* c = as(comm);
  {
    std::lock_guard<std::mutex> lk(c->w->mu);
    c->w->aborted = true;
  }
  c->w->cv.notify_all();
  log_line("{\"op\": \"CommAbort\", \"world\": %d, \"rank\": %d}", c->w->id, c->rank);
  release(c);
  return ncclSuccess;
}

ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError) {
  if (!comm || !asyncError) return ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(as(comm)->w->mu);
  *asyncError = as(comm)->w->aborted ? ncclSystemError : ncclSuccess;
  return ncclSuccess;
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank) {
  if (!comm || !rank) return ncclInvalidArgument;
  *rank = as(comm)->rank;
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
  t_group_depth++;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (t_group_depth <= 0) return ncclInvalidUsage;
  if (--t_group_depth > 0) return ncclSuccess;
  auto group = std::move(t_group);
  t_group.clear();
  ncclResult_t rc = ncclSuccess;
  for (auto& g : group) {
    Comm* c = g.first;
    std::string ss, rs;
    for (const Op& o : g.second.sends) ss += (ss.empty() ? "" : ",") + std::string("[") + std::to_string(o.peer) + "," + std::to_string(o.bytes) + "]";
    for (const Op& o : g.second.recvs) rs += (rs.empty() ? "" : ",") + std::string("[") + std::to_string(o.peer) + "," + std::to_string(o.bytes) + "]";
    log_line("{\"op\": \"Group\", \"world\": %d, \"rank\": %d, \"sends\": [%s], \"recvs\": [%s]}", c->w->id, c->rank,
             ss.c_str(), rs.c_str());
    const ncclResult_t r = run_step(c, K_P2P, g.second.sends, g.second.recvs, g.second.s, "Group");
    if (rc == ncclSuccess) rc = r;
  }
  return rc;
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
  Comm* c = as(comm);
  if (!c || peer < 0 || peer >= c->w->P) return ncclInvalidArgument;
  const bool solo = t_group_depth == 0;
  if (solo) ncclGroupStart();
  pending_for(c, stream).sends.push_back({peer, (void*)sendbuff, count * type_size(datatype)});
  return solo ? ncclGroupEnd() : ncclSuccess;
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
  Comm* c = as(comm);
  if (!c || peer < 0 || peer >= c->w->P) return ncclInvalidArgument;
  const bool solo = t_group_depth == 0;
  if (solo) ncclGroupStart();
  pending_for(c, stream).recvs.push_back({peer, recvbuff, count * type_size(datatype)});
  return solo ? ncclGroupEnd() : ncclSuccess;
}

ncclResult_t ncclAllToAllv(const void* sendbuff, const size_t sendcounts[], const size_t sdispls[], void* recvbuff,
                           const size_t recvcounts[], const size_t rdispls[], ncclDataType_t datatype, ncclComm_t comm,
                           hipStream_t stream) {
  Comm* c = as(comm);
  if (!c) return ncclInvalidArgument;
  const int P = c->w->P, me = c->rank;
  const size_t es = type_size(datatype);
  log_line("{\"op\": \"AllToAllv\", \"world\": %d, \"rank\": %d, \"elem\": %zu, \"sendcounts\": %s, \"sdispls\": %s, "
           "\"recvcounts\": %s, \"rdispls\": %s}", c->w->id, me, es, arr(sendcounts, P).c_str(),
           arr(sdispls, P).c_str(), arr(recvcounts, P).c_str(), arr(rdispls, P).c_str());
  if (injected_failure(c, "AllToAllv")) return ncclInternalError;
  std::vector<Op> sends, recvs;
  for (int j = 0; j < P; j++) {
    if (j == me) continue;
    sends.push_back({j, (char*)sendbuff + sdispls[j] * es, sendcounts[j] * es});
    recvs.push_back({j, (char*)recvbuff + rdispls[j] * es, recvcounts[j] * es});
  }
  if (sendcounts[me] != recvcounts[me]) {
    log_line("{\"error\": \"AllToAllv: rank %d sends itself %zu elements but receives %zu\"}", me, sendcounts[me],
             recvcounts[me]);
    return ncclInvalidUsage;
  }
  if (sendcounts[me] &&
      hipMemcpyAsync((char*)recvbuff + rdispls[me] * es, (const char*)sendbuff + sdispls[me] * es, sendcounts[me] * es,
                     hipMemcpyDeviceToDevice, stream) != hipSuccess)
    return ncclUnhandledCudaError;
  return run_step(c, K_ALLTOALLV, sends, recvs, stream, "AllToAllv");
}

ncclResult_t ncclAllToAll(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype, ncclComm_t comm,
                          hipStream_t stream) {
  Comm* c = as(comm);
  if (!c) return ncclInvalidArgument;
  const int P = c->w->P, me = c->rank;
  const size_t es = type_size(datatype), b = count * es;
  log_line("{\"op\": \"AllToAll\", \"world\": %d, \"rank\": %d, \"elem\": %zu, \"count\": %zu, \"in_place\": %s}",
           c->w->id, me, es, count, sendbuff == recvbuff ? "true" : "false");
  if (injected_failure(c, "AllToAll")) return ncclInternalError;
  std::vector<Op> sends, recvs;
  for (int j = 0; j < P; j++) {
    if (j == me) continue;
    sends.push_back({j, (char*)sendbuff + j * b, b});
    recvs.push_back({j, (char*)recvbuff + j * b, b});
  }
  if (b && hipMemcpyAsync((char*)recvbuff + me * b, (const char*)sendbuff + me * b, b, hipMemcpyDeviceToDevice,
                          stream) != hipSuccess)
    return ncclUnhandledCudaError;
  return run_step(c, K_ALLTOALL, sends, recvs, stream, "AllToAll");
}

ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount, ncclDataType_t datatype,
                           ncclComm_t comm, hipStream_t stream) {
  Comm* c = as(comm);
  if (!c) return ncclInvalidArgument;
  const int P = c->w->P, me = c->rank;
  const size_t b = sendcount * type_size(datatype);
  const long long rel = (long long)((const char*)sendbuff - (const char*)recvbuff);
  const bool in_place = rel == (long long)(me * b);
  log_line("{\"op\": \"AllGather\", \"world\": %d, \"rank\": %d, \"bytes\": %zu, \"send_minus_recv\": %lld, "
           "\"in_place\": %s}", c->w->id, me, b, rel, in_place ? "true" : "false");
  if (injected_failure(c, "AllGather")) return ncclInternalError;
  std::vector<Op> sends, recvs;
  for (int j = 0; j < P; j++) {
    if (j == me) continue;
    sends.push_back({j, (void*)sendbuff, b});
    recvs.push_back({j, (char*)recvbuff + j * b, b});
  }
  if (!in_place && b &&
      hipMemcpyAsync((char*)recvbuff + me * b, sendbuff, b, hipMemcpyDeviceToDevice, stream) != hipSuccess)
    return ncclUnhandledCudaError;
  return run_step(c, K_ALLGATHER, sends, recvs, stream, "AllGather");
}

ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t stream) {
  Comm* c = as(comm);
  if (!c) return ncclInvalidArgument;
  const int P = c->w->P, me = c->rank;
  if (P > 64) return ncclInvalidArgument;
  const size_t es = type_size(datatype), b = count * es;
  log_line("{\"op\": \"AllReduce\", \"world\": %d, \"rank\": %d, \"count\": %zu, \"datatype\": %d, \"redop\": %d, "
           "\"in_place\": %s}", c->w->id, me, count, (int)datatype, (int)op, sendbuff == recvbuff ? "true" : "false");
  if (injected_failure(c, "AllReduce")) return ncclInternalError;
  const size_t need = (size_t)P * ((b + 255) & ~(size_t)255) + 64 * sizeof(void*);
  if (need > c->tmp_bytes) {
    if (c->tmp) {
      (void)hipStreamSynchronize(stream);
      (void)hipFree(c->tmp);
    }
    c->tmp = nullptr;
    c->tmp_bytes = 0;
    if (hipMalloc((void**)&c->tmp, need) != hipSuccess) return ncclUnhandledCudaError;
    c->tmp_bytes = need;
  }
  const size_t stride = (b + 255) & ~(size_t)255;
  std::vector<Op> sends, recvs;
  for (int j = 0; j < P; j++) {
    if (j == me) continue;
    sends.push_back({j, (void*)sendbuff, b});
    recvs.push_back({j, c->tmp + j * stride, b});
  }
  ncclResult_t rc = run_step(c, K_ALLREDUCE, sends, recvs, stream, "AllReduce");
  if (rc != ncclSuccess || count == 0) return rc;
  PtrTable tab{};
  for (int j = 0; j < P; j++) tab.p[j] = j == me ? sendbuff : (const void*)(c->tmp + j * stride);
  const void** dtab = (const void**)(c->tmp + P * stride);
  if (hipMemcpyAsync(dtab, &tab, sizeof(void*) * P, hipMemcpyHostToDevice, stream) != hipSuccess)
    return ncclUnhandledCudaError;
  hipError_t e = hipErrorInvalidValue;
  switch (datatype) {
    case ncclInt8: e = fold_t<int8_t>(dtab, P, recvbuff, count, op, stream); break;
    case ncclUint8: e = fold_t<uint8_t>(dtab, P, recvbuff, count, op, stream); break;
    case ncclInt32: e = fold_t<int32_t>(dtab, P, recvbuff, count, op, stream); break;
    case ncclUint32: e = fold_t<uint32_t>(dtab, P, recvbuff, count, op, stream); break;
    case ncclInt64: e = fold_t<int64_t>(dtab, P, recvbuff, count, op, stream); break;
    case ncclUint64: e = fold_t<uint64_t>(dtab, P, recvbuff, count, op, stream); break;
    case ncclFloat32: e = fold_t<float>(dtab, P, recvbuff, count, op, stream); break;
    case ncclFloat64: e = fold_t<double>(dtab, P, recvbuff, count, op, stream); break;
    default: return ncclInvalidArgument;
  }
  // the pointer table is host stack memory copied asynchronously: complete before it goes out of scope
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  return e == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

}  // extern "C"

// ---- test controls (default visibility) -------------------------------------------------------------
// The log as a JSON array; returns the bytes needed (with the NUL); writes at most cap bytes.
RSI_EXPORT size_t rsi_log(char* buf, size_t cap) {
  std::lock_guard<std::mutex> lk(g_log_mu);
  std::string s = "[";
  for (size_t i = 0; i < g_log.size(); i++) s += (i ? ",\n" : "") + g_log[i];
  s += "]";
  if (buf && cap) {
    const size_t n = std::min(cap - 1, s.size());
    memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return s.size() + 1;
}

RSI_EXPORT void rsi_log_clear() {
  std::lock_guard<std::mutex> lk(g_log_mu);
  g_log.clear();
}

RSI_EXPORT int rsi_is_standin() { return 1; }

RSI_EXPORT void rsi_fail_next(int rank, const char* op) {
  std::lock_guard<std::mutex> lk(g_fail_mu);
  g_fail_rank = rank;
  g_fail_op = op ? op : "";
}
