// mpjx_ipc.hip — cross-process direct engine: ranks are processes of one node (one per GPU, or
// several sharing a GPU) that map each other's device staging regions through HIP IPC, no RCCL.
//
// The reference's multi-process deployments on one node (niodev ranks started by the runtime,
// src/runtime/starter/MPJRun.java; or the native device under mpirun) move every operand through
// the transport edge by edge (src/mpi/PureIntracomm.java:1943-1992). Here every collective runs on
// the Direct engine the multicore mode uses (mpjx_collectives.hip): rank r's P-way kernel combines
// block r of every rank's send and stores the result block into every rank's receive region, so an
// Allreduce is one push of the blocks (push mode), one kernel per rank and one local copy-out,
// between two host barriers: each byte crosses a link at most twice.
//
// Rendezvous: a POSIX shared-memory segment named from the world's 128-byte unique id holds a
// sense-reversing barrier and one row per rank: the IPC handle and size of the rank's device
// staging region (mapped by every peer once, at init), plus the pieces an exchange() round posts.
// User buffers never cross processes (why: IpcTransport in mpjx_engine.hpp).
#include "mpjx_internal.hpp"

#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>

using namespace mpjx;

namespace mpjx {

constexpr int kIpcMaxRanks = 64;
// [A: kIpcMaxRanks][B: kIpcMaxRanks] sequence numbers, then the last-block counter of the fused
// copies + flags launch (launch_copies_flags)
constexpr size_t kIpcFlagBytes = 2 * kIpcMaxRanks * sizeof(unsigned long long) + 256;

struct IpcSend {
  int32_t peer, pad;
  unsigned long long off, bytes;  // block for `peer` at stage + off (this round's piece)
};

struct IpcRow {
  unsigned long long cap;        // bytes per half of the rank's staging region
  char handle[sizeof(hipIpcMemHandle_t)];
  int32_t nsend, rounds;         // exchange(): posted pieces; rounds this rank needs
  int32_t dsync, pull;           // MPJX_IPC_SYNC on this rank: 0 host, 1 device, 2 device-shared;
                                 // MPJX_IPC_MODE: 0 push, 1 pull (both read once, at init)
  char bus[32];                  // PCI bus id of the rank's GPU (device sync needs one rank per GPU)
  IpcSend sends[kIpcMaxRanks];
};

struct IpcSeg {
  std::atomic<uint32_t> attached;
  std::atomic<uint32_t> arrived;
  std::atomic<unsigned long long> gen;
  std::atomic<int32_t> failed;  // a rank gave up: every later barrier reports it
  IpcRow row[kIpcMaxRanks];
};

static_assert(std::atomic<uint32_t>::is_always_lock_free && std::atomic<unsigned long long>::is_always_lock_free,
              "shared-memory atomics must be lock-free");

static bool debug() {
  static const bool d = [] { const char* e = getenv("MPJX_IPC_DEBUG"); return e && *e && *e != '0'; }();
  return d;
}

static double timeout_s() {
  const char* e = getenv("MPJX_IPC_TIMEOUT_S");
  const double t = e ? atof(e) : 300.0;
  return t > 0 ? t : 300.0;
}

// Spin, then yield, then sleep until pred() or the timeout; false on timeout.
template <class Pred>
static bool wait_for(Pred pred, const IpcSeg* seg) {
  for (int i = 0; i < (1 << 14); i++) {
    if (pred()) return true;
    __builtin_ia32_pause();
  }
  const auto t0 = std::chrono::steady_clock::now();
  const double lim = timeout_s();
  for (unsigned it = 0;; it++) {
    if (pred()) return true;
    if (seg->failed.load(std::memory_order_acquire)) return false;
    if (it < 1000) {
      sched_yield();
    } else {
      usleep(20);
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > lim) return false;
    }
  }
}

}  // namespace mpjx

IpcTransport::~IpcTransport() {
  if (tail_dev) (void)hipFree(tail_dev);
  for (int j = 0; j < (int)peers.size(); j++)
    if (peers[j].base) (void)hipIpcCloseMemHandle(peers[j].base);
  if (stage) (void)hipFree(stage);
  if (herr) (void)hipHostFree(herr);
  if (seg_registered) (void)hipHostUnregister(seg);
  if (seg) munmap(seg, sizeof(IpcSeg));
}

void IpcTransport::abort_world() { seg->failed.store(1, std::memory_order_release); }

int IpcTransport::hbarrier() {
  if (seg->failed.load(std::memory_order_acquire))
    return fail(MPJX_ERR_INTERNAL, "ipc world: another rank failed; the communicator is unusable");
  const unsigned long long g = seg->gen.load(std::memory_order_acquire);
  if (seg->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)P) {
    seg->arrived.store(0, std::memory_order_relaxed);
    seg->gen.store(g + 1, std::memory_order_release);
    return MPJX_SUCCESS;
  }
  if (wait_for([&] { return seg->gen.load(std::memory_order_acquire) != g; }, seg)) return MPJX_SUCCESS;
  if (seg->failed.load(std::memory_order_acquire))
    return fail(MPJX_ERR_INTERNAL, "ipc world: another rank failed; the communicator is unusable");
  seg->failed.store(1, std::memory_order_release);
  return fail(MPJX_ERR_INTERNAL, "ipc barrier: rank %d gave up after %.0f s (a peer died, failed or called "
              "a different collective); MPJX_IPC_TIMEOUT_S sets the limit", me, timeout_s());
}

// A local failure before a barrier must not leave the peers waiting for this rank: mark the world.
#define IPC_LOCAL(expr)                                        \
  do {                                                         \
    int c_ = (expr);                                           \
    if (c_ != MPJX_SUCCESS) {                                  \
      seg->failed.store(1, std::memory_order_release);         \
      return c_;                                               \
    }                                                          \
  } while (0)

// MPJX_IPC_FUSED (for comparisons): 0 = separate copy and flag launches everywhere; "share" = only
// share()'s copies + flags fused (round 3's engine); "fence" = share() and fence() fused, the fence flag
// stored by fence(); unset = the same with the flag stored from the combine kernel's tail.
static bool fused_off() {
  const char* e = getenv("MPJX_IPC_FUSED");
  return e && strcmp(e, "0") == 0;
}
static bool fence_fused_off() {
  const char* e = getenv("MPJX_IPC_FUSED");
  return e && (strcmp(e, "0") == 0 || strcmp(e, "share") == 0);
}

// Largest call (bytes copied by the launch) that takes the fused forms above: every block of a fused
// launch makes its stores visible system-wide before it counts itself in, which eventually costs more
// than the kernel boundary it saves. Round 3 put the limit at 512 KiB (2 MiB: 50.4 fused vs 37.1 us);
// round 4's launches measure the other way on the same A/B (tools/latency ipc 4 2, 4 rank processes on
// one GPU, device sync: 1 MiB 328 -> 262 us, 2 MiB 328 -> 272 us fused, 8 B-256 KiB unchanged,
// profiles/r04/latency_ipc_p4_fuse*_k.json), so the default is 2 MiB — configs[0]'s 1 MiB call at P = 4
// is fused end to end. MPJX_IPC_FUSE_KIB overrides it.
static int64_t fuse_max_bytes() {
  static const int64_t b = [] {
    const char* e = getenv("MPJX_IPC_FUSE_KIB");
    const long k = e ? atol(e) : 2048;
    // capped at 32 MiB: the fused wait + copy-out launch takes at most 4096 blocks of 16 KiB tiles
    return (int64_t)std::min(k >= 0 ? k : 2048, 32768L) << 10;
  }();
  return b;
}

// MPJX_IPC_SYNC=device. Lane j stores seq into peer j's flag[phase][me] (a system-scope release
// through the IPC mapping: everything this stream wrote before, the pushed blocks or this rank's
// result stores, is complete at the kernel boundary ahead of it), then spins until flag[phase][j]
// in this rank's own area reaches seq. Every wave leaves: after `ticks` of the constant wall clock
// it records the timeout in the host-mapped *err and exits, and the call fails at the next wait().
struct FlagPeers {
  unsigned long long* at[kIpcMaxRanks];
};

__global__ __launch_bounds__(64) void k_ipc_flags(FlagPeers peer, const unsigned long long* mine, int P, int me,
                                                   unsigned long long seq, long long ticks, int* err,
                                                   const int* failed, int store) {
  const int j = threadIdx.x;
  if (j >= P || j == me) return;
  if (store) __hip_atomic_store(peer.at[j], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  const long long t0 = wall_clock64();
  for (unsigned it = 1; __hip_atomic_load(mine + j, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < seq; it++) {
    // a rank that left the call marks the world in the shared segment (mapped here from the host):
    // give up at once instead of at the time limit
    const bool gone = (it & 63) == 0 && __hip_atomic_load(failed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (gone || wall_clock64() - t0 > ticks) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

int IpcTransport::dev_signal(int phase, hipStream_t s, bool store) {
  FlagPeers fp{};
  for (int j = 0; j < P; j++)
    if (j != me)
      fp.at[j] = (unsigned long long*)(peers[j].base + 2 * peers[j].cap) + (size_t)phase * kIpcMaxRanks + me;
  hipLaunchKernelGGL(k_ipc_flags, dim3(1), dim3(64), 0, s, fp, flags + (size_t)phase * kIpcMaxRanks, P, me, seq,
                     wait_ticks, derr, dfailed, store ? 1 : 0);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) IPC_LOCAL(fail(MPJX_ERR_HIP, "ipc flag kernel: %s", hipGetErrorString(e)));
  return MPJX_SUCCESS;
}

int IpcTransport::wait(hipStream_t s) {
  HIPCHK(hipStreamSynchronize(s));
  if (herr && __atomic_load_n(herr, __ATOMIC_ACQUIRE)) {
    seg->failed.store(1, std::memory_order_release);
    return fail(MPJX_ERR_INTERNAL, "ipc device wait: rank %d gave up after %.0f s (a peer died, failed or called "
                "a different collective); MPJX_IPC_TIMEOUT_S sets the limit", me, timeout_s());
  }
  return MPJX_SUCCESS;
}

int IpcTransport::map_peers() {
  for (int j = 0; j < P; j++) {
    if (j == me) continue;
    const IpcRow& row = seg->row[j];
    hipIpcMemHandle_t h;
    memcpy(&h, row.handle, sizeof h);
    void* b = nullptr;
    HIPCHK(hipIpcOpenMemHandle(&b, h, hipIpcMemLazyEnablePeerAccess));
    peers[j] = Peer{(char*)b, (size_t)row.cap};
    if (debug()) fprintf(stderr, "[mpjx ipc r%d] mapped rank %d staging at %p (2 x %zu B)\n", me, j, b, (size_t)row.cap);
  }
  return MPJX_SUCCESS;
}


int IpcTransport::share(const void* send, size_t send_bytes, void* recv, size_t recv_bytes, const Parts& parts,
                        hipStream_t s, std::vector<std::vector<const void*>>* all, bool /*leader*/) {
  if (send_bytes > cap || recv_bytes > cap)  // the collectives window their calls to cap
    IPC_LOCAL(fail(MPJX_ERR_INTERNAL, "ipc: %zu/%zu B exceed the %zu B staging window", send_bytes, recv_bytes, cap));
  // push: block j of send -> slot `me` of rank j's `in` region; every rank's kernel then reads its
  // own block of every rank's send from local HBM. Needs P slots of the largest block per region
  // (the same decision on every rank: the partition is the same everywhere). Slots are 4 KiB apart
  // beyond the block: P streams at a power-of-two stride collide in HBM (K_MST P=8 over 32 MiB slots
  // 50.0 vs 47.2 us cold, profiles/r03/slot_skew_cold*.jsonl).
  size_t slot = 0;
  for (size_t l : parts.len) slot = std::max(slot, (l + 255) & ~(size_t)255);
  slot += kSlotSkew;
  bool push = !pull && (int)parts.len.size() == P && (size_t)P * slot <= cap;
  for (int j = 0; push && j < P; j++) push = j == me || (size_t)P * slot <= peers[j].cap;
  if (dsync && __atomic_load_n(herr, __ATOMIC_ACQUIRE))
    IPC_LOCAL(fail(MPJX_ERR_INTERNAL, "ipc world: an earlier device wait timed out; the communicator is unusable"));
  hipError_t err = hipSuccess;
  CopyList cl;
  if (push) {
    for (int j = 0; j < P; j++)
      if (j != me && parts.len[j]) cl.add(in_of(j) + (size_t)me * slot, (const char*)send + parts.off[j], parts.len[j]);
  } else if (send_bytes) {
    cl.add(stage, send, (int64_t)send_bytes);
  }
  if (dsync) {  // stream order covers the previous copy-out; the flags order the ranks
    seq++;
    int64_t copy_bytes = 0;
    for (int i = 0; i < cl.n; i++) copy_bytes += cl.bytes[i];
    // the copies and the flag store + wait in one launch — for calls up to fuse_max_bytes(): every
    // block of the fused kernel makes its stores visible system-wide before counting itself in
    if (cl.n > 0 && copy_bytes <= fuse_max_bytes() && !fused_off()) {
      FlagTail f{};
      for (int j = 0; j < P; j++)
        if (j != me) f.peer[j] = (unsigned long long*)(peers[j].base + 2 * peers[j].cap) + me;
      f.mine = flags;
      f.P = P;
      f.me = me;
      f.seq = seq;
      f.ticks = wait_ticks;
      f.err = derr;
      f.failed = dfailed;
      f.counter = (unsigned*)(flags + 2 * kIpcMaxRanks);
      err = launch_copies_flags(cl, f, s);
      if (err != hipSuccess) IPC_LOCAL(fail(MPJX_ERR_HIP, "ipc staging: %s", hipGetErrorString(err)));
    } else {
      err = launch_copies(cl, s);
      if (err != hipSuccess) IPC_LOCAL(fail(MPJX_ERR_HIP, "ipc staging: %s", hipGetErrorString(err)));
      CHK(dev_signal(0, s));
    }
  } else {
    err = launch_copies(cl, s);
    if (err == hipSuccess) err = hipStreamSynchronize(s);  // staged / pushed, and the previous copy-out is done
    if (err != hipSuccess) IPC_LOCAL(fail(MPJX_ERR_HIP, "ipc staging: %s", hipGetErrorString(err)));
    CHK(hbarrier());
  }
  all->assign(P, {});
  const size_t mine = push ? parts.off[me] : 0;
  // This rank's own result block goes straight into its recv buffer (its own device memory, no IPC
  // involved); fence() copies only the peers' blocks out of the staging region. recv has the send
  // layout (Allreduce, Scan, Reduce at the root) or is this rank's block alone (Reduce_scatter).
  void* own_out = out_of(me);
  own_lo = own_hi = 0;
  if (recv && recv_bytes) {
    if (recv_bytes == send_bytes && (int)parts.len.size() == P) {
      own_lo = parts.off[me];
      own_hi = std::min(recv_bytes, own_lo + parts.len[me]);
    } else {
      own_hi = recv_bytes;
    }
    own_out = recv;
  }
  for (int j = 0; j < P; j++) {
    if (!push && j != me && peers[j].cap < send_bytes)
      IPC_LOCAL(fail(MPJX_ERR_INTERNAL, "ipc: rank %d stages %zu B, rank %d sends %zu (mismatched windows)", j,
                     peers[j].cap, me, send_bytes));
    const void* in;
    if (j == me) in = send;
    else if (push) in = (const void*)((uintptr_t)(stage + (size_t)j * slot) - mine);  // base + off[me] = slot j
    else in = in_of(j);
    (*all)[j] = {in, j == me ? (const void*)own_out : (const void*)out_of(j)};
  }
  pend_recv = recv;
  pend_bytes = recv_bytes;
  return MPJX_SUCCESS;
}

// The combine kernel of a small device-synchronised call stores this rank's phase-B flag from its tail
// (k_pway, PwayArgs::tail) when the collective arms it for its one combine launch: the peers' fence waits
// then end with that kernel, and fence() only waits. Up to fuse_max_bytes() per call (beyond, every
// block's system-scope fence costs more than the kernel boundary it saves, as for share()'s fused launch).
const TailSignal* IpcTransport::tail_arm(size_t bytes, unsigned long long* sq) {
  const char* e = getenv("MPJX_IPC_FUSED");
  if (!dsync || !tail_dev || fence_fused_off() || (e && strcmp(e, "fence") == 0) || (int64_t)bytes > fuse_max_bytes())
    return nullptr;
  *sq = seq;  // share() of this call numbered it
  return tail_dev;
}

int IpcTransport::fence(hipStream_t s, bool /*leader*/, bool signalled, bool /*blocking*/) {
  const size_t b = pend_bytes;
  pend_bytes = 0;
  CopyList cl;  // the peers' blocks: everything but [own_lo, own_hi), which this rank wrote in place
  if (own_lo > 0) cl.add(pend_recv, stage + cap, (int64_t)std::min(own_lo, b));
  if (own_hi < b) cl.add((char*)pend_recv + own_hi, stage + cap + own_hi, (int64_t)(b - own_hi));
  int64_t copy_bytes = 0;
  for (int i = 0; i < cl.n; i++) copy_bytes += cl.bytes[i];
  if (dsync && cl.n > 0 && copy_bytes <= fuse_max_bytes() && !fence_fused_off()) {
    // small calls: the flags and the copy-out in ONE launch (every block stores this rank's flag and
    // waits for the peers' before copying its tile) — one kernel boundary less on the call's chain
    FlagTail f{};
    for (int j = 0; j < P; j++)
      if (j != me) f.peer[j] = (unsigned long long*)(peers[j].base + 2 * peers[j].cap) + (size_t)kIpcMaxRanks + me;
    f.mine = flags + kIpcMaxRanks;
    f.P = P;
    f.me = me;
    f.seq = seq;
    f.ticks = wait_ticks;
    f.err = derr;
    f.failed = dfailed;
    f.store = signalled ? 0 : 1;
    const hipError_t err = launch_flags_copies(cl, f, s);
    if (err != hipSuccess) IPC_LOCAL(fail(MPJX_ERR_HIP, "ipc fence: %s", hipGetErrorString(err)));
    return MPJX_SUCCESS;
  }
  if (dsync) {
    CHK(dev_signal(1, s, !signalled));  // this rank's result stores are done, and so are every other rank's
  } else {
    hipError_t err = hipStreamSynchronize(s);  // this rank's kernel wrote its block into every rank's `out`
    if (err != hipSuccess) IPC_LOCAL(fail(MPJX_ERR_HIP, "hipStreamSynchronize: %s", hipGetErrorString(err)));
    CHK(hbarrier());  // ... and so did every other rank's
  }
  if (cl.n) HIPCHK(launch_copies(cl, s));
  return MPJX_SUCCESS;
}

// Blocks move in rounds: round k carries bytes [k*piece, (k+1)*piece) of every block, so any number
// of blocks of any size fits the fixed staging region (piece = cap/P, 256-B aligned).
int IpcTransport::exchange(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s) {
  if ((int)sends.size() > kIpcMaxRanks || (int)recvs.size() > CopyList::kMax)
    IPC_LOCAL(fail(MPJX_ERR_INTERNAL, "ipc: too many blocks in one exchange"));
  const size_t piece = std::max<size_t>(256, (cap / P) & ~(size_t)255);
  size_t need = 0;
  for (const Xfer& x : sends) need = std::max(need, (x.bytes + piece - 1) / piece);
  for (const Xfer& x : recvs) need = std::max(need, (x.bytes + piece - 1) / piece);
  IpcRow& row = seg->row[me];
  row.rounds = (int32_t)need;
  hipError_t err = hipStreamSynchronize(s);  // the blocks to send are complete
  if (err != hipSuccess) IPC_LOCAL(fail(MPJX_ERR_HIP, "hipStreamSynchronize: %s", hipGetErrorString(err)));
  CHK(hbarrier());
  int rounds = 0;
  for (int j = 0; j < P; j++) rounds = std::max(rounds, (int)seg->row[j].rounds);
  CHK(hbarrier());  // every rank has read the round counts before any row is rewritten
  for (int k = 0; k < rounds; k++) {
    const size_t lo = (size_t)k * piece;
    row.nsend = (int32_t)sends.size();
    CopyList cl;
    for (size_t i = 0; i < sends.size(); i++) {
      const size_t len = sends[i].bytes > lo ? std::min(piece, sends[i].bytes - lo) : 0;
      row.sends[i] = IpcSend{sends[i].peer, 0, (unsigned long long)(i * piece), (unsigned long long)len};
      if (len) cl.add(stage + i * piece, (const char*)sends[i].ptr + lo, (int64_t)len);
    }
    err = launch_copies(cl, s);
    if (err == hipSuccess) err = hipStreamSynchronize(s);
    if (err != hipSuccess) IPC_LOCAL(fail(MPJX_ERR_HIP, "ipc staging: %s", hipGetErrorString(err)));
    CHK(hbarrier());
    // pull this round's piece of every block addressed to this rank out of its owner's region, from
    // every owner at once
    CopyList pl;
    for (const Xfer& r : recvs) {
      const IpcRow& pr = seg->row[r.peer];
      int q = -1;
      for (int i = 0; i < pr.nsend; i++)
        if (pr.sends[i].peer == me) { q = i; break; }
      const size_t len = r.bytes > lo ? std::min(piece, r.bytes - lo) : 0;
      if (q < 0 || pr.sends[q].bytes != len)
        IPC_LOCAL(fail(MPJX_ERR_INTERNAL, "ipc exchange mismatch: rank %d expects %zu B from %d in round %d, got %llu",
                       me, len, r.peer, k, q < 0 ? 0ull : pr.sends[q].bytes));
      if (len) pl.add((char*)r.ptr + lo, in_of(r.peer) + pr.sends[q].off, (int64_t)len);
    }
    err = launch_copies(pl, s);
    if (err != hipSuccess) IPC_LOCAL(fail(MPJX_ERR_HIP, "ipc pull: %s", hipGetErrorString(err)));
    err = hipStreamSynchronize(s);
    if (err != hipSuccess) IPC_LOCAL(fail(MPJX_ERR_HIP, "hipStreamSynchronize: %s", hipGetErrorString(err)));
    CHK(hbarrier());  // a sender restages only once every puller has copied this round
  }
  return MPJX_SUCCESS;
}

int IpcTransport::barrier(hipStream_t s) {
  hipError_t err = hipStreamSynchronize(s);
  if (err != hipSuccess) IPC_LOCAL(fail(MPJX_ERR_HIP, "hipStreamSynchronize: %s", hipGetErrorString(err)));
  return hbarrier();
}

extern "C" int mpjx_comm_init_ipc(mpjx_comm_t* comm, int nranks, const mpjx_unique_id* id, int rank, int device) {
  if (!comm || !id) return fail(MPJX_ERR_ARG, "NULL argument");
  if (nranks < 1 || nranks > kIpcMaxRanks || rank < 0 || rank >= nranks)
    return fail(MPJX_ERR_ARG, "rank %d of %d (ipc worlds hold at most %d ranks)", rank, nranks, kIpcMaxRanks);
  CHK(check_device(device));
  unsigned long long h = 1469598103934665603ull;  // FNV-1a of the id names the segment
  for (size_t i = 0; i < sizeof id->internal; i++) h = (h ^ (unsigned char)id->internal[i]) * 1099511628211ull;
  char name[64];
  snprintf(name, sizeof name, "/mpjx-ipc-%016llx", h);
  const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
  if (fd < 0) return fail(MPJX_ERR_INTERNAL, "shm_open(%s): %s", name, strerror(errno));
  if (ftruncate(fd, sizeof(IpcSeg)) != 0) {
    const int e = errno;
    close(fd);
    return fail(MPJX_ERR_INTERNAL, "ftruncate(%s): %s", name, strerror(e));
  }
  void* mem = mmap(nullptr, sizeof(IpcSeg), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (mem == MAP_FAILED) return fail(MPJX_ERR_INTERNAL, "mmap(%s): %s", name, strerror(errno));
  auto t = std::make_unique<IpcTransport>();
  t->seg = (IpcSeg*)mem;
  t->me = rank;
  t->P = nranks;
  t->peers.resize(nranks);
  IpcSeg* seg = t->seg;
  // every rank maps the segment before rank 0 removes its name (the mappings stay valid)
  seg->attached.fetch_add(1, std::memory_order_acq_rel);
  if (!wait_for([&] { return seg->attached.load(std::memory_order_acquire) >= (uint32_t)nranks; }, seg)) {
    seg->failed.store(1, std::memory_order_release);
    if (rank == 0) shm_unlink(name);
    return fail(MPJX_ERR_INTERNAL, "ipc init: only %u of %d ranks attached to %s within %.0f s",
                seg->attached.load(), nranks, name, timeout_s());
  }
  if (rank == 0) shm_unlink(name);
  // the staging region: allocated, exported and mapped by every peer once, here
  const char* ev = getenv("MPJX_IPC_STAGE_MIB");
  const long mib = ev && atol(ev) > 0 ? atol(ev) : 256;
  // + room for the 256-B rounding and the 4 KiB skew of up to kIpcMaxRanks block slots
  // (window_bytes()), so a vector of exactly MPJX_IPC_STAGE_MIB runs as ONE window, not a full window
  // and a small tail
  t->cap = ((size_t)mib << 20) + (size_t)kIpcMaxRanks * IpcTransport::kSlotPad;
  if (hipSetDevice(device) != hipSuccess) IPC_LOCAL(fail(MPJX_ERR_HIP, "hipSetDevice(%d)", device));
  {
    // Peers write into this region through their IPC mappings (over xGMI when each rank has its own
    // GPU) while this rank's kernels read it locally, so by default it is fine-grained memory, whose
    // cached lines do not outlive a kernel boundary, as the buffers RCCL's peers write into are; a
    // coarse-grained region's L2 lines are only kept coherent for this device's own writes.
    // Measured cost on one GPU: none (P=4 push 0.981 ms fine vs 0.985 ms coarse, 0.996 ms uncached).
    // MPJX_IPC_STAGE_ALLOC=coarse (hipMalloc) | fine (default) | uncached selects the class.
    const char* av = getenv("MPJX_IPC_STAGE_ALLOC");
    const unsigned aflag = !av || strcmp(av, "fine") == 0 ? hipDeviceMallocFinegrained
                           : strcmp(av, "uncached") == 0  ? hipDeviceMallocUncached
                                                          : 0u;
    // + the flag area of MPJX_IPC_SYNC=device: [A: kIpcMaxRanks][B: kIpcMaxRanks] sequence numbers
    const size_t bytes = 2 * t->cap + kIpcFlagBytes;
    hipError_t e = aflag ? hipExtMallocWithFlags((void**)&t->stage, bytes, aflag) : hipMalloc((void**)&t->stage, bytes);
    if (e == hipSuccess) e = hipMemset(t->stage + 2 * t->cap, 0, kIpcFlagBytes);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    hipIpcMemHandle_t h;
    if (e == hipSuccess) e = hipIpcGetMemHandle(&h, t->stage);
    if (e != hipSuccess)
      IPC_LOCAL(fail(MPJX_ERR_HIP, "ipc staging region (2 x %ld MiB): %s", mib, hipGetErrorString(e)));
    memcpy(seg->row[rank].handle, &h, sizeof h);
    seg->row[rank].cap = t->cap;
    // MPJX_IPC_SYNC=device needs staging whose lines do not outlive a kernel boundary (not coarse)
    // "device": only when every rank has a GPU of its own, the deployment it is built for; rank
    // processes sharing a GPU would spin their flag waits beside peers' kernels competing for the
    // same hardware queues, so there the calls stay host-synchronised (a conservative choice, not a
    // measured stall). "device-shared" uses it regardless (the one-GPU tests and latency runs).
    const char* sv = getenv("MPJX_IPC_SYNC");
    const int want = !sv || aflag == 0 ? 0 : strcmp(sv, "device") == 0 ? 1 : strcmp(sv, "device-shared") == 0 ? 2 : 0;
    t->dsync = want != 0;
    memset(seg->row[rank].bus, 0, sizeof seg->row[rank].bus);
    if (hipDeviceGetPCIBusId(seg->row[rank].bus, (int)sizeof seg->row[rank].bus - 1, device) != hipSuccess)
      snprintf(seg->row[rank].bus, sizeof seg->row[rank].bus, "dev%d", device);
    t->flags = (unsigned long long*)(t->stage + 2 * t->cap);
    if (t->dsync) {
      int khz = 0;
      hipError_t e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device);
      if (e == hipSuccess) e = hipHostMalloc((void**)&t->herr, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent);
      if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&t->derr, t->herr, 0);
      if (e == hipSuccess) e = hipHostRegister(seg, sizeof(IpcSeg), hipHostRegisterMapped);
      if (e == hipSuccess) t->seg_registered = true;
      if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&t->dfailed, (void*)&seg->failed, 0);
      if (e != hipSuccess) IPC_LOCAL(fail(MPJX_ERR_HIP, "ipc device sync setup: %s", hipGetErrorString(e)));
      *t->herr = 0;
      t->wait_ticks = (long long)(timeout_s() * 1e3 * (khz > 0 ? khz : 100000));
    }
    seg->row[rank].dsync = want;
    const char* mv = getenv("MPJX_IPC_MODE");
    t->pull = mv && strcmp(mv, "pull") == 0;
    seg->row[rank].pull = t->pull;
  }
  CHK(t->hbarrier());
  for (int j = 0; j < nranks; j++) {  // one rank waiting on flags its peers never store would hang
    if (seg->row[j].dsync != seg->row[rank].dsync)
      IPC_LOCAL(fail(MPJX_ERR_ARG, "ipc init: ranks %d and %d have different MPJX_IPC_SYNC settings (set the same "
                     "on every rank)", rank, j));
    // a pushing rank reads the slots peers push into; a pulling rank overwrites them: silently wrong
    if (seg->row[j].pull != seg->row[rank].pull)
      IPC_LOCAL(fail(MPJX_ERR_ARG, "ipc init: ranks %d and %d have different MPJX_IPC_MODE settings (set the same "
                     "on every rank)", rank, j));
  }
  // Rank processes sharing one GPU are a rehearsal of the one-process-per-GPU deployment. With
  // several processes on one MI355X, a kernel can be served a stale translation of a 2 MiB page its
  // process freed and re-allocated at the same virtual address, i.e. read another process's memory
  // (tools/va_alias_probe.cpp: 8 processes, 19 of 195k fresh 16 MiB buffers; 4 processes beside a
  // fifth holding a context, 3 of 41k; DMA read-back correct every time). That is how
  // the one wrong IPC result of round 1 arose, and no process count below which it never happens has
  // been found, so two rank processes on one GPU are refused unless MPJX_IPC_OVERSUBSCRIBE=1 (callers
  // that do not free device memory while the world exists: the one-GPU tests and rehearsals).
  {
    const char* lv = getenv("MPJX_IPC_MAX_PER_GPU");
    const int lim = lv && atoi(lv) > 0 ? atoi(lv) : 1;
    const char* ov = getenv("MPJX_IPC_OVERSUBSCRIBE");
    int most = 0;
    for (int i = 0; i < nranks; i++) {
      int k = 0;
      for (int j = 0; j < nranks; j++) k += strncmp(seg->row[i].bus, seg->row[j].bus, sizeof seg->row[i].bus) == 0;
      most = std::max(most, k);
    }
    if (most > lim && !(ov && strcmp(ov, "1") == 0))
      IPC_LOCAL(fail(MPJX_ERR_UNSUPPORTED, "ipc init: %d rank processes share one GPU (limit %d, "
                     "MPJX_IPC_MAX_PER_GPU): kernels of processes that oversubscribe one MI355X can read a "
                     "stale page translation after free/re-allocation; run one rank per GPU, or set "
                     "MPJX_IPC_OVERSUBSCRIBE=1 if no rank frees device memory while the world exists", most, lim));
  }
  if (seg->row[rank].dsync == 1)  // the same rows on every rank: the same decision
    for (int i = 0; i < nranks && t->dsync; i++)
      for (int j = i + 1; j < nranks && t->dsync; j++)
        if (strncmp(seg->row[i].bus, seg->row[j].bus, sizeof seg->row[i].bus) == 0) {
          t->dsync = false;
          if (debug()) fprintf(stderr, "[mpjx ipc r%d] ranks %d and %d share GPU %s: host-synchronised calls\n",
                               rank, i, j, seg->row[i].bus);
        }
  IPC_LOCAL(t->map_peers());
  if (t->dsync) {  // the fence-signal targets for the combine kernel's tail: this rank's slot in every peer
    TailSignal ts{};
    for (int j = 0; j < nranks; j++)
      if (j != rank)
        ts.peer[j] = (unsigned long long*)(t->peers[j].base + 2 * t->peers[j].cap) + (size_t)kIpcMaxRanks + rank;
    ts.P = nranks;
    ts.me = rank;
    ts.counter = (unsigned*)(t->flags + 2 * kIpcMaxRanks) + 1;  // [0]: share()'s fused launch
    hipError_t e = hipMalloc((void**)&t->tail_dev, sizeof ts);
    if (e == hipSuccess) e = hipMemcpy(t->tail_dev, &ts, sizeof ts, hipMemcpyHostToDevice);
    if (e != hipSuccess) IPC_LOCAL(fail(MPJX_ERR_HIP, "ipc tail signal: %s", hipGetErrorString(e)));
  }
  CHK(t->hbarrier());  // every rank mapped every region before any is used
  auto c = std::make_unique<mpjx_comm>();
  c->rank = rank;
  c->size = nranks;
  c->device = device;
  IPC_LOCAL(comm_common_init(c.get()));
  c->tr = std::move(t);
  *comm = c.release();
  return MPJX_SUCCESS;
}
