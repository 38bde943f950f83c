// mpjx_engine.hpp — internal (C++) structure of libmpjx: transports, communicator, collectives.
//
// Every reduction collective of the reference (src/mpi/PureIntracomm.java:1923-2545) is re-planned
// for one node of fully connected MI355X GPUs as
//     exchange #1 (block j of every rank -> rank j, all xGMI links at once)
//  -> ONE P-way HIP combine per rank that evaluates the reference's combine order per element
//  -> exchange #2 (all-gather / gather-to-root / result scatter)
// so each byte crosses a link at most twice and HBM sees one read of each operand block.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <condition_variable>
#include <memory>
#include <atomic>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "mpjx_kernels.hpp"

namespace mpjx {

// One point-to-point transfer of an exchange step.
struct Xfer {
  int peer;
  void* ptr;
  size_t bytes;
};

// Byte transport between the ranks of a communicator. exchange() is a grouped set of sends and
// receives that all progress together and complete in order on `s`.
struct Transport {
  virtual ~Transport() = default;
  virtual int exchange(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s) = 0;
  virtual int barrier(hipStream_t s) = 0;
  // Wait until `s` has drained (the blocking end of a call). RCCL overrides it to poll the
  // communicator's asynchronous error state while it waits.
  virtual int wait(hipStream_t s);
  virtual const char* name() const = 0;
  // This rank leaves a collective early (bad arguments): transports that can, make the other ranks'
  // matching calls fail instead of waiting for it.
  virtual void abort_world() {}
  // A collective call of this rank returned an error (the C-ABI entry points, `ended` in
  // mpjx_collectives.hip): the rank skipped the collective or stopped part-way, so the world is out of
  // step — the same as leaving early. Multicore and IPC worlds are marked failed (every peer's waiting
  // and later call errors out instead of waiting for this rank forever); RCCL aborts at P > 1.
  virtual void call_failed() { abort_world(); }
  // All-to-all with per-peer byte counts/displacements (entry `me` may be non-zero: a local copy).
  virtual int alltoallv(int me, const char* send, const std::vector<size_t>& scount,
                        const std::vector<size_t>& sdispl, char* recv, const std::vector<size_t>& rcount,
                        const std::vector<size_t>& rdispl, hipStream_t s);
  // In-place all-gather of equal blocks: rank r's `bytes` live at buf + r*bytes.
  virtual int allgather_equal(int me, int P, char* buf, size_t bytes, hipStream_t s);
  // A second lane over the same ranks whose exchanges may run concurrently with this one's on another
  // stream (the chunk pipeline's all-gathers beside its exchange #1). Creating it may be collective:
  // every rank asks for it at the same point of the same call. Default: this transport (exchanges are
  // host rendezvous, their device copies overlap on different streams anyway).
  virtual Transport* lane2() { return this; }
};

// One process per GPU: RCCL point-to-point over xGMI (ncclSend/ncclRecv inside one group, which
// RCCL maps onto the direct links of the fully connected node).
// Exchange steps with equal blocks use RCCL's own collectives (ncclAllToAll / ncclAllGather), ragged
// ones ncclAllToAllv / grouped ncclSend-ncclRecv; MPJX_RCCL_P2P=1 (at init) forces grouped point-to-point.
struct RcclTransport final : Transport {
  ncclComm_t nccl = nullptr;
  int* dflag = nullptr;  // 4-int device buffer: barrier() and the init-time agreement (agree())
  // Routing decided ONCE per communicator, at mpjx_comm_init_rank, from this rank's environment and
  // checked equal on every rank there (a rank taking ncclAllToAll while a peer posts grouped
  // send/recv, or ncclAllReduce while a peer runs the exchange engine, would hang or corrupt):
  bool p2p_only = false;  // MPJX_RCCL_P2P=1: exchanges as grouped ncclSend/ncclRecv
  int native = 0;         // MPJX_RCCL_NATIVE=1 -> 1 (any P), MPJX_RCCL_NATIVE_P2=1 -> 2 (P = 2 only)
  bool aborted = false;   // an RCCL error, MPJX_RCCL_TIMEOUT_S or a rank-local rejection ended this communicator
  int nranks = 1;
  RcclTransport* parent = nullptr;  // set on the pipeline's second lane: an abort ends both communicators
  bool p2p() const { return p2p_only; }
  // ncclCommAbort on both lanes; every later call fails in usable(). After any failure between a
  // rank's first and last RCCL call of a collective — or a rejection before its first — this rank's
  // operation sequence no longer matches its peers': its next call would pair with their pending one.
  void abort_comms();
  // A rank leaving a collective early (reject() in mpjx_collectives.hip) at P > 1: abort, so its later
  // calls fail instead of pairing with the peers' earlier operation. The peers cannot be released from
  // here (RCCL's kernels on their GPUs wait for this rank's data): they wait as MPI ranks do, unless
  // MPJX_RCCL_TIMEOUT_S ends the wait.
  void abort_world() override;
  // A synchronous RCCL failure: abort (above), MPJX_ERR_RCCL naming the call.
  int failed_call(const char* what, ncclResult_t r);
  // Reads the routing knobs above and checks them equal on every rank (one small ncclAllReduce, MAX of
  // each value and of its negation); MPJX_ERR_ARG on every rank if any two ranks differ.
  int agree(hipStream_t s);
  ~RcclTransport() override;
  // Polls hipStreamQuery and ncclCommGetAsyncError instead of blocking in hipStreamSynchronize: a
  // peer that failed (RCCL reports it asynchronously) or, with MPJX_RCCL_TIMEOUT_S set, a call that
  // does not complete in time aborts the communicator (ncclCommAbort) and returns MPJX_ERR_RCCL
  // instead of hanging the rank (the JNI shim turns it into mpi.MPIException).
  int wait(hipStream_t s) override;
  int usable() const;
  int exchange(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s) override;
  int barrier(hipStream_t s) override;
  const char* name() const override { return "rccl"; }
  int alltoallv(int me, const char* send, const std::vector<size_t>& scount, const std::vector<size_t>& sdispl,
                char* recv, const std::vector<size_t>& rcount, const std::vector<size_t>& rdispl,
                hipStream_t s) override;
  int allgather_equal(int me, int P, char* buf, size_t bytes, hipStream_t s) override;
  // RCCL's own ncclAllReduce over typed elements: only where its result is the reference's bit for bit
  // whatever order RCCL combines in (rccl_native_ok in mpjx_collectives.hip, MPJX_RCCL_NATIVE=1).
  int allreduce(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s);
  // RCCL serialises the operations of one communicator, whatever their streams: the second lane is a
  // second communicator over the same ranks (ncclCommSplit, created on first use), so exchange #1 of
  // chunk k+1 and the all-gather of chunk k can drive the links in both directions at once.
  std::unique_ptr<RcclTransport> second;
  Transport* lane2() override;
};

// Direct access between ranks: the collectives' one-kernel engine. share() publishes this rank's send
// buffer (send_bytes, read by peers) and recv buffer (recv_bytes, written by peers) once its stream
// has reached this point, and returns every rank's pair, addressable from this rank's device: rank
// r's P-way kernel then reads block r of every rank's send buffer in place and stores its result
// block straight into every rank's recv buffer. fence(): `s` continues (and the call returns) only
// after every rank's kernel is done. Implemented by SmpTransport (ranks are threads of one process)
// and IpcTransport (ranks are processes; the pairs it returns are its peers' mapped staging buffers).
// The block partition of a direct call (bytes): rank r's P-way kernel reads [off[r], off[r]+len[r])
// of every rank's send buffer. Lets a transport move exactly those blocks ahead of the kernel.
struct Parts {
  std::vector<size_t> off, len;
};

struct Direct {
  virtual ~Direct() = default;
  virtual bool direct_ok() const = 0;  // every rank can load/store every other rank's memory
  virtual bool single() const = 0;     // one device, one process: rank 0 launches for everyone
  virtual int share(const void* send, size_t send_bytes, void* recv, size_t recv_bytes, const Parts& parts,
                    hipStream_t s, std::vector<std::vector<const void*>>* all, bool leader = false) = 0;
  // signalled: the call's last combine kernel already stored this rank's fence flag (tail_arm);
  // blocking: the call returns only once complete (MPJX_FLAG_BLOCKING), so a transport may finish it
  // with a host rendezvous after the launching ranks' streams have drained
  virtual int fence(hipStream_t s, bool leader = false, bool signalled = false, bool blocking = false) = 0;
  virtual size_t window_bytes() const { return SIZE_MAX; }  // largest send/recv extent per share()
  // The fence signal for the combine kernel's tail (IPC device sync, small calls), or nullptr.
  virtual const TailSignal* tail_arm(size_t /*bytes*/, unsigned long long* /*seq*/) { return nullptr; }
};

// Multicore mode (the reference's smpdev: ranks are threads of one process). Ranks rendezvous on
// the host; each receiver pulls its blocks straight from the sender's device buffer
// (hipMemcpyAsync, peer access enabled between distinct devices), ordered by HIP events.
struct SmpWorld {
  int P = 0;
  std::vector<int> devices;
  bool direct = false;  // every rank can load/store every other rank's device memory
  bool single = false;  // every rank on the same device: rank 0 launches the whole collective
  std::vector<std::vector<const void*>> shared;  // share(): pointers published per rank
  std::vector<char> idle;  // share(): the rank's stream had no pending work (no ready event to wait on)
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<int> arrived{0};
  std::atomic<unsigned long long> gen{0};
  std::vector<std::vector<Xfer>> posted;
  std::vector<hipEvent_t> ready, done;
  std::vector<char> synced;  // fence(): the rank's stream drained before the rendezvous (no done[] wait)
  int refs = 0;
  std::atomic<int> failed{0};  // a rank left a collective early: every barrier fails from now on
  // Host-direct Allreduce, result across the host link once (mpjx_collectives.hip, host_once): before
  // share() each rank says whether its recv is page-locked host memory of a synchronous *_host call
  // (host_out); rank 0, launching for all, writes the result into the first such rank's recv only and
  // names it in copy_src[r] for the other such ranks, which copy it host-to-host after the fence.
  // copy_round (set by rank 0 before the fence's barrier, so every rank reads the same value after it):
  // the call ends with one more rendezvous, once every copy is done.
  std::vector<char> host_out;
  std::vector<const void*> copy_src;
  size_t copy_bytes = 0;
  int copy_round = 0;
  int barrier();
  void abort();
};

struct SmpTransport final : Transport, Direct {
  std::shared_ptr<SmpWorld> w;
  int me = 0;
  ~SmpTransport() override;
  int exchange(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s) override;
  int barrier(hipStream_t s) override;
  const char* name() const override { return "smp"; }
  void abort_world() override { w->abort(); }
  bool direct_ok() const override { return w->direct; }
  bool single() const override { return w->single; }
  // Direct access (ranks share an address space): publish this rank's pointers once its stream has
  // reached this point and receive every rank's; on return `s` is ordered after every rank's
  // publish point. fence(): `s` continues only after every rank's stream reached its fence.
  // leader = true (one device): only rank 0's stream waits for every rank's publish point (rank 0
  // then launches the work of all ranks), and fence() orders the other ranks after rank 0's stream.
  int share(const std::vector<const void*>& mine, hipStream_t s, std::vector<std::vector<const void*>>* all,
            bool leader = false);
  int share(const void* send, size_t, void* recv, size_t, const Parts&, hipStream_t s,
            std::vector<std::vector<const void*>>* all, bool leader = false) override {
    return share(std::vector<const void*>{send, recv}, s, all, leader);
  }
  int fence(hipStream_t s, bool leader = false, bool signalled = false, bool blocking = false) override;
};

// Ranks are processes of one node (one per GPU, or several sharing a GPU), with no RCCL. A POSIX
// shared-memory segment (named from the world's unique id) carries a cross-process barrier and one
// row per rank describing its staging region; each rank owns one device staging region [in | out],
// exported once through HIP IPC and mapped by every peer. share() copies the send buffer into the
// rank's `in` half and hands the P-way kernels every rank's (in, out) halves; fence() copies the
// `out` half into the recv buffer. Two modes (MPJX_IPC_MODE, read at init, the same on every rank): "push" (default) —
// share() writes block j of the send buffer straight into rank j's `in` region (one k_copies launch,
// every xGMI link at once), so each kernel reads only local HBM and only its result stores cross the
// links; "pull" — share() copies send into the rank's own `in` and the kernels read the peers' `in`
// over xGMI. Same bytes on the links either way; push trades remote loads for remote stores. User buffers never cross processes: HIP's IPC imports are cached
// per exporting address, and a torch tensor freed and reallocated at the same address came back as
// the old memory (observed on ROCm 7.2). The region is sized once (MPJX_IPC_STAGE_MIB per half,
// default 256) and mapped by every peer at init — re-opening a re-allocated 2 GiB region later hung
// in hipIpcOpenMemHandle on the same image — so longer vectors run as consecutive windows and
// exchange() moves its blocks in rounds of at most cap/P bytes per block.
struct IpcSeg;
struct IpcTransport final : Transport, Direct {
  IpcSeg* seg = nullptr;
  int me = 0, P = 0;
  char* stage = nullptr;           // [in: cap][out: cap], allocated and exported once at init
  size_t cap = 0;
  struct Peer { char* base = nullptr; size_t cap = 0; };
  std::vector<Peer> peers;         // mapped staging of every other rank
  void* pend_recv = nullptr;       // fence(): copy-out of this call's result
  size_t pend_bytes = 0;
  size_t own_lo = 0, own_hi = 0;   // recv bytes this rank's own kernel wrote in place (not copied out)
  // MPJX_IPC_SYNC=device: share()/fence() order the ranks with per-call sequence flags that kernels
  // store into the peers' staging regions and wait on in their own, instead of stream
  // synchronisation + host barrier: the call is enqueued without a host round trip.
  bool dsync = false;
  bool pull = false;               // MPJX_IPC_MODE=pull at init (checked equal on every rank)
  unsigned long long seq = 0;      // direct calls so far (the same on every rank)
  unsigned long long* flags = nullptr;  // this rank's flag area: [A: P][B: P] at stage + 2*cap
  int* herr = nullptr;             // host-mapped: a device wait timed out (every later call fails)
  int* derr = nullptr;             // herr's device address
  const int* dfailed = nullptr;    // the shared segment's `failed` word, mapped for the device waits
  bool seg_registered = false;
  long long wait_ticks = 0;        // device wait limit in wall-clock ticks (MPJX_IPC_TIMEOUT_S)
  // store seq into every peer's flag[phase][me] (unless !store), then wait until every peer's
  // flag[phase][j] in ours reaches seq
  int dev_signal(int phase, hipStream_t s, bool store = true);
  int wait(hipStream_t s) override;
  ~IpcTransport() override;
  int exchange(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t s) override;
  int barrier(hipStream_t s) override;
  const char* name() const override { return "ipc"; }
  void abort_world() override;
  bool direct_ok() const override { return true; }
  bool single() const override { return false; }
  int share(const void* send, size_t send_bytes, void* recv, size_t recv_bytes, const Parts& parts, hipStream_t s,
            std::vector<std::vector<const void*>>* all, bool leader = false) override;
  int fence(hipStream_t s, bool leader = false, bool signalled = false, bool blocking = false) override;
  const TailSignal* tail_arm(size_t bytes, unsigned long long* seq) override;
  TailSignal* tail_dev = nullptr;  // device copy of this rank's fence-signal targets (device sync)
  // room for P block slots of an even partition (each rounded up to 256 B, plus the 4 KiB slot skew
  // of share()'s push layout) in one half
  static constexpr size_t kSlotSkew = 4096;
  static constexpr size_t kSlotPad = 512 + kSlotSkew;
  size_t window_bytes() const override { return cap > (size_t)P * kSlotPad ? cap - (size_t)P * kSlotPad : cap; }
  int hbarrier();                    // host barrier across the processes (with a timeout)
  int map_peers();                   // map every peer's staging region (once, at init)
  char* in_of(int r) const { return r == me ? stage : peers[r].base; }
  char* out_of(int r) const { return r == me ? stage + cap : peers[r].base + peers[r].cap; }
};

}  // namespace mpjx

struct mpjx_comm {
  int rank = 0, size = 1, device = 0;
  hipStream_t stream = nullptr;
  std::unique_ptr<mpjx::Transport> tr;
  // device scratch, grown on demand (slots for received blocks / results, P>8 temporaries)
  char* scratch = nullptr;
  size_t scratch_bytes = 0;
  // host-variant staging
  char* hstage = nullptr;
  size_t hstage_bytes = 0;
  // the host variants' pipeline: its two copy streams and per-chunk events, created on first use and
  // kept (creating them inside every call cost ~5 % of a 256 MiB host Allreduce)
  hipStream_t h2d = nullptr, d2h = nullptr;
  std::vector<hipEvent_t> host_in_ev, host_coll_ev;  // one per chunk: H2D done / collective done
  hipEvent_t last_ev = nullptr;
  hipStream_t last_stream = nullptr;
  bool last_recorded = false;  // last_ev already marks the end of the previous call on last_stream
  // chunked Allreduce pipeline: combine stream + per-chunk events (created on first use)
  hipStream_t cstream = nullptr;
  hipStream_t gstream = nullptr;  // the pipeline's all-gathers (on the transport's second lane)
  std::vector<hipEvent_t> pipe_ev;
  // mpjx_comm_phase_timing: timing events at the phase boundaries of Allreduce calls (measurement)
  bool phase_on = false;
  int phase_engine = 0;  // engine of the last instrumented call: 1 exchange, 2 direct, 3 pipelined
  hipEvent_t phase_ev[4] = {nullptr, nullptr, nullptr, nullptr};
  // with phase timing on, the chunk pipeline's per-chunk intervals (mpjx_comm_pipeline_trace): a base
  // event, then per chunk exchange #1 start/end (call stream), combine start/end (combine stream),
  // all-gather start/end (gather stream)
  std::vector<hipEvent_t> trace_ev;
  int trace_chunks = 0;
  // the form the last *_host call took (mpjx_comm_last_host_form): 1 staged through device buffers
  // (chunk pipeline), 2 host-direct (the kernel loads and stores the page-locked host buffers); 0 none
  int host_form = 0;
  // Device buffers outgrown during the communicator's life, freed only by mpjx_comm_destroy. Growing
  // never frees-then-reallocates: on a GPU shared by several processes, a hipMalloc that gets back
  // the virtual address of a just-freed 2 MiB page can be served the old page's translation in
  // kernels (the page may belong to another process by then) — DESIGN.md §6, tools/va_alias_probe.cpp.
  std::vector<void*> retired;
};

namespace mpjx {
// Make *buf hold at least `need` bytes (grown geometrically, 2 MiB granules). The outgrown buffer is
// retired (kept allocated until the communicator is destroyed) once `s` has drained its users.
int grow_device(mpjx_comm* c, char** buf, size_t* cap, size_t need, hipStream_t s);
}  // namespace mpjx
