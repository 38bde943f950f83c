// mpjx_internal.hpp — declarations shared by the libmpjx translation units (not installed):
// error reporting, status-check macros, the P-way launch dispatcher and the Combine planner that
// maps each reference combine ORDER onto k_pway launches.
#pragma once
#include "../../include/mpjx.h"
#include "mpjx_engine.hpp"

#include <stdint.h>

#include <vector>

namespace mpjx {

// Records a printf-style message for mpjx_last_error() (per thread) and returns `code`.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
const char* type_name(int t);
const char* op_name(int o);
bool is_pair(int t);
// One k_pway launch (P <= MAXP); picks the 16-B vector instantiation when every pointer allows it.
int launch_pway(int op, int type, unsigned flags, int kind, int P, const PwayArgs& a, hipStream_t s);
// MPJX_ERR_ARG unless `p` (non-NULL) is memory a kernel may dereference (device, managed or
// registered host memory).
int check_dev_ptr(const void* p, const char* what);
// Communicator plumbing shared by the transports (mpjx_transport.hip).
int check_device(int device);
int comm_common_init(mpjx_comm* c);

}  // namespace mpjx

#define HIPCHK(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(MPJX_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                  __LINE__);                                                              \
  } while (0)

#define NCCLCHK(expr)                                                                      \
  do {                                                                                     \
    ncclResult_t r_ = (expr);                                                              \
    if (r_ != ncclSuccess)                                                                 \
      return fail(MPJX_ERR_RCCL, "%s: %s (%s:%d)", #expr, ncclGetErrorString(r_), __FILE__, \
                  __LINE__);                                                               \
  } while (0)

#define CHK(expr)              \
  do {                         \
    int c_ = (expr);           \
    if (c_ != MPJX_SUCCESS) return c_; \
  } while (0)

#define COMM_ARG(c) \
  if (!(c)) return fail(MPJX_ERR_ARG, "comm is NULL")

namespace mpjx {

// Stack of device temporaries for P > MAXP compositions (carved from the comm scratch tail).
struct TempStack {
  char* base = nullptr;
  size_t cap = 0, top = 0, elt = 0;
  void* push(int64_t n) {
    size_t b = ((size_t)n * elt + 255) & ~(size_t)255;
    if (top + b > cap) return nullptr;
    void* p = base + top;
    top += b;
    return p;
  }
};

// Maps each reference combine ORDER onto k_pway launches. Byte order (MPJX_FLAG_SEND_BIG_ENDIAN /
// MPJX_FLAG_RECV_BIG_ENDIAN, the same on every rank like `type` and `op`): the inputs handed to a
// public method are "leaves" — user send data, or raw copies of it moved by an exchange — in the send
// order, and its outputs are "finals" — user recv, or buffers moved raw into it — in the recv order.
// The kernels swap in registers (PwayArgs::swap_in/swap_out); the temporaries of the P > 8
// compositions are native. No separate byte-swap pass over the vector.
struct Combine {
  int op, type;
  unsigned flags;
  int esz;
  hipStream_t s;
  TempStack* tmp;

  int word() const { return mpjx_type_size(type & 0xff); }
  bool sbe() const { return (flags & MPJX_FLAG_SEND_BIG_ENDIAN) && word() > 1; }
  bool rbe() const { return (flags & MPJX_FLAG_RECV_BIG_ENDIAN) && word() > 1; }
  // swap_in mask for P inputs that are all leaves, except input 0 when it is a native temporary
  unsigned leaf_mask(int P, bool first_native = false) const {
    if (!sbe()) return 0;
    unsigned m = (P >= 32) ? ~0u : ((1u << P) - 1);
    return first_native ? (m & ~1u) : m;
  }
  // The IPC device-sync tail (TailSignal): armed around ONE single-launch combine call, the launch
  // carries it; a second launch in the same armed window is a bug (the signal would precede it).
  const TailSignal* tail = nullptr;
  unsigned long long tail_seq = 0;
  bool tail_used = false;
  void arm_tail(const TailSignal* t, unsigned long long seq) {
    tail = t;
    tail_seq = seq;
    tail_used = false;
  }
  bool disarm_tail() {  // true if a kernel carried the signal (else the fence must store it)
    const bool u = tail_used;
    tail = nullptr;
    tail_used = false;
    return u;
  }

  int launch(int kind, int P, PwayArgs& a, unsigned in_mask, bool out_be) {
    a.swap_in = in_mask;
    a.swap_out = out_be ? 1u : 0u;
    if (tail) {
      if (tail_used) return fail(MPJX_ERR_INTERNAL, "device-sync tail armed on a multi-launch combine");
      a.tail = tail;
      a.tail_seq = tail_seq;
      tail_used = true;
    }
    return launch_pway(op, type, flags, kind, P, a, s);
  }

  // dst = src (device), byte-swapped when `swap`. 16-B aligned pairs take k_copies (one 16 KiB tile
  // per block, non-temporal beyond 64 MiB: the combine's stream shape), which outruns the runtime's
  // D2D blit (profiles/r02/copy_vs_blit.json); other alignments go to hipMemcpyAsync.
  int copy_o(void* dst, const void* src, int64_t n, bool swap) {
    if (n <= 0) return MPJX_SUCCESS;
    if (swap) {
      HIPCHK(launch_bswap(dst, src, n * esz, word(), s));
      return MPJX_SUCCESS;
    }
    if (dst == src) return MPJX_SUCCESS;
    if ((((uintptr_t)dst | (uintptr_t)src) & 15u) == 0) {
      CopyList cl;
      cl.add(dst, src, n * esz);
      HIPCHK(launch_copies(cl, s));
    } else {
      HIPCHK(hipMemcpyAsync(dst, src, (size_t)n * esz, hipMemcpyDeviceToDevice, s));
    }
    return MPJX_SUCCESS;
  }
  // leaf -> final (Reduce's arraycopy send -> recv at P = 1, PureIntracomm.java:1937)
  int copy(void* dst, const void* src, int64_t n) { return copy_o(dst, src, n, sbe() != rbe()); }
  // final -> final (a result moved to another output buffer)
  int copy_raw(void* dst, const void* src, int64_t n) { return copy_o(dst, src, n, false); }

  // out = in[P-1] (op) (... (op) (in[1] (op) in[0])); inputs are leaves (input 0 native when
  // first_native), out is a final (native when !out_final)
  int fold_o(int P, const void* const* in, bool first_native, void* out, bool out_final, int64_t n) {
    if (n <= 0) return MPJX_SUCCESS;
    const bool obe = out_final && rbe();
    if (P == 1) return copy_o(out, in[0], n, (leaf_mask(1, first_native) != 0) != obe);
    if (P <= MAXP) {
      PwayArgs a{};
      for (int p = 0; p < P; p++) a.in[p] = in[p];
      a.out[0] = out;
      a.n = n;
      return launch(K_FOLD, P, a, leaf_mask(P, first_native), obe);
    }
    // chunked left-to-right fold through a native temporary (out may alias a later input)
    void* t = tmp->push(n);
    if (!t) return fail(MPJX_ERR_INTERNAL, "scratch temporaries exhausted (P=%d)", P);
    CHK(fold_o(MAXP, in, first_native, t, false, n));
    for (int k = MAXP; k < P; k += MAXP - 1) {
      const void* lst[MAXP];
      int m = 0;
      lst[m++] = t;
      for (int j = k; j < P && m < MAXP; j++) lst[m++] = in[j];
      CHK(fold_o(m, lst, true, t, false, n));
    }
    CHK(copy_o(out, t, n, obe));
    tmp->top -= ((size_t)n * esz + 255) & ~(size_t)255;
    return MPJX_SUCCESS;
  }
  int fold(int P, const void* const* in, void* out, int64_t n) { return fold_o(P, in, false, out, true, n); }

  // out = MST_Reduce tree over in[l..r] (leaves) rooted at `root` (absolute rank index)
  int mst_o(const void* const* in, int l, int r, int root, void* out, bool out_final, int64_t n) {
    if (n <= 0) return MPJX_SUCCESS;
    const int P = r - l + 1;
    if (P == 1) return copy_o(out, in[l], n, sbe() != (out_final && rbe()));
    if (P == 2) {  // acc = in[root], recv = the other
      const void* lst[2] = {in[root], in[root == l ? r : l]};
      return fold_o(2, lst, false, out, out_final, n);
    }
    if (P <= MAXP) {
      PwayArgs a{};
      for (int p = 0; p < P; p++) a.in[p] = in[l + p];
      a.out[0] = out;
      a.n = n;
      a.root = root - l;  // the tree over [l, r] is the tree over [0, r-l] shifted
      return launch(K_MST, P, a, leaf_mask(P), out_final && rbe());
    }
    const int mid = (l + r) / 2;
    int al, ar, aroot, rl, rr, rroot;
    if (root <= mid) { al = l; ar = mid; aroot = root; rl = mid + 1; rr = r; rroot = r; }
    else { al = mid + 1; ar = r; aroot = root; rl = l; rr = mid; rroot = l; }
    void* ta = tmp->push(n);
    void* tb = tmp->push(n);
    if (!ta || !tb) return fail(MPJX_ERR_INTERNAL, "scratch temporaries exhausted (P=%d)", P);
    CHK(mst_o(in, al, ar, aroot, ta, false, n));
    CHK(mst_o(in, rl, rr, rroot, tb, false, n));
    // acc = own half, then fold the received half: both native temporaries
    PwayArgs a{};
    a.in[0] = ta;
    a.in[1] = tb;
    a.out[0] = out;
    a.n = n;
    CHK(launch(K_FOLD, 2, a, 0, out_final && rbe()));
    tmp->top -= 2 * (((size_t)n * esz + 255) & ~(size_t)255);
    return MPJX_SUCCESS;
  }
  int mst(const void* const* in, int l, int r, int root, void* out, int64_t n) {
    return mst_o(in, l, r, root, out, true, n);
  }

  // out[r] = in[r-1] (op) (... (in[0] (op) in[r]))
  int scan(int P, const void* const* in, void* const* out, int64_t n) {
    if (n <= 0) return MPJX_SUCCESS;
    if (P == 1) return copy(out[0], in[0], n);
    if (P <= MAXP) {
      PwayArgs a{};
      for (int p = 0; p < P; p++) { a.in[p] = in[p]; a.out[p] = out[p]; }
      a.n = n;
      return launch(K_SCAN, P, a, leaf_mask(P), rbe());
    }
    std::vector<const void*> lst;
    for (int r = P - 1; r >= 0; r--) {  // descending: out[r] may alias in[r], which only ranks > r read
      lst.clear();
      lst.push_back(in[r]);
      for (int i = 0; i < r; i++) lst.push_back(in[i]);
      CHK(fold((int)lst.size(), lst.data(), out[r], n));
    }
    return MPJX_SUCCESS;
  }

  // Same results as mst()/fold(), stored to every outs[q] (q < nout): the multicore all-gather fused
  // into the combine. P <= MAXP and nout <= MAXP in one launch; otherwise compute then copy.
  int mst_rep(const void* const* in, int P, int root, void* const* outs, int nout, int64_t n) {
    if (n <= 0) return MPJX_SUCCESS;
    if (P == 2) {  // MST over two ranks: acc = in[root], then the other
      const void* lst[2] = {in[root], in[1 - root]};
      return fold_rep(2, lst, outs, nout, n);
    }
    if (P >= 3 && P <= MAXP && nout <= MAXP) {
      PwayArgs a{};
      for (int p = 0; p < P; p++) a.in[p] = in[p];
      for (int q = 0; q < nout; q++) a.out[q] = outs[q];
      a.n = n;
      a.root = root;
      a.nrep = nout;
      return launch(K_MST, P, a, leaf_mask(P), rbe());
    }
    CHK(mst(in, 0, P - 1, root, outs[0], n));
    for (int q = 1; q < nout; q++) CHK(copy_raw(outs[q], outs[0], n));
    return MPJX_SUCCESS;
  }
  int fold_rep(int P, const void* const* in, void* const* outs, int nout, int64_t n) {
    if (n <= 0) return MPJX_SUCCESS;
    if (P >= 2 && P <= MAXP && nout <= MAXP) {
      PwayArgs a{};
      for (int p = 0; p < P; p++) a.in[p] = in[p];
      for (int q = 0; q < nout; q++) a.out[q] = outs[q];
      a.n = n;
      a.nrep = nout;
      return launch(K_FOLD, P, a, leaf_mask(P), rbe());
    }
    CHK(fold(P, in, outs[0], n));
    for (int q = 1; q < nout; q++) CHK(copy_raw(outs[q], outs[0], n));
    return MPJX_SUCCESS;
  }

  // buf[i] = F(0, buf[i]), `times` times over, buf in the SEND byte order: BKT_Reduce_scatter's arr
  // folding its zero tmpbuf outside the rank's own block in every round and storing arr back into the
  // caller's sendbuf (PureIntracomm.java:2409,2427-2428). zeros: n zeroed elements (any byte order).
  int zero_fold(void* buf, const void* zeros, int times, int64_t n) {
    for (int t = 0; t < times && n > 0; t++) {
      PwayArgs a{};
      a.in[0] = buf;
      a.in[1] = zeros;
      a.out[0] = buf;
      a.n = n;
      CHK(launch(K_FOLD, 2, a, sbe() ? 1u : 0u, sbe()));
    }
    return MPJX_SUCCESS;
  }

  int bkt(const void* own, const void* succ, int rounds, void* out, int64_t n) {
    if (n <= 0) return MPJX_SUCCESS;
    PwayArgs a{};
    a.in[0] = own;
    a.in[1] = succ;
    a.out[0] = out;
    a.n = n;
    a.root = rounds;
    return launch(K_BKT, 2, a, leaf_mask(2), rbe());
  }
};

}  // namespace mpjx
