// mpjx_kernels.hpp — the P-way element-wise combine kernels for gfx950 (CDNA4).
//
// One streaming kernel template covers every reduction step of the path: it reads P operand
// slices (the local send block plus the P-1 blocks received over xGMI), evaluates the reference's
// combine ORDER per element in registers, and writes Q result slices:
//   K_FOLD  out = v[P-1] (op) (... (op) (v[1] (op) v[0]))  — one typed perform per input in list
//           order. P=2 is Op.perform itself (inout = in (op) inout); with the pointer list permuted
//           on the host it is FT_Reduce / FT_Allreduce (src/mpi/PureIntracomm.java:2033-2056,
//           2267-2311) and the P<=2 bucket Reduce_scatter (:2404-2428).
//   K_MST   out = the MST_Reduce tree rooted at `root` (PureIntracomm.java:1943-1992): at every
//           merge the root folds the partial it receives into its own (acc = recv (op) acc).
//   K_SCAN  Q = P outputs, out[r] = v[r-1] (op) (... (op) (v[0] (op) v[r])) (Scan, :2526-2544).
//   K_BKT   FAITHFUL P>=3 bucket Reduce_scatter (:2377-2439, defect A9): v[0] = own block,
//           v[1] = the successor's copy of it, `root` = rounds.
// Big-endian operands (mpjbuf payloads, src/mpjbuf/NIOBuffer.java:42) are byte-swapped in registers
// between the 16-B load and the combine, and results between the combine and the store
// (PwayArgs::swap_in per operand, swap_out for every output): one HBM pass instead of a swap pass
// before and after. Calls with swaps launch a kernel of their own (SW = true), so the native kernel's
// register allocation does not cover the swap body.
// No MFMA: the op is pointwise; the kernel is an HBM stream. Each lane moves 16 B per operand per
// step (global_load_dwordx4), U steps in flight, grid-strided so every wave-instruction touches one
// contiguous 1 KiB; the sub-16-B tail is finished by block 0. Misaligned pointer sets run the W=1
// (one element per lane) instantiation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "mpjx_ops.hpp"

namespace mpjx {

enum Kind { K_FOLD = 0, K_MST = 1, K_SCAN = 2, K_BKT = 3 };
constexpr int MAXP = 8;

// The IPC engine's device-synchronised fence signal, stored from the combine kernel's tail (small calls):
// where this rank's phase-B sequence flag goes in every peer's staging region, and the last-block
// counter. Device-resident (mpjx_ipc.hip, filled once at init).
struct TailSignal {
  unsigned long long* peer[64];
  int P, me;
  unsigned* counter;  // zero between calls: the last block resets it
};

struct PwayArgs {
  const void* in[MAXP];
  void* out[MAXP];
  int64_t n;     // elements per slice
  int root;      // K_MST root, K_BKT rounds
  int nrep = 1;  // K_FOLD/K_MST/K_BKT: the result is stored to out[0..nrep) (multicore all-gather fused in)
  unsigned swap_in = 0;  // bit p: in[p] holds big-endian words (byte-swapped after the load)
  unsigned swap_out = 0; // nonzero: every output is stored big-endian
  const TailSignal* tail = nullptr;  // non-null: the last block to finish stores tail_seq into the peers' flags
  unsigned long long tail_seq = 0;
};

// ---- per-element order evaluators ------------------------------------------------------------

template <class F, int L, int R, class T, int P>
__device__ __forceinline__ T mst_eval(const T (&v)[P], int root) {
  if constexpr (L == R) {
    return v[L];
  } else {
    constexpr int M = (L + R) / 2;  // MST_Reduce: mid = (left + right) / 2
    if (root <= M) {                // srce = right: the right half reduces onto R
      T acc = mst_eval<F, L, M>(v, root);
      T rcv = mst_eval<F, M + 1, R>(v, R);
      return F::apply(rcv, acc);
    } else {                        // srce = left: the left half reduces onto L
      T acc = mst_eval<F, M + 1, R>(v, root);
      T rcv = mst_eval<F, L, M>(v, L);
      return F::apply(rcv, acc);
    }
  }
}

// The same tree with the root known at compile time. The MAXLOC/MINLOC pairs take it behind a uniform
// branch on the root (mst_switch): with mst_eval's runtime `root <= M` tests the compiler selected
// between whole subtrees of 2-word structs, and K_MST P=8 on 32 MiB slices ran at 0.50-0.60 of the
// spec cold (FLOAT2 63.6 us, INT2 54.0, DOUBLE2 65.8) against 0.80 with one tree per root value
// (46.5-47.4 us; profiles/r02/cold/loc_pairs_mst_cold.jsonl).
template <class F, int L, int R, int ROOT, class T, int P>
__device__ __forceinline__ T mst_ct(const T (&v)[P]) {
  if constexpr (L == R) {
    return v[L];
  } else {
    constexpr int M = (L + R) / 2;
    if constexpr (ROOT <= M) {
      T acc = mst_ct<F, L, M, ROOT>(v);
      T rcv = mst_ct<F, M + 1, R, R>(v);
      return F::apply(rcv, acc);
    } else {
      T acc = mst_ct<F, M + 1, R, ROOT>(v);
      T rcv = mst_ct<F, L, M, L>(v);
      return F::apply(rcv, acc);
    }
  }
}

template <class T>
struct IsPair : std::false_type {};

// Runtime root, one compile-time tree per root value behind a uniform branch.
template <class F, int P, class T, int... Rs>
__device__ __forceinline__ T mst_switch(const T (&v)[P], int root, std::integer_sequence<int, Rs...>) {
  T out = v[0];
  (void)((root == Rs ? (out = mst_ct<F, 0, P - 1, Rs>(v), true) : false) || ...);
  return out;
}

template <int KIND, int P>
struct NumOut {
  static constexpr int value = (KIND == K_SCAN) ? P : 1;
};

template <class F, int P, int KIND, class T, int Q>
__device__ __forceinline__ void eval_elem(const T (&v)[P], T (&o)[Q], int root) {
  if constexpr (KIND == K_FOLD) {
    T acc = v[0];
#pragma unroll
    for (int k = 1; k < P; k++) acc = F::apply(v[k], acc);
    o[0] = acc;
  } else if constexpr (KIND == K_MST) {
    if constexpr (IsPair<T>::value) o[0] = mst_switch<F, P>(v, root, std::make_integer_sequence<int, P>{});
    else o[0] = mst_eval<F, 0, P - 1>(v, root);
  } else if constexpr (KIND == K_SCAN) {
#pragma unroll
    for (int r = 0; r < P; r++) {
      T acc = v[r];
#pragma unroll
      for (int i = 0; i < r; i++) acc = F::apply(v[i], acc);
      o[r] = acc;
    }
  } else {  // K_BKT
    T a = v[0], b = v[1];
    for (int k = 0; k < root; k++) {
      T t = b;
      b = F::apply(T(0), b);  // successor folds its zero tmpbuf block into its copy
      a = F::apply(t, a);
    }
    o[0] = a;
  }
}

// ---- the streaming kernel ------------------------------------------------------------------------

using v4u = unsigned int __attribute__((ext_vector_type(4)));

template <class T, int W>
struct Pack {  // W elements moved by one load/store
  using type = typename std::conditional<W == 1, T, v4u>::type;
};

template <bool NT, class L>
__device__ __forceinline__ L ld(const L* p) {
  if constexpr (NT && (std::is_arithmetic<L>::value || std::is_same<L, v4u>::value)) {
    return __builtin_nontemporal_load(p);
  } else if constexpr (NT && sizeof(L) == 16) {  // 16-B structs (DOUBLE2/LONG2 pairs)
    v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    L r;
    __builtin_memcpy(&r, &v, 16);
    return r;
  } else {
    return *p;
  }
}
template <bool NT, class L>
__device__ __forceinline__ void st(L* p, L v) {
  if constexpr (NT && (std::is_arithmetic<L>::value || std::is_same<L, v4u>::value)) {
    __builtin_nontemporal_store(v, p);
  } else if constexpr (NT && sizeof(L) == 16) {
    v4u w;
    __builtin_memcpy(&w, &v, 16);
    __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(p));
  } else {
    *p = v;
  }
}

// Byte-order words of an element type: the type itself, or the value type of a MAXLOC/MINLOC pair.
template <class T>
struct WordOf {
  static constexpr int value = sizeof(T);
};
template <class V>
struct WordOf<Pair<V>> {
  static constexpr int value = sizeof(V);
};
template <class V>
struct IsPair<Pair<V>> : std::true_type {};

// Reverse the bytes of every WS-byte word of v (a 16-B vector, or one element).
template <int WS, class L>
__device__ __forceinline__ L swap_words(L v) {
  if constexpr (WS == 1 || sizeof(L) == 1) {
    return v;
  } else if constexpr (sizeof(L) == 2) {
    uint16_t h;
    __builtin_memcpy(&h, &v, 2);
    h = __builtin_bswap16(h);
    __builtin_memcpy(&v, &h, 2);
    return v;
  } else {
    constexpr int ND = sizeof(L) / 4;
    uint32_t d[ND];
    __builtin_memcpy(d, &v, sizeof(L));
    if constexpr (WS == 8) {  // swap each 32-bit half and exchange the halves
#pragma unroll
      for (int k = 0; k < ND; k += 2) {
        const uint32_t lo = d[k], hi = d[k + 1];
        d[k] = __builtin_bswap32(hi);
        d[k + 1] = __builtin_bswap32(lo);
      }
    } else if constexpr (WS == 4) {
#pragma unroll
      for (int k = 0; k < ND; k++) d[k] = __builtin_bswap32(d[k]);
    } else {  // 2
#pragma unroll
      for (int k = 0; k < ND; k++) d[k] = ((d[k] & 0x00ff00ffu) << 8) | ((d[k] >> 8) & 0x00ff00ffu);
    }
    __builtin_memcpy(&v, d, sizeof(L));
    return v;
  }
}

constexpr int kThreads = 256;  // small (cache-resident) launches and the scalar instantiation

// One tile = TH * U consecutive loads per operand; lane t handles base + u*TH + t, so every
// wave-instruction covers one contiguous 1 KiB. FULL tiles skip the bounds checks.
// Cache policy of one launch (POL): 0 = default loads and stores (launches that stream < 64 MiB:
// their operands were just written and sit in the caches); 1 = non-temporal loads and stores;
// 4 = operand 0 with the default policy, every other operand and the stores non-temporal.
// Chosen on COLD operands — every launch on buffers no earlier launch left in the 256 MiB Infinity
// Cache, as a reduction over freshly received message data runs (tools/tune_cold.hip,
// profiles/r02/cold/tune_cold_sweep{1,2}.txt): 2 x 256 MiB in-place fold, all non-temporal 122.6 us at
// 1024 x 1 per block; operand 0 plain (4) 49.5 vs 52.5-54 us for 8 x 32 MiB slices. (Round 2's mixed
// policies — the accumulator non-temporal, the other operand default, 109-111 us — were tuned with
// the same buffers every launch, where the default-policy operand is partly served from the
// Infinity Cache left by the previous launch; on cold operands they ran 124-131 us.)
// 5 = loads as 4, stores with the default policy; 6 = every load non-temporal, default stores (the
// short-launch forms: stores left to the caches are written back after the kernel, tools/tuning/tune_short.hip).
template <int POL>
__host__ __device__ constexpr bool nt_load(int p) { return POL == 1 || POL == 6 || ((POL == 4 || POL == 5) && p != 0); }
template <int POL>
__host__ __device__ constexpr bool nt_store() { return POL == 1 || POL == 4; }

// x[p] = operand p's vector i, each with its policy chosen at compile time. (A runtime ternary
// between a non-temporal and a plain load of the same address is merged by the optimiser into one
// PLAIN load — the non-temporal hint is dropped — so the choice must never reach the IR.)
// Load issue groups (G < P, streaming form only): after every G-th operand's load the lane drains its
// loads (s_waitcnt vmcnt(0)) before the next group issues; scheduler barriers keep the compiler from
// moving loads across the boundary. G = P issues all P loads before the first wait.
template <int G, int I, int P>
__device__ __forceinline__ void group_boundary() {
  if constexpr (G < P && (I + 1) % G == 0 && I + 1 < P) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt((7u << 4) | (15u << 8));  // vmcnt(0), expcnt/lgkmcnt at their maxima
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int POL, int G, class L, int P, int... Is>
__device__ __forceinline__ void load_operands(L (&x)[P], const PwayArgs& a, int64_t i,
                                              std::integer_sequence<int, Is...>) {
  ((x[Is] = ld<nt_load<POL>(Is)>(reinterpret_cast<const L*>(a.in[Is]) + i), group_boundary<G, Is, P>()), ...);
}

// Chosen per shape on cold operands in the engines' slot layout, the library body at every G beside
// each other in one process (tools/tuning/tune_stagger.hip, profiles/r03/tuning/tune_stagger_*.jsonl):
// K_MST P=4 on 64 MiB slices 55.1-55.6 us at G=4 -> 53.2-53.9 at G=1; K_SCAN P=4 on 64 MiB 83.3-85.4
// -> 82.3-82.4 at G=2. K_MST / K_SCAN P=8 and the 2-operand fold keep G=P (every G<P as fast or slower;
// the first variant timed after the K_SCAN P=8 shape pays ~2 us for that shape's write-back, which a
// first look had mistaken for a G=4 gain at K_MST P=8).
template <int P, int KIND, int POL>
struct LoadGroup {
  static constexpr int value = POL == 0 ? P
                             : (KIND == K_MST && P == 4) ? 1
                             : (KIND == K_SCAN && P == 4) ? 2
                             : P;
};

template <class F, int P, int KIND, int W, int TH, int U, int POL, bool FULL, bool SW, int G>
__device__ __forceinline__ void pway_tile(const PwayArgs& a, int64_t base, int64_t nv) {
  constexpr bool NT = nt_store<POL>();  // stores
  using T = typename F::T;
  using L = typename Pack<T, W>::type;
  constexpr int Q = NumOut<KIND, P>::value;
  constexpr int WS = WordOf<T>::value;
  L x[U][P];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int64_t i = base + u * TH + threadIdx.x;
    if (FULL || i < nv) {
      load_operands<POL, (U == 1 ? G : P)>(x[u], a, i, std::make_integer_sequence<int, P>{});
    }
  }
  if constexpr (SW) {
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int p = 0; p < P; p++)
        if (a.swap_in & (1u << p)) x[u][p] = swap_words<WS>(x[u][p]);
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int64_t i = base + u * TH + threadIdx.x;
    if constexpr (KIND == K_SCAN) {
      // Output q is computed and stored as soon as operands 0..q are in (q outer): the compiler then
      // interleaves the P stores with the load waits instead of issuing all of them after the last
      // load (K_SCAN P=8 on 8 x 32 MiB slices ran 89.9 us with the stores bunched at the end against
      // 84.8 us for a kernel storing each output early, tools/tuning/tune_stagger.hip).
      if (FULL || i < nv) {
        T e[P][W];
#pragma unroll
        for (int p = 0; p < P; p++) __builtin_memcpy(e[p], &x[u][p], sizeof(L));
#pragma unroll
        for (int q = 0; q < Q; q++) {
          T rq[W];
#pragma unroll
          for (int w = 0; w < W; w++) {  // out[q] = v[q-1] (op) (... (op) (v[0] (op) v[q])), as eval_elem
            T acc = e[q][w];
#pragma unroll
            for (int k = 0; k < q; k++) acc = F::apply(e[k][w], acc);
            rq[w] = acc;
          }
          L y;
          __builtin_memcpy(&y, rq, sizeof(L));
          if constexpr (SW) {
            if (a.swap_out) y = swap_words<WS>(y);
          }
          st<NT>(reinterpret_cast<L*>(a.out[q]) + i, y);
        }
      }
    } else if (FULL || i < nv) {
      T e[P][W], r[Q][W];
#pragma unroll
      for (int p = 0; p < P; p++) __builtin_memcpy(e[p], &x[u][p], sizeof(L));
#pragma unroll
      for (int w = 0; w < W; w++) {
        T col[P], out[Q];
#pragma unroll
        for (int p = 0; p < P; p++) col[p] = e[p][w];
        eval_elem<F, P, KIND>(col, out, a.root);
#pragma unroll
        for (int q = 0; q < Q; q++) r[q][w] = out[q];
      }
      L y;
      __builtin_memcpy(&y, r[0], sizeof(L));
      if constexpr (SW) {
        if (a.swap_out) y = swap_words<WS>(y);
      }
      for (int q = 0; q < a.nrep; q++) st<NT>(reinterpret_cast<L*>(a.out[q]) + i, y);
    }
  }
}

template <class F, int P, int KIND, int W, int TH, int U, int POL, bool SW, int G>
__device__ __forceinline__ void pway_body(const PwayArgs& a) {
  using T = typename F::T;
  constexpr int Q = NumOut<KIND, P>::value;
  constexpr int WS = WordOf<T>::value;
  const int64_t nv = a.n / W;
  const int64_t tile = (int64_t)TH * U;
  for (int64_t base = (int64_t)blockIdx.x * tile; base < nv; base += (int64_t)gridDim.x * tile) {
    if (base + tile <= nv) pway_tile<F, P, KIND, W, TH, U, POL, true, SW, G>(a, base, nv);
    else pway_tile<F, P, KIND, W, TH, U, POL, false, SW, G>(a, base, nv);
  }
  if constexpr (W > 1) {  // sub-vector tail (< W elements), block 0
    if (blockIdx.x == 0) {
      for (int64_t e = nv * W + threadIdx.x; e < a.n; e += blockDim.x) {
        T col[P], out[Q];
#pragma unroll
        for (int p = 0; p < P; p++) {
          col[p] = reinterpret_cast<const T*>(a.in[p])[e];
          if constexpr (SW) {
            if (a.swap_in & (1u << p)) col[p] = swap_words<WS>(col[p]);
          }
        }
        eval_elem<F, P, KIND>(col, out, a.root);
        if constexpr (SW) {
          if (a.swap_out)
#pragma unroll
            for (int q = 0; q < Q; q++) out[q] = swap_words<WS>(out[q]);
        }
        if constexpr (KIND == K_SCAN) {
#pragma unroll
          for (int q = 0; q < Q; q++) reinterpret_cast<T*>(a.out[q])[e] = out[q];
        } else {
          for (int q = 0; q < a.nrep; q++) reinterpret_cast<T*>(a.out[q])[e] = out[0];
        }
      }
    }
  }
}

// Big-endian operands or results (SW) run a kernel of their own: with both bodies behind a uniform
// branch in one kernel, the register allocation covered the swap body too, and the native K_SCAN P=8
// streaming kernel held 75 VGPRs — 6 waves per SIMD, one 1024-lane block per CU (88.7 us on 8 x 32 MiB
// slices, against 85.4 us for the same body at 42 VGPRs, tools/tuning/tune_stagger.hip).
// The device-sync tail (PwayArgs::tail): every block makes its result stores (local and into the peers'
// staging regions) visible system-wide and counts itself in; the block that counts last stores the call's
// sequence number into every peer's phase-B flag slot (a system-scope release), so the peers' fence waits
// end as soon as this kernel does, not one launch later (mpjx_ipc.hip fence()).
// Every wave fences its OWN stores to system scope before the workgroup barrier (a workgroup barrier
// alone does not wait for another wave's stores into a peer's staging to complete, so thread 0's fence
// could not cover them); the last block fences again after it has seen the counter, before its release
// stores to the peers' flags, as k_copies_flags does.
__device__ __forceinline__ void pway_tail(const TailSignal* t, unsigned long long seq) {
  __shared__ int last;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(t->counter, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) {
    __hip_atomic_store(t->counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next call
    __threadfence_system();
  }
  __syncthreads();
  const int j = threadIdx.x;
  if (j < t->P && j != t->me) __hip_atomic_store(t->peer[j], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <class F, int P, int KIND, int W, int TH, int U, int POL, int G = LoadGroup<P, KIND, POL>::value,
          bool SW = false>
__global__ __launch_bounds__(TH) void k_pway(PwayArgs a) {
  using T = typename F::T;
  static_assert(W == 1 || W * sizeof(T) == 16, "vector width is 16 bytes");
  static_assert(!SW || WordOf<T>::value > 1, "byte-wide types have no byte order");
  pway_body<F, P, KIND, W, TH, U, POL, SW, G>(a);
  if (a.tail) pway_tail(a.tail, a.tail_seq);  // uniform: one branch after the streaming loop
}

// ---- launch -----------------------------------------------------------------------------------------

// Launches that stream >= kStreamBytes of operands + results (MPJX_NT_MIN_MIB overrides it for
// tuning runs) take the streaming form: 1024-lane blocks, one 16-B vector per operand per lane
// (16 KiB per operand per block), non-temporal (POL 1 at P <= 2, POL 4 above). Cold sweeps
// (profiles/r02/cold/tune_cold_sweep2.txt, medians of 9 interleaved rounds): 2 x 256 MiB in place,
// all non-temporal, 122.6 us at 1024 x 1 against 124.8 (512 x 1), 125.5 (256 x 1), 126.6 (256 x 4,
// round 1's tile), 129.0 (1024 x 2); 8 x 32 MiB slices under POL 4 49.5 us at 1024 x 1 and 49.9 at
// 512 x 1 against 51.7 at 256 x 1. Smaller launches keep 256-lane blocks, the default policy and
// the round-1 unroll (their operands are cache-resident: just exchanged or just computed).
constexpr int64_t kMaxBlocks = (int64_t)1 << 30;
constexpr size_t kStreamBytes = (size_t)64 << 20;
constexpr int kStreamThreads = 1024;
// Streaming launches below kShortBytes (operands + results) are SHORT: 12-30 us at the configs[3] shapes,
// where a one-tile-per-block grid pays a whole load latency in its drain (DESIGN.md §4 "Short launches").
constexpr size_t kShortBytes = (size_t)256 << 20;

size_t nt_min_bytes();     // kStreamBytes unless MPJX_NT_MIN_MIB is set (read once)
size_t short_max_bytes();  // kShortBytes unless MPJX_SHORT_MAX_MIB is set (read once; 0 = no short form)
int cu_count();            // compute units of the current device (cached per device)

// Loads in flight per lane for the cache-resident (POL 0) form: 8 operands at P = 2, the VGPR budget
// at larger P (round 1's tune_combine sweep).
template <int P>
struct Unroll {
  static constexpr int value = P <= 2 ? 4 : (P <= 4 ? 2 : 1);
};

// Operand streams whose addresses are equal modulo 16 MiB (P slots at a power-of-two stride in one
// allocation: the RCCL exchange engine's contiguous input slots for one ncclAllToAll) meet in the same
// HBM channels; staggering the loads in pairs recovers most of it. K_MST P=8 on 32 MiB slices, cold
// (tools/tuning/tune_stagger.hip with skew 0, profiles/r03/tuning/tune_stagger_skew0.jsonl): contiguous
// 50.3 us at G = 8 -> 47.7 us at G = 2 (0.75 -> 0.79); with the 4 KiB slot skew G = 8 stays best
// (45.9-46.3 vs 46.9-47.2 us), so the group is chosen per launch from the pointers. K_SCAN P=8 with
// contiguous inputs and skewed outputs (the engine's Scan layout): 90.1-91.0 us at G = 8, 89.2 at G = 4
// (tune_stagger_in0_out4k.jsonl).
template <int P, int KIND>
struct CollideGroup {
  static constexpr int value = (KIND == K_MST && P == 8) ? 2
                             : (KIND == K_SCAN && P == 8) ? 4
                             : LoadGroup<P, KIND, 4>::value;
};

template <int P>
inline bool streams_collide(const PwayArgs& a, uintptr_t mod = (uintptr_t)16 << 20) {
  const uintptr_t b = (uintptr_t)a.in[0] % mod;
  for (int p = 1; p < P; p++)
    if ((uintptr_t)a.in[p] % mod != b) return false;
  return true;
}

// Load groups of the short form's persistent grid (tools/tuning/tune_short.hip sweep c,
// profiles/r04/tuning/tune_short_c*.jsonl): K_MST issues at most 4 loads before it drains (the
// streaming form's G = 1 at P = 4 costs 7 % here: 15.1 vs 14.1 us on 16 MiB int32 slices); at P >= 5 with
// the input slots equal modulo 4 MiB (the RCCL engine's contiguous slots at the BASELINE shapes) pairs:
// int32 P = 8 on 8 MiB slices 13.33 (G = 4) -> 13.07 us (G = 2), while with 4 KiB-skewed slots G = 4 ties
// or wins (byte / f64 8 MiB: 13.68 / 13.02 vs 14.31 / 13.63 us at G = 2).
template <int P, int KIND, int POL>
struct ShortGroup {
  static constexpr int value = KIND == K_MST ? (P < 4 ? P : 4) : LoadGroup<P, KIND, POL>::value;
  static constexpr int collide = (KIND == K_MST && P >= 5) ? 2 : value;
};

template <class F, int P, int KIND, int W, int TH, int U, int POL, int G = LoadGroup<P, KIND, POL>::value>
inline hipError_t launch_one(const PwayArgs& a, hipStream_t s, int64_t max_blocks = kMaxBlocks) {
  const int64_t nv = a.n / W;
  int64_t blocks = (nv + (int64_t)TH * U - 1) / ((int64_t)TH * U);
  if (blocks < 1) blocks = 1;
  if (blocks > max_blocks) blocks = max_blocks;  // a persistent grid: the body grid-strides over the tiles
  if constexpr (WordOf<typename F::T>::value > 1) {
    if (a.swap_in | a.swap_out) {
      hipLaunchKernelGGL((k_pway<F, P, KIND, W, TH, U, POL, G, true>), dim3((unsigned)blocks), dim3(TH), 0, s, a);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((k_pway<F, P, KIND, W, TH, U, POL, G, false>), dim3((unsigned)blocks), dim3(TH), 0, s, a);
  return hipGetLastError();
}

template <class F, int P, int KIND>
inline hipError_t launch_pw(const PwayArgs& a, hipStream_t s, bool vec) {
  using T = typename F::T;
  constexpr int VW = 16 / sizeof(T);
  if (!vec) return launch_one<F, P, KIND, 1, kThreads, Unroll<P>::value, 0>(a, s);
  const int Q = (KIND == K_SCAN) ? P : a.nrep;
  const size_t streamed = (size_t)a.n * sizeof(T) * (P + Q);
  if (streamed < nt_min_bytes()) return launch_one<F, P, KIND, VW, kThreads, Unroll<P>::value, 0>(a, s);
  // 1024 lanes leave 128 VGPRs per lane: enough for P x 16 B of operands unpacked into up to 32
  // elements; narrower types at large P (more elements per vector) take 512 lanes instead of spilling
  constexpr int TH = P * VW <= 32 ? kStreamThreads : kStreamThreads / 2;
  constexpr int POL = P <= 2 ? 1 : 4;
  if (streamed < short_max_bytes()) {
    // Short launches (tools/tuning/tune_short.hip, profiles/r04/tuning/tune_short_{a,b,c}.jsonl, cold, the
    // RCCL engine's layout). K_SCAN, whose P outputs double the bytes: deep 256-lane tiles, U vectors per
    // operand per lane in flight — int32 P=8 on 8 MiB slices 25.3 -> 22.4 us, P=4 on 16 MiB 22.8 -> 21.9.
    // The one-output kinds: the streaming tile on a persistent grid of one block per CU (grid-strided) with
    // the short form's load groups — fold P=2 on 32 MiB slices 18.3 -> 17.3 us, K_MST P=4 on 16 MiB
    // 14.3 -> 14.1, P=8 on 8 MiB 13.5 -> 13.1 (sweeps b, c).
    if constexpr (KIND == K_SCAN) {
      // 8-deep tiles stay in registers (<= 256 VGPRs + AGPRs) for 32/64-bit elements; byte types (16 elements
      // per vector) and the SHORT2 pairs spill at P >= 4 (168-2592 B/lane), 16-bit types at P >= 7: shallower
      constexpr int U = P < 4 ? 4 : (VW >= 16 || IsPair<T>::value) ? 2 : (VW >= 8 && P >= 7) ? 4 : 8;
      return launch_one<F, P, KIND, VW, 256, U, POL, P>(a, s);
    } else {
      const int64_t grid = (int64_t)cu_count() * (TH == kStreamThreads ? 1 : 2);
      using SG = ShortGroup<P, KIND, POL>;
      if constexpr (SG::collide != SG::value) {
        if (streams_collide<P>(a, (uintptr_t)4 << 20)) return launch_one<F, P, KIND, VW, TH, 1, POL, SG::collide>(a, s, grid);
      }
      return launch_one<F, P, KIND, VW, TH, 1, POL, SG::value>(a, s, grid);
    }
  }
  if constexpr (CollideGroup<P, KIND>::value != LoadGroup<P, KIND, POL>::value) {
    if (streams_collide<P>(a)) return launch_one<F, P, KIND, VW, TH, 1, POL, CollideGroup<P, KIND>::value>(a, s);
  }
  return launch_one<F, P, KIND, VW, TH, 1, POL>(a, s);
}

// All kinds and P for one functor. Returns hipErrorInvalidValue for an unsupported (kind, P).
template <class F>
inline hipError_t launch_functor(int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (kind) {
    case K_FOLD:
      switch (P) {
        case 2: return launch_pw<F, 2, K_FOLD>(a, s, vec);
        case 3: return launch_pw<F, 3, K_FOLD>(a, s, vec);
        case 4: return launch_pw<F, 4, K_FOLD>(a, s, vec);
        case 5: return launch_pw<F, 5, K_FOLD>(a, s, vec);
        case 6: return launch_pw<F, 6, K_FOLD>(a, s, vec);
        case 7: return launch_pw<F, 7, K_FOLD>(a, s, vec);
        case 8: return launch_pw<F, 8, K_FOLD>(a, s, vec);
      }
      break;
    case K_MST:
      switch (P) {
        case 3: return launch_pw<F, 3, K_MST>(a, s, vec);
        case 4: return launch_pw<F, 4, K_MST>(a, s, vec);
        case 5: return launch_pw<F, 5, K_MST>(a, s, vec);
        case 6: return launch_pw<F, 6, K_MST>(a, s, vec);
        case 7: return launch_pw<F, 7, K_MST>(a, s, vec);
        case 8: return launch_pw<F, 8, K_MST>(a, s, vec);
      }
      break;
    case K_SCAN:
      switch (P) {
        case 2: return launch_pw<F, 2, K_SCAN>(a, s, vec);
        case 3: return launch_pw<F, 3, K_SCAN>(a, s, vec);
        case 4: return launch_pw<F, 4, K_SCAN>(a, s, vec);
        case 5: return launch_pw<F, 5, K_SCAN>(a, s, vec);
        case 6: return launch_pw<F, 6, K_SCAN>(a, s, vec);
        case 7: return launch_pw<F, 7, K_SCAN>(a, s, vec);
        case 8: return launch_pw<F, 8, K_SCAN>(a, s, vec);
      }
      break;
    case K_BKT:
      if constexpr (std::is_arithmetic<typename F::T>::value)
        if (P == 2) return launch_pw<F, 2, K_BKT>(a, s, vec);
      break;
  }
  return hipErrorInvalidValue;
}

// Implemented per op family in mpjx_k_<family>.hip (split for parallel compilation).
// `faithful` selects the Keep functor for BOR/BXOR (defect A3).
hipError_t launch_sum(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec);
hipError_t launch_prod(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec);
hipError_t launch_max(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec);
hipError_t launch_min(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec);
hipError_t launch_bitwise(int op, int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec);
hipError_t launch_band(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec);
hipError_t launch_bor(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec);
hipError_t launch_bxor(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec);
hipError_t launch_maxloc(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec);
hipError_t launch_minloc(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec);
hipError_t launch_logical(int op, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec);
hipError_t launch_keep(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec);
hipError_t launch_loc(int op, int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec);
hipError_t launch_bswap(void* dst, const void* src, int64_t nbytes, int word, hipStream_t s);
// acc = (payload of the mpjbuf image msg, big-endian, sections walked on the device) (op) acc
// (mpjx_k_mpjbuf.hip); a malformed image stores an error code into *status.
hipError_t launch_mpjbuf(int op, int type, bool faithful, void* acc, const void* msg, int64_t msg_bytes,
                         int64_t count, int* status, hipStream_t s);
// Up to kMax independent device copies in one launch (each may cross a different xGMI link).
struct CopyList {
  static constexpr int kMax = 64;
  const unsigned char* src[kMax];
  unsigned char* dst[kMax];
  int64_t bytes[kMax];
  int n = 0;
  void add(void* d, const void* s_, int64_t b) {
    src[n] = (const unsigned char*)s_;
    dst[n] = (unsigned char*)d;
    bytes[n] = b;
    n++;
  }
};
hipError_t launch_copies(const CopyList& l, hipStream_t s);

// IPC device sync (mpjx_ipc.hip): flag slots of the peers (peer[j] = peer j's slot for this rank),
// this rank's own slots, and the bounded wait's limits; counter = a zeroed device word for the
// last-block count of launch_copies_flags.
struct FlagTail {
  unsigned long long* peer[64];
  const unsigned long long* mine;
  int P, me;
  unsigned long long seq;
  long long ticks;
  int* err;
  const int* failed;
  unsigned* counter;
  int store = 1;  // 0: the combine kernel's tail already stored this rank's flag; only wait
};
// The copies of l, then (from the last block) the flag store + wait of the IPC device sync.
hipError_t launch_copies_flags(const CopyList& l, const FlagTail& f, hipStream_t s);
// The flag store + wait of the IPC device sync in every block, then the copies of l (small copies only).
hipError_t launch_flags_copies(const CopyList& l, const FlagTail& f, hipStream_t s);

}  // namespace mpjx
