// mpjx_k_util.hip — byte-order kernels: big-endian mpjbuf payloads (src/mpjbuf/NIOBuffer.java:42)
// <-> the device's little-endian words. One HBM read + write per swapped buffer; 16 B per lane.
// Plus k_copies: up to 64 independent copies in one launch (the IPC engine's block scatter to, and
// pulls from, every peer over its own xGMI link at once, instead of one serialized copy per peer).
#include "mpjx_kernels.hpp"

#include <algorithm>

namespace mpjx {

template <int WS>
__device__ __forceinline__ v4u bswap_vec(v4u v) {
  if constexpr (WS == 2) {
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = ((v[i] & 0x00ff00ffu) << 8) | ((v[i] >> 8) & 0x00ff00ffu);
  } else if constexpr (WS == 4) {
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = __builtin_bswap32(v[i]);
  } else {  // 8: swap each 32-bit half and exchange the halves
    v4u r;
    r[0] = __builtin_bswap32(v[1]);
    r[1] = __builtin_bswap32(v[0]);
    r[2] = __builtin_bswap32(v[3]);
    r[3] = __builtin_bswap32(v[2]);
    v = r;
  }
  return v;
}

template <int WS>
__global__ __launch_bounds__(256) void k_bswap(unsigned char* dst, const unsigned char* src, int64_t nbytes) {
  const int64_t nv = nbytes / 16;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride)
    reinterpret_cast<v4u*>(dst)[i] = bswap_vec<WS>(reinterpret_cast<const v4u*>(src)[i]);
  if (blockIdx.x == 0) {  // tail words
    for (int64_t w = nv * 16 / WS + threadIdx.x; w < nbytes / WS; w += blockDim.x) {
      unsigned char tmp[WS];
#pragma unroll
      for (int b = 0; b < WS; b++) tmp[b] = src[w * WS + WS - 1 - b];
#pragma unroll
      for (int b = 0; b < WS; b++) dst[w * WS + b] = tmp[b];
    }
  }
}

template <int WS>
__global__ __launch_bounds__(256) void k_bswap_unaligned(unsigned char* dst, const unsigned char* src, int64_t nwords) {
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += (int64_t)gridDim.x * blockDim.x) {
    unsigned char tmp[WS];
#pragma unroll
    for (int b = 0; b < WS; b++) tmp[b] = src[w * WS + WS - 1 - b];
#pragma unroll
    for (int b = 0; b < WS; b++) dst[w * WS + b] = tmp[b];
  }
}

// dst = byte-swapped words of src (word size 2, 4 or 8; 1 = plain copy); dst may equal src.
hipError_t launch_bswap(void* dst, const void* src, int64_t nbytes, int word, hipStream_t s) {
  if (nbytes <= 0) return hipSuccess;
  if (word == 1) return dst == src ? hipSuccess : hipMemcpyAsync(dst, src, (size_t)nbytes, hipMemcpyDeviceToDevice, s);
  const bool al = (((uintptr_t)dst | (uintptr_t)src) & 15u) == 0;
  int64_t blocks = (nbytes / 16 + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
  auto d = (unsigned char*)dst;
  auto q = (const unsigned char*)src;
  switch (word) {
    case 2:
      if (al) hipLaunchKernelGGL(k_bswap<2>, dim3(blocks), dim3(256), 0, s, d, q, nbytes);
      else hipLaunchKernelGGL(k_bswap_unaligned<2>, dim3(blocks), dim3(256), 0, s, d, q, nbytes / 2);
      break;
    case 4:
      if (al) hipLaunchKernelGGL(k_bswap<4>, dim3(blocks), dim3(256), 0, s, d, q, nbytes);
      else hipLaunchKernelGGL(k_bswap_unaligned<4>, dim3(blocks), dim3(256), 0, s, d, q, nbytes / 4);
      break;
    case 8:
      if (al) hipLaunchKernelGGL(k_bswap<8>, dim3(blocks), dim3(256), 0, s, d, q, nbytes);
      else hipLaunchKernelGGL(k_bswap_unaligned<8>, dim3(blocks), dim3(256), 0, s, d, q, nbytes / 8);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// blockIdx.y = copy; one tile (TH lanes x U x 16 B) per x block. NT = the streaming form for copies of
// >= 64 MiB in one launch: 512 lanes x one 16-B vector, non-temporal loads and stores — on cold
// buffers (tools/tune_cold.hip, profiles/r02/cold/tune_cold_sweep2.txt) 83.3 us per 256 MiB against 84.3
// (1024 x 1), 85.6 (512 x 2) and 91.1 for round 2's default-policy loads (tuned on one buffer reused
// every launch, where the source partly stayed in the Infinity Cache: 73-75 us warm).
template <bool NT>
struct CopyTile {
  static constexpr int TH = NT ? 512 : 256;
  static constexpr int U = NT ? 1 : 4;
  static constexpr int64_t bytes = TH * U * 16;
};
// Tile `x` of copy `c` (the launches below: c = blockIdx.y, x = blockIdx.x; k_flags_copies strides).
template <bool NT>
__device__ __forceinline__ void copy_tile(const CopyList& l, int c, int64_t x) {
  const unsigned char* src = l.src[c];
  unsigned char* dst = l.dst[c];
  const int64_t n = l.bytes[c];
  constexpr int TH = CopyTile<NT>::TH;
  constexpr int U = CopyTile<NT>::U;
  constexpr int64_t TB = CopyTile<NT>::bytes;
  const int64_t t = x * TB;
  if (t >= n) return;
  if (((((uintptr_t)src) | ((uintptr_t)dst)) & 15u) == 0) {
    const int64_t nv = n / 16, t4 = t / 16;
    const v4u* s4 = reinterpret_cast<const v4u*>(src);
    v4u* d4 = reinterpret_cast<v4u*>(dst);
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t i = t4 + u * TH + threadIdx.x;
      if (i < nv) {
        if constexpr (NT) v[u] = __builtin_nontemporal_load(s4 + i);
        else v[u] = s4[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t i = t4 + u * TH + threadIdx.x;
      if (i < nv) {
        if (NT) __builtin_nontemporal_store(v[u], d4 + i);
        else d4[i] = v[u];
      }
    }
    if (t + TB >= n)  // the block holding the end also copies the sub-16-B tail
      for (int64_t b = nv * 16 + threadIdx.x; b < n; b += TH) dst[b] = src[b];
  } else {
    const int64_t e = t + TB < n ? t + TB : n;
    for (int64_t b = t + threadIdx.x; b < e; b += TH) dst[b] = src[b];
  }
}

template <bool NT>
__global__ __launch_bounds__(CopyTile<NT>::TH) void k_copies(CopyList l) {
  copy_tile<NT>(l, blockIdx.y, blockIdx.x);
}

// The copies, then the IPC device-sync flags (mpjx_ipc.hip k_ipc_flags) from the last block to
// finish: every block makes its stores visible system-wide and counts itself in; the block that
// counts last stores seq into every peer's flag slot and waits for the peers' slots in its own area
// (bounded by the wall clock and the world's failed mark). One launch instead of two.
// Every wave fences its OWN stores to system scope before the block's barrier (a fence orders only the
// issuing wave's stores: one on thread 0 after __syncthreads would leave the other waves' stores into
// the peers' staging unordered with the count, hence with the flag the last block releases), as
// pway_tail does.
template <bool NT>
__global__ __launch_bounds__(CopyTile<NT>::TH) void k_copies_flags(CopyList l, FlagTail f) {
  copy_tile<NT>(l, blockIdx.y, blockIdx.x);
  __shared__ int last;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned total = gridDim.x * gridDim.y;
    last = atomicAdd(f.counter, 1u) == total - 1;
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) {
    __hip_atomic_store(f.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next call
    __threadfence_system();
  }
  __syncthreads();
  const int j = threadIdx.x;
  if (j >= f.P || j == f.me) return;
  __hip_atomic_store(f.peer[j], f.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  const long long t0 = wall_clock64();
  for (unsigned it = 1; __hip_atomic_load(f.mine + j, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < f.seq; it++) {
    const bool gone = (it & 63) == 0 && __hip_atomic_load(f.failed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (gone || wall_clock64() - t0 > f.ticks) {
      __hip_atomic_store(f.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

hipError_t launch_copies_flags(const CopyList& l, const FlagTail& f, hipStream_t s) {
  if (l.n <= 0 || l.n > CopyList::kMax) return hipErrorInvalidValue;
  int64_t mx = 0, total = 0;
  for (int i = 0; i < l.n; i++) {
    mx = l.bytes[i] > mx ? l.bytes[i] : mx;
    total += l.bytes[i];
  }
  const bool nt = total >= ((int64_t)64 << 20);
  const int64_t tb = nt ? CopyTile<true>::bytes : CopyTile<false>::bytes;
  const int64_t bx = mx > 0 ? (mx + tb - 1) / tb : 1;
  if (bx * l.n > 0x7fffffff) return hipErrorInvalidValue;
  if (nt)
    hipLaunchKernelGGL(k_copies_flags<true>, dim3((unsigned)bx, (unsigned)l.n), dim3(CopyTile<true>::TH), 0, s, l, f);
  else
    hipLaunchKernelGGL(k_copies_flags<false>, dim3((unsigned)bx, (unsigned)l.n), dim3(CopyTile<false>::TH), 0, s, l, f);
  return hipGetLastError();
}

// The IPC device-sync fence and the copy-out in one launch (small calls): every block first stores seq
// into every peer's flag slot (a system-scope release; idempotent, so no block depends on another
// being resident — the result stores of this rank's combine kernel are complete at the kernel boundary
// ahead of it; skipped when that kernel's tail already stored it, FlagTail::store = 0), then waits for
// every peer's slot in its own area to reach seq (the peers' result blocks have landed in this rank's
// `out` staging), then copies tiles. A wait that exceeds the wall-clock limit or sees the world's
// failed mark records the error and leaves without copying.
// The grid is at most kFlagCopyBlocks blocks that stride over the tiles: every block spins,
// and with one block per tile a 2 MiB call put ~256 spinning blocks per rank on the GPU (up to 4096 at
// MPJX_IPC_FUSE_KIB's cap). Where rank processes share a GPU, the slow rank's combine kernel — which
// stores the flag the spinners wait on — needs those CU slots; 64 blocks of 256 lanes per rank leave
// them free at P = 8 (16 KiB tiles: 1 MiB per pass, two passes for a 2 MiB call).
constexpr int kFlagCopyBlocks = 64;
template <bool NT>
__global__ __launch_bounds__(CopyTile<NT>::TH) void k_flags_copies(CopyList l, FlagTail f, int64_t bx) {
  const int j = threadIdx.x;
  __shared__ int bad;
  if (j == 0) bad = 0;
  __syncthreads();
  if (j < f.P && j != f.me) {
    if (f.store) __hip_atomic_store(f.peer[j], f.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const long long t0 = wall_clock64();
    for (unsigned it = 1; __hip_atomic_load(f.mine + j, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < f.seq; it++) {
      const bool gone = (it & 63) == 0 && __hip_atomic_load(f.failed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (gone || wall_clock64() - t0 > f.ticks) {
        __hip_atomic_store(f.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        bad = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (bad) return;
  const int64_t tiles = bx * l.n;
  for (int64_t g = blockIdx.x; g < tiles; g += gridDim.x) copy_tile<NT>(l, (int)(g / bx), g % bx);
}

hipError_t launch_flags_copies(const CopyList& l, const FlagTail& f, hipStream_t s) {
  if (l.n <= 0 || l.n > CopyList::kMax) return hipErrorInvalidValue;
  int64_t mx = 0;
  for (int i = 0; i < l.n; i++) mx = l.bytes[i] > mx ? l.bytes[i] : mx;
  const int64_t tb = CopyTile<false>::bytes;
  const int64_t bx = mx > 0 ? (mx + tb - 1) / tb : 1;
  if (bx * l.n > 4096) return hipErrorInvalidValue;  // small calls only (MPJX_IPC_FUSE_KIB)
  const int64_t grid = std::min<int64_t>(bx * l.n, kFlagCopyBlocks);
  hipLaunchKernelGGL(k_flags_copies<false>, dim3((unsigned)grid), dim3(CopyTile<false>::TH), 0, s, l, f, bx);
  return hipGetLastError();
}

hipError_t launch_copies(const CopyList& l, hipStream_t s) {
  if (l.n <= 0) return hipSuccess;
  if (l.n > CopyList::kMax) return hipErrorInvalidValue;
  int64_t mx = 0, total = 0;
  for (int i = 0; i < l.n; i++) {
    mx = l.bytes[i] > mx ? l.bytes[i] : mx;
    total += l.bytes[i];
  }
  if (mx == 0) return hipSuccess;
  const bool nt = total >= ((int64_t)64 << 20);
  const int64_t tb = nt ? CopyTile<true>::bytes : CopyTile<false>::bytes;
  const int64_t bx = (mx + tb - 1) / tb;
  if (bx > 0x7fffffff) return hipErrorInvalidValue;
  if (nt)
    hipLaunchKernelGGL(k_copies<true>, dim3((unsigned)bx, (unsigned)l.n), dim3(CopyTile<true>::TH), 0, s, l);
  else
    hipLaunchKernelGGL(k_copies<false>, dim3((unsigned)bx, (unsigned)l.n), dim3(CopyTile<false>::TH), 0, s, l);
  return hipGetLastError();
}

}  // namespace mpjx
