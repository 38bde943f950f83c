// mpjx_k_mpjbuf.hip — the per-edge combine of MST_Reduce on a packed message, with the mpjbuf
// section walk on the device: acc[i] = payload[i] (op) acc[i], where the payload is the big-endian
// element run of the sections of an mpjbuf static-buffer image (src/mpjbuf/Buffer.java:609-704:
// each section = type code byte, 3 pad bytes, big-endian int32 element count, then the elements,
// the next header at the next 8-byte boundary; src/mpjbuf/NIOBuffer.java:520-563 big-endian bulk
// get). The reference unpacks such a message into recvbuf on the host (byte swap + copy,
// SimplePackerDouble.java:81-99) and then runs perform(); here the kernel reads the headers, swaps
// the payload words in registers and combines: one HBM pass (read payload + acc, write acc) with no
// host involvement, so the image may sit anywhere the device can read (device memory, or pinned host
// memory a NIC wrote into).
//
// Every block walks the section headers itself (a few L2-resident 8-byte reads; one section for a
// typed message) into LDS. A one-section image (the typed message) takes the streaming body: 16 B
// of acc and payload per lane, the payload fetched with the widest loads its alignment allows (its
// start is 8-byte aligned), swapped in registers. Otherwise each
// lane combines elements, fetching each base word from the section holding it (sections may split
// a MAXLOC pair) with one naturally aligned load and a register byte swap. Malformed images (wrong type code, counts
// that overrun the image or do not add up to `count`, more than kMaxSections sections) leave acc
// untouched and store an error code into *status (one vector store from block 0).
#include "mpjx_kernels.hpp"

namespace mpjx {

constexpr int kMaxSections = 64;
// the single-section body's tile: 1024 lanes x one 16-B step, the streaming form of the combines
// (mpjx_kernels.hpp: cold operands favour it over 256 x 4)
constexpr int kThreadsMb = 1024;
constexpr int kVecU = 1;

// 16 bytes from p with the widest loads its alignment `al` (16, 8, 4 or 1) allows (uniform per launch);
// non-temporal, as every operand of the streaming combines (mpjx_kernels.hpp, cold-operand tuning)
__device__ __forceinline__ v4u load16(const unsigned char* p, int al) {
  v4u v;
  if (al == 16) {
    v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  } else if (al == 8) {
    const uint64_t lo = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(p));
    const uint64_t hi = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(p) + 1);
    __builtin_memcpy(&v, &lo, 8);
    __builtin_memcpy(reinterpret_cast<char*>(&v) + 8, &hi, 8);
  } else if (al == 4) {
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = reinterpret_cast<const uint32_t*>(p)[k];
  } else {
    unsigned char b[16];
#pragma unroll
    for (int k = 0; k < 16; k++) b[k] = p[k];
    __builtin_memcpy(&v, b, 16);
  }
  return v;
}

struct MpjbufArgs {
  void* acc;                  // native, count elements of F::T
  const unsigned char* msg;   // mpjbuf static-buffer image (its data start, after any device overhead)
  int64_t msg_bytes;
  int64_t count;              // F::T elements expected
  int code;                   // section type code expected (mpjbuf.Type code: base type - 1)
  int* status;                // device word: 0 = ok, else MPJX_MPJBUF_* error
};

__device__ __forceinline__ int64_t be32(const unsigned char* p) {
  return (int64_t)(int32_t)(((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]);
}

template <class F>
__global__ __launch_bounds__(kThreadsMb) void k_mpjbuf(MpjbufArgs a) {
  using T = typename F::T;
  constexpr int WS = WordOf<T>::value;
  constexpr int M = sizeof(T) / WS;  // base words per element (2 for the pair types)
  __shared__ int64_t pos[kMaxSections], first[kMaxSections + 1];
  __shared__ int nsec, bad;
  if (threadIdx.x == 0) {
    const int64_t want = a.count * M;  // base words
    int64_t p = 0, have = 0;
    int k = 0, err = 0;
    while (have < want) {
      const int64_t h = (p + 7) / 8 * 8;  // ALIGNMENT_UNIT
      if (k == kMaxSections) { err = 4; break; }
      if (h + 8 > a.msg_bytes) { err = 3; break; }
      const int64_t n = be32(a.msg + h + 4);
      if ((int)a.msg[h] != a.code) { err = 1; break; }
      if (n < 0 || h + 8 + n * WS > a.msg_bytes) { err = 3; break; }
      pos[k] = h + 8;
      first[k] = have;
      k++;
      have += n;
      p = h + 8 + n * WS;
    }
    if (!err && have != want) err = 2;
    first[k] = have;
    nsec = k;
    bad = err;
    if (err && blockIdx.x == 0) *a.status = err;
  }
  __syncthreads();
  if (bad) return;
  const int ns = nsec;
  const bool aligned = ((uintptr_t)a.msg & 7u) == 0;
  T* acc = reinterpret_cast<T*>(a.acc);
  int64_t first_scalar = 0;  // elements below this were done by the vector body
  if (ns == 1 && ((uintptr_t)acc & 15u) == 0) {
    // one section (a typed message): 16 B of acc and of the payload per lane and step; the payload
    // start is only 8-byte aligned in general (header at 0, data at 8), so its 16 B are fetched with
    // the widest loads its alignment allows. (Realigning across lanes instead — one aligned 16-B load
    // plus a lane shift, the wave's last lane loading its second half itself — ran 142-143 us cold
    // against 131 for the two 8-B loads, profiles/r02/cold/mpjbuf_cold.jsonl.) Then swap, combine, store.
    constexpr int W = 16 / sizeof(T);
    const unsigned char* pay = a.msg + pos[0];
    const int al = ((uintptr_t)pay & 15u) == 0 ? 16 : (((uintptr_t)pay & 7u) == 0 ? 8 : (((uintptr_t)pay & 3u) == 0 ? 4 : 1));
    const int64_t nv = a.count / W;
    const int64_t tile = (int64_t)blockDim.x * kVecU;
    for (int64_t base = (int64_t)blockIdx.x * tile; base < nv; base += (int64_t)gridDim.x * tile) {
      v4u x[kVecU], y[kVecU];
#pragma unroll
      for (int u = 0; u < kVecU; u++) {
        const int64_t i = base + u * blockDim.x + threadIdx.x;
        if (i < nv) {
          x[u] = load16(pay + i * 16, al);
          y[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(acc) + i);
        }
      }
#pragma unroll
      for (int u = 0; u < kVecU; u++) {
        const int64_t i = base + u * blockDim.x + threadIdx.x;
        if (i < nv) {
          const v4u xs = swap_words<WS>(x[u]);
          T e[W], f[W];
          __builtin_memcpy(e, &xs, 16);
          __builtin_memcpy(f, &y[u], 16);
#pragma unroll
          for (int w = 0; w < W; w++) f[w] = F::apply(e[w], f[w]);
          v4u r;
          __builtin_memcpy(&r, f, 16);
          __builtin_nontemporal_store(r, reinterpret_cast<v4u*>(acc) + i);
        }
      }
    }
    if (blockIdx.x != 0) return;  // block 0 finishes the sub-vector tail below
    first_scalar = nv * W;
  }
  for (int64_t i = first_scalar + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.count;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t w[M];
    int s = 0;
#pragma unroll
    for (int j = 0; j < M; j++) {
      const int64_t g = i * M + j;
      while (s + 1 < ns && g >= first[s + 1]) s++;
      const unsigned char* src = a.msg + pos[s] + (g - first[s]) * WS;
      uint64_t v = 0;
      if (aligned) {  // payloads start 8-aligned: one naturally aligned load per word, swapped
        if constexpr (WS == 1) v = *src;
        else if constexpr (WS == 2) v = __builtin_bswap16(*reinterpret_cast<const uint16_t*>(src));
        else if constexpr (WS == 4) v = __builtin_bswap32(*reinterpret_cast<const uint32_t*>(src));
        else v = __builtin_bswap64(*reinterpret_cast<const uint64_t*>(src));
      } else {
#pragma unroll
        for (int b = 0; b < WS; b++) v = (v << 8) | src[b];  // big-endian word -> value
      }
      w[j] = v;
    }
    T in;
    if constexpr (M == 1) {
      if constexpr (WS == 1) { uint8_t x = (uint8_t)w[0]; __builtin_memcpy(&in, &x, 1); }
      else if constexpr (WS == 2) { uint16_t x = (uint16_t)w[0]; __builtin_memcpy(&in, &x, 2); }
      else if constexpr (WS == 4) { uint32_t x = (uint32_t)w[0]; __builtin_memcpy(&in, &x, 4); }
      else { __builtin_memcpy(&in, &w[0], 8); }
    } else {
      unsigned char raw[sizeof(T)];
#pragma unroll
      for (int j = 0; j < M; j++) {
        if constexpr (WS == 2) { uint16_t x = (uint16_t)w[j]; __builtin_memcpy(raw + j * WS, &x, WS); }
        else if constexpr (WS == 4) { uint32_t x = (uint32_t)w[j]; __builtin_memcpy(raw + j * WS, &x, WS); }
        else { __builtin_memcpy(raw + j * WS, &w[j], WS); }
      }
      __builtin_memcpy(&in, raw, sizeof(T));
    }
    acc[i] = F::apply(in, acc[i]);
  }
}

template <class F>
static hipError_t go(const MpjbufArgs& a, hipStream_t s) {
  // one kThreadsMb-lane x kVecU x 16-B tile per block for the single-section body; the scalar body strides
  const int64_t per = kThreadsMb * kVecU * (int64_t)(16 / sizeof(typename F::T));
  int64_t blocks = (a.count + per - 1) / per;
  blocks = blocks < 1 ? 1 : (blocks > (1 << 20) ? (1 << 20) : blocks);
  hipLaunchKernelGGL(k_mpjbuf<F>, dim3((unsigned)blocks), dim3(kThreadsMb), 0, s, a);
  return hipGetLastError();
}

template <template <class> class F>
static hipError_t by_int(int type, const MpjbufArgs& a, hipStream_t s) {
  switch (type) {
    case 1: return go<F<uint8_t>>(a, s);
    case 2: case 3: return go<F<uint16_t>>(a, s);
    case 5: return go<F<uint32_t>>(a, s);
    case 6: return go<F<uint64_t>>(a, s);
  }
  return hipErrorInvalidValue;
}
template <template <class> class F>
static hipError_t by_num(int type, const MpjbufArgs& a, hipStream_t s) {  // signed compare, CHAR unsigned
  switch (type) {
    case 1: return go<F<int8_t>>(a, s);
    case 2: return go<F<uint16_t>>(a, s);
    case 3: return go<F<int16_t>>(a, s);
    case 5: return go<F<int32_t>>(a, s);
    case 6: return go<F<int64_t>>(a, s);
    case 7: return go<F<float>>(a, s);
    case 8: return go<F<double>>(a, s);
  }
  return hipErrorInvalidValue;
}
template <template <class> class F>
static hipError_t by_wrap(int type, const MpjbufArgs& a, hipStream_t s) {  // Java wraparound: unsigned storage
  switch (type) {
    case 1: return go<F<uint8_t>>(a, s);
    case 2: case 3: return go<F<uint16_t>>(a, s);
    case 5: return go<F<uint32_t>>(a, s);
    case 6: return go<F<uint64_t>>(a, s);
    case 7: return go<F<float>>(a, s);
    case 8: return go<F<double>>(a, s);
  }
  return hipErrorInvalidValue;
}
template <template <class> class F>
static hipError_t by_pair(int type, const MpjbufArgs& a, hipStream_t s) {
  switch (type) {
    case 0x103: return go<F<int16_t>>(a, s);
    case 0x105: return go<F<int32_t>>(a, s);
    case 0x106: return go<F<int64_t>>(a, s);
    case 0x107: return go<F<float>>(a, s);
    case 0x108: return go<F<double>>(a, s);
  }
  return hipErrorInvalidValue;
}

// The same functors the collectives use (mpjx_k_<family>.hip): signed MAX/MIN except CHAR, unsigned
// storage for the wrapping ops.
hipError_t launch_mpjbuf(int op, int type, bool faithful, void* acc, const void* msg, int64_t msg_bytes,
                         int64_t count, int* status, hipStream_t s) {
  MpjbufArgs a{acc, (const unsigned char*)msg, msg_bytes, count, (type & 0xff) - 1, status};
  if (faithful && (op == 8 || op == 10)) return by_int<Keep>(type, a, s);
  switch (op) {
    case 1: return by_num<Max>(type, a, s);
    case 2: return by_num<Min>(type, a, s);
    case 3: return by_wrap<Sum>(type, a, s);
    case 4: return by_wrap<Prod>(type, a, s);
    case 5: return go<Land>(a, s);
    case 6: return by_int<Band>(type, a, s);
    case 7: return go<Lor>(a, s);
    case 8: return by_int<Bor>(type, a, s);
    case 9: return go<Lxor>(a, s);
    case 10: return by_int<Bxor>(type, a, s);
    case 11: return by_pair<Maxloc>(type, a, s);
    case 12: return by_pair<Minloc>(type, a, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace mpjx
