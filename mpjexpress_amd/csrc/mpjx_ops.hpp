// mpjx_ops.hpp — the element-wise Op functors (device side), one per typed class of the reference.
//
// Each functor F has `using T` (storage type) and `static T apply(T in, T acc)` computing what the
// reference's typed perform() body stores into arr[i] given arr1[i] = in and arr[i] = acc:
//   SUM   src/mpi/SumDouble.java:52-53   arr[i] = (T)(arr1[i] + arr[i])
//   PROD  src/mpi/ProdInt.java:51-52     arr[i] = (T)(arr1[i] * arr[i])
//   MAX   src/mpi/MaxDouble.java:51-53   if (arr1[i] > arr[i]) arr[i] = arr1[i]
//   MIN   src/mpi/MinDouble.java:53-55   if (arr1[i] < arr[i]) arr[i] = arr1[i]
//   BAND/BOR/BXOR src/mpi/BandInt.java:39-40, BorInt.java:53-54, BxorInt.java:52-53
//   LAND/LOR/LXOR src/mpi/LandBoolean.java:53-54, LorBoolean.java:53-54, LxorBoolean.java:52-53
// Java integer arithmetic wraps, so SUM/PROD/B* are computed on unsigned storage of the same width
// (identical bits for byte/short/int/long, and char is unsigned anyway); products of 8/16-bit
// values are formed in uint32 because C++ would promote them to (overflowing) int. MAX/MIN keep the
// signedness of the Java type (char unsigned) and, for float/double, the exact comparison form —
// a NaN never replaces the accumulator and a +0/-0 tie keeps it — which fmax/v_max would not.
#pragma once
#include <stdint.h>

#ifndef MPJX_HD
#define MPJX_HD __host__ __device__ __forceinline__
#endif

namespace mpjx {

template <class U> struct Sum {
  using T = U;
  static MPJX_HD T apply(T x, T y) {
    if constexpr (sizeof(T) < 4 && !(T(-1) < T(0)))  // u8/u16: avoid int promotion
      return (T)((uint32_t)x + (uint32_t)y);
    else
      return (T)(x + y);
  }
};
template <class U> struct Prod {
  using T = U;
  static MPJX_HD T apply(T x, T y) {
    if constexpr (sizeof(T) < 4 && !(T(-1) < T(0)))
      return (T)((uint32_t)x * (uint32_t)y);
    else
      return (T)(x * y);
  }
};
template <class U> struct Max {
  using T = U;
  static MPJX_HD T apply(T x, T y) { return (x > y) ? x : y; }
};
template <class U> struct Min {
  using T = U;
  static MPJX_HD T apply(T x, T y) { return (x < y) ? x : y; }
};
template <class U> struct Band {
  using T = U;
  static MPJX_HD T apply(T x, T y) { return (T)(x & y); }
};
template <class U> struct Bor {
  using T = U;
  static MPJX_HD T apply(T x, T y) { return (T)(x | y); }
};
template <class U> struct Bxor {
  using T = U;
  static MPJX_HD T apply(T x, T y) { return (T)(x ^ y); }
};
struct Land {
  using T = uint8_t;
  static MPJX_HD T apply(T x, T y) { return (T)((x != 0) & (y != 0)); }
};
struct Lor {
  using T = uint8_t;
  static MPJX_HD T apply(T x, T y) { return (T)((x != 0) | (y != 0)); }
};
struct Lxor {
  using T = uint8_t;
  static MPJX_HD T apply(T x, T y) { return (T)((x != 0) ^ (y != 0)); }
};
// FAITHFUL BOR/BXOR: the typed classes declare perform(Object, Object, int), an overload that never
// overrides Op.perform(Object, int, int) (src/mpi/BorInt.java:50, BxorInt.java:48 vs Op.java:56),
// so every call site runs the empty base method and the accumulator is kept unchanged.
template <class U> struct Keep {
  using T = U;
  static MPJX_HD T apply(T, T y) { return y; }
};

// MAXLOC / MINLOC on (value, index) pairs (src/mpi/Maxloc.java, src/mpi/Minloc.java, the
// User_function pair ops of MPI.MAXLOC / MPI.MINLOC): `in` replaces `acc` when its value compares
// strictly greater (smaller); on equal values only the index is lowered. Like the typed ops, a NaN
// value never wins and an equal +0/-0 keeps the accumulator's value.
template <class V>
struct alignas(2 * sizeof(V)) Pair {
  V v, l;
};
// Written with selects, not early returns: returning one of two structs from branches left the
// P = 8 MST tree's pairs in scratch memory (80-160 B per lane) on gfx950.
template <class V> struct Maxloc {
  using T = Pair<V>;
  static MPJX_HD T apply(T x, T y) {
    const bool win = x.v > y.v, tie = x.v == y.v;
    T r;
    r.v = win ? x.v : y.v;
    r.l = (win || (tie && x.l < y.l)) ? x.l : y.l;
    return r;
  }
};
template <class V> struct Minloc {
  using T = Pair<V>;
  static MPJX_HD T apply(T x, T y) {
    const bool win = x.v < y.v, tie = x.v == y.v;
    T r;
    r.v = win ? x.v : y.v;
    r.l = (win || (tie && x.l < y.l)) ? x.l : y.l;
    return r;
  }
};

}  // namespace mpjx
