/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see mpjx_oracle.h). Never linked into libmpjx.
 *
 * Plain-C restatement of MPJ Express 0.44's reduction path, written from the Java source:
 *   - typed element-wise Op bodies  src/mpi/{Sum,Prod,Max,Min}{Byte,Short,Int,Long,Char,Float,Double}.java,
 *     src/mpi/{Band,Bor,Bxor}{Byte,Short,Int,Long,Char}.java, src/mpi/{Land,Lor,Lxor}Boolean.java
 *     (templates src/mpi/<Op>Type.java.in expanded by src/mpi/generate.pl:80-113)
 *   - worker validity tables         src/mpi/<Op>Worker.java (e.g. SumWorker.java:47-77, BandWorker.java:44-62)
 *   - collective algorithms          src/mpi/PureIntracomm.java:702-736 (MST_Broadcast),
 *     :1923-1992 (Reduce/MST_Reduce), :1994-2057 (FT_Reduce), :2168-2314 (Allreduce/FT_Allreduce),
 *     :2355-2456 (Reduce_scatter/BKT/FT), :2495-2545 (Scan), :1132-1171 (FT_Scatter)
 *   - host staging cost model         src/mpjbuf/NIOBuffer.java:42,520-563 (big-endian bulk put/get)
 *
 * Compiled -O2 without fast-math: IEEE results, subnormals kept, no FMA contraction needed (every
 * combine is a single + or *).
 */
#define _GNU_SOURCE
#include "mpjx_oracle.h"

#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

int ora_type_size(int type) {
  /* src/mpi/BasicType.java:50-140 byteSize */
  switch (type) {
    case ORA_BYTE: return 1;
    case ORA_CHAR: return 2;
    case ORA_SHORT: return 2;
    case ORA_BOOLEAN: return 1;
    case ORA_INT: return 4;
    case ORA_LONG: return 8;
    case ORA_FLOAT: return 4;
    case ORA_DOUBLE: return 8;
    case ORA_SHORT2: return 4;
    case ORA_INT2: case ORA_FLOAT2: return 8;
    case ORA_LONG2: case ORA_DOUBLE2: return 16;
    default: return 0;
  }
}

static int is_pair(int type) { return type >= 0x103 && type <= 0x108 && type != 0x104; }

int ora_check(int op, int type) {
  if (ora_type_size(type) == 0) return 2; /* `default: return null` in every *Worker */
  if (op == ORA_MAXLOC || op == ORA_MINLOC) return is_pair(type) ? 0 : 1; /* Maxloc.java: else Abort */
  if (is_pair(type)) return 1; /* typed workers on a Contiguous(2) buffer: not a valid reduction */
  switch (op) {
    case ORA_SUM: case ORA_PROD: case ORA_MAX: case ORA_MIN:
      /* SumWorker.java:60 ProdWorker MaxWorker MinWorker: BOOLEAN throws */
      return type == ORA_BOOLEAN ? 1 : 0;
    case ORA_BAND: case ORA_BOR: case ORA_BXOR:
      /* BandWorker.java:44-62: BOOLEAN, FLOAT, DOUBLE throw */
      return (type == ORA_BOOLEAN || type == ORA_FLOAT || type == ORA_DOUBLE) ? 1 : 0;
    case ORA_LAND: case ORA_LOR: case ORA_LXOR:
      /* LandWorker.java:48-74: every non-boolean throws */
      return type == ORA_BOOLEAN ? 0 : 1;
    default: return 2;
  }
}

/* acc[i] = in[i] (op) acc[i]; x = in (arr1[i]), y = acc (arr[i]) exactly as in the Java bodies. */
#define LOOP(T, EXPR)                                          \
  do {                                                         \
    T *a_ = (T *)acc;                                          \
    const T *b_ = (const T *)in;                               \
    for (int64_t i = lo; i < hi; i++) {                        \
      T x = b_[i], y = a_[i];                                  \
      a_[i] = (T)(EXPR);                                       \
    }                                                          \
  } while (0)

/* byte/short/char: Java promotes to int, computes, narrows with (T) — two's-complement wrap.
 * int/long: Java wraps mod 2^32/2^64 — computed in unsigned to avoid C signed-overflow UB.
 * char*char can overflow Java int; the narrowed low 16 bits equal the low 16 bits of the exact
 * product, computed here in uint32. */
#define INTEGRAL_CASES(OPX)                                                          \
  case ORA_BYTE: LOOP(int8_t, OPX(int8_t, uint32_t)); break;                          \
  case ORA_SHORT: LOOP(int16_t, OPX(int16_t, uint32_t)); break;                       \
  case ORA_CHAR: LOOP(uint16_t, OPX(uint16_t, uint32_t)); break;                      \
  case ORA_INT: LOOP(int32_t, OPX(int32_t, uint32_t)); break;                         \
  case ORA_LONG: LOOP(int64_t, OPX(int64_t, uint64_t)); break;

#define ADD_W(T, U) ((T)((U)x + (U)y))
#define MUL_W(T, U) ((T)((U)x * (U)y))
#define AND_W(T, U) ((T)((U)x & (U)y))
#define OR_W(T, U) ((T)((U)x | (U)y))
#define XOR_W(T, U) ((T)((U)x ^ (U)y))
#define MAX_J(T, U) ((x > y) ? x : y) /* MaxDouble.java:51-53: if (arr1[i] > arr[i]) arr[i] = arr1[i] */
#define MIN_J(T, U) ((x < y) ? x : y) /* MinDouble.java:53-55: if (arr1[i] < arr[i]) arr[i] = arr1[i] */

/* MAXLOC / MINLOC (src/mpi/Maxloc.java, src/mpi/Minloc.java, User_function.Call(invec, outvec)):
 * for each pair, if (inval > outval) out = (inval, inloc); else if (inval == outval and
 * inloc < outloc) outloc = inloc. MINLOC with `<`. Here in = `in`, out = `acc`. */
#define LOC_LOOP(V, CMP)                                                   \
  do {                                                                     \
    V *o_ = (V *)acc;                                                      \
    const V *x_ = (const V *)in;                                           \
    for (int64_t i = lo; i < hi; i++) {                                    \
      V inval = x_[2 * i], outval = o_[2 * i];                             \
      if (inval CMP outval) {                                              \
        o_[2 * i] = inval;                                                 \
        o_[2 * i + 1] = x_[2 * i + 1];                                     \
      } else if (inval == outval) {                                        \
        V inloc = x_[2 * i + 1];                                           \
        if (inloc < o_[2 * i + 1]) o_[2 * i + 1] = inloc;                  \
      }                                                                    \
    }                                                                      \
  } while (0)

static void apply_loc(int op, int type, void *acc, const void *in, int64_t lo, int64_t hi) {
  if (op == ORA_MAXLOC) {
    switch (type) {
      case ORA_SHORT2: LOC_LOOP(int16_t, >); break;
      case ORA_INT2: LOC_LOOP(int32_t, >); break;
      case ORA_LONG2: LOC_LOOP(int64_t, >); break;
      case ORA_FLOAT2: LOC_LOOP(float, >); break;
      case ORA_DOUBLE2: LOC_LOOP(double, >); break;
    }
  } else {
    switch (type) {
      case ORA_SHORT2: LOC_LOOP(int16_t, <); break;
      case ORA_INT2: LOC_LOOP(int32_t, <); break;
      case ORA_LONG2: LOC_LOOP(int64_t, <); break;
      case ORA_FLOAT2: LOC_LOOP(float, <); break;
      case ORA_DOUBLE2: LOC_LOOP(double, <); break;
    }
  }
}

void ora_apply(int op, int type, void *acc, const void *in, int64_t lo, int64_t hi) {
  if (op == ORA_MAXLOC || op == ORA_MINLOC) {
    apply_loc(op, type, acc, in, lo, hi);
    return;
  }
  switch (op) {
    case ORA_SUM: /* SumDouble.java:52-53 arr[i] = (T)(arr1[i] + arr[i]) */
      switch (type) {
        INTEGRAL_CASES(ADD_W)
        case ORA_FLOAT: LOOP(float, x + y); break;
        case ORA_DOUBLE: LOOP(double, x + y); break;
      }
      break;
    case ORA_PROD: /* ProdInt.java:51-52 arr[i] = (T)(arr1[i] * arr[i]) */
      switch (type) {
        INTEGRAL_CASES(MUL_W)
        case ORA_FLOAT: LOOP(float, x * y); break;
        case ORA_DOUBLE: LOOP(double, x * y); break;
      }
      break;
    case ORA_MAX:
      switch (type) {
        INTEGRAL_CASES(MAX_J)
        case ORA_FLOAT: LOOP(float, MAX_J(, )); break;
        case ORA_DOUBLE: LOOP(double, MAX_J(, )); break;
      }
      break;
    case ORA_MIN:
      switch (type) {
        INTEGRAL_CASES(MIN_J)
        case ORA_FLOAT: LOOP(float, MIN_J(, )); break;
        case ORA_DOUBLE: LOOP(double, MIN_J(, )); break;
      }
      break;
    case ORA_BAND: /* BandInt.java:39-40 */
      switch (type) { INTEGRAL_CASES(AND_W) }
      break;
    case ORA_BOR: /* BorInt.java:53-54 (body; see A3 for dispatch) */
      switch (type) { INTEGRAL_CASES(OR_W) }
      break;
    case ORA_BXOR: /* BxorInt.java:52-53 (body; see A3 for dispatch) */
      switch (type) { INTEGRAL_CASES(XOR_W) }
      break;
    /* Java booleans: 0/1 bytes. LandBoolean.java:53-54, LorBoolean.java:53-54, LxorBoolean.java:52-53 */
    case ORA_LAND: LOOP(uint8_t, (x != 0) && (y != 0)); break;
    case ORA_LOR: LOOP(uint8_t, (x != 0) || (y != 0)); break;
    case ORA_LXOR: LOOP(uint8_t, (x != 0) != (y != 0)); break;
  }
}

/* ------------------------------------------------------------------------------------------- */
/* The typed Op object: createInitialBuffer / perform / getResultant (SumDouble.java:49-67).    */

typedef struct {
  int op, type, esz;
  unsigned flags;
  char *arr;
  int len;
} jop;

static char *E(void *base, int idx, int esz) { return (char *)base + (int64_t)idx * esz; }

/* createInitialBuffer(buf, offset, count): arr = new T[len]; arraycopy(buf, offset, arr, offset, count) */
static void jop_init(jop *o, int op, int type, unsigned flags, const void *buf, int offset, int count,
                     int len) {
  o->op = op;
  o->type = type;
  o->esz = ora_type_size(type);
  o->flags = flags;
  o->len = len;
  o->arr = (char *)calloc((size_t)(len > 0 ? len : 1), (size_t)o->esz);
  memcpy(E(o->arr, offset, o->esz), E((void *)buf, offset, o->esz), (size_t)count * o->esz);
}

/* perform(buf1, offset, count). Faithful: the class's own loop bound (A4) and the BOR/BXOR
 * overload that never overrides Op.perform (A3: BorInt.java:50, BxorInt.java:48 vs Op.java:56). */
static void jop_perform(jop *o, const void *buf1, int offset, int count) {
  if ((o->flags & ORA_FLAG_FAITHFUL) && o->op <= 10) {
    if (o->op == ORA_BOR || o->op == ORA_BXOR) return;
    int lo = (o->op == ORA_MIN || o->op == ORA_PROD) ? 0 : offset; /* MinDouble.java:53 vs SumDouble.java:52 */
    ora_apply(o->op, o->type, o->arr, buf1, lo, count);
  } else {
    ora_apply(o->op, o->type, o->arr, buf1, offset, (int64_t)offset + count);
  }
}

/* getResultant(buf, offset, count): arraycopy(arr, offset, buf, offset, count) */
static void jop_result(jop *o, void *buf, int offset, int count) {
  memcpy(E(buf, offset, o->esz), E(o->arr, offset, o->esz), (size_t)count * o->esz);
}
static void jop_free(jop *o) { free(o->arr); o->arr = NULL; }

static int maxi(int a, int b) { return a > b ? a : b; }

/* ------------------------------------------------------------------------------------------- */
/* MST_Reduce (PureIntracomm.java:1943-1992), simulated for all ranks at once. Each rank recurses
 * into its own half first (root's half with `root`, the other with `srce`), then srce sends its
 * partial and root folds it in: acc = received (op) acc. */
static void mst_reduce(void *const *buf, int offset, int count, int type, int op, unsigned flags,
                       int root, int left, int right) {
  if (left == right) return;
  int mid = (left + right) / 2;
  int srce = (root <= mid) ? right : left;
  if (root <= mid) {
    mst_reduce(buf, offset, count, type, op, flags, root, left, mid);
    mst_reduce(buf, offset, count, type, op, flags, srce, mid + 1, right);
  } else {
    mst_reduce(buf, offset, count, type, op, flags, srce, left, mid);
    mst_reduce(buf, offset, count, type, op, flags, root, mid + 1, right);
  }
  int esz = ora_type_size(type);
  jop o;
  jop_init(&o, op, type, flags, buf[root], offset, count, offset + count);
  /* recv(buf, offset, count, ..., srce): the message is srce's buf region at send time */
  memcpy(E(buf[root], offset, esz), E(buf[srce], offset, esz), (size_t)count * esz);
  jop_perform(&o, buf[root], offset, count);
  jop_result(&o, buf[root], offset, count);
  jop_free(&o);
}

/* MST_Broadcast (PureIntracomm.java:702-736) */
static void mst_bcast(void *const *buf, int offset, int count, int esz, int root, int left, int right) {
  if (left == right) return;
  int mid = (left + right) / 2;
  int dest = (root <= mid) ? right : left;
  memcpy(E(buf[dest], offset, esz), E(buf[root], offset, esz), (size_t)count * esz);
  if (root <= mid) {
    mst_bcast(buf, offset, count, esz, root, left, mid);
    mst_bcast(buf, offset, count, esz, dest, mid + 1, right);
  } else {
    mst_bcast(buf, offset, count, esz, dest, left, mid);
    mst_bcast(buf, offset, count, esz, root, mid + 1, right);
  }
}

/* Scratch copies [0, count) of each rank's send region, for MPI-semantics runs. */
static void **scratch_from(int P, void *const *src, int off, int count, int esz) {
  void **w = (void **)calloc((size_t)P, sizeof(void *));
  for (int r = 0; r < P; r++) {
    w[r] = calloc((size_t)(count > 0 ? count : 1), (size_t)esz);
    if (src) memcpy(w[r], E(src[r], off, esz), (size_t)count * esz);
  }
  return w;
}
static void scratch_free(int P, void **w) {
  for (int r = 0; r < P; r++) free(w[r]);
  free(w);
}

/* FT_Reduce (PureIntracomm.java:2033-2056): root starts from its own send, folds i = 0..P-1 (i != root). */
static void ft_reduce(int P, unsigned flags, void *const *send, int soff, void *const *recv, int roff,
                      int count, int type, int op, int root) {
  int esz = ora_type_size(type);
  for (int r = 0; r < P; r++) {
    jop o;
    jop_init(&o, op, type, flags, send[r], soff, count, maxi(soff, roff) + count);
    if (soff != roff) { /* arr indexed at recvoffset below (quirk A4): move the copy there */
      memmove(E(o.arr, roff, esz), E(o.arr, soff, esz), (size_t)count * esz);
    }
    if ((flags & ORA_FLAG_FAITHFUL) && soff != roff) {
      /* Java leaves arr filled at sendoffset; perform/getResultant read at recvoffset. */
      memset(o.arr, 0, (size_t)o.len * esz);
      memcpy(E(o.arr, soff, esz), E(send[r], soff, esz), (size_t)count * esz);
    }
    if (r == root) {
      for (int i = 0; i < P; i++) {
        if (i == r) continue;
        memcpy(E(recv[r], roff, esz), E(send[i], soff, esz), (size_t)count * esz);
        jop_perform(&o, recv[r], roff, count);
      }
    }
    if (r == root || (flags & ORA_FLAG_FAITHFUL)) jop_result(&o, recv[r], roff, count);
    jop_free(&o);
  }
}

int ora_reduce(int P, unsigned flags, void *const *send, int soff, void *const *recv, int roff,
               int count, int type, int op, int root) {
  int c = ora_check(op, type);
  if (c) return c;
  int esz = ora_type_size(type);
  if (flags & ORA_FLAG_OLD) {
    if (flags & ORA_FLAG_FAITHFUL) {
      ft_reduce(P, flags, send, soff, recv, roff, count, type, op, root);
    } else {
      void **w = scratch_from(P, send, soff, count, esz);
      void **o = scratch_from(P, NULL, 0, count, esz);
      ft_reduce(P, flags, w, 0, o, 0, count, type, op, root);
      memcpy(E(recv[root], roff, esz), o[root], (size_t)count * esz);
      scratch_free(P, w);
      scratch_free(P, o);
    }
    return 0;
  }
  if (flags & ORA_FLAG_FAITHFUL) {
    /* PureIntracomm.java:1937-1939: copy at recvoffset, reduce at sendoffset (quirk A4) */
    for (int r = 0; r < P; r++)
      memcpy(E(recv[r], roff, esz), E(send[r], soff, esz), (size_t)count * esz);
    mst_reduce(recv, soff, count, type, op, flags, root, 0, P - 1);
  } else {
    void **w = scratch_from(P, send, soff, count, esz);
    mst_reduce(w, 0, count, type, op, flags, root, 0, P - 1);
    memcpy(E(recv[root], roff, esz), w[root], (size_t)count * esz);
    scratch_free(P, w);
  }
  return 0;
}

int ora_bcast(int P, unsigned flags, void *const *buf, int off, int count, int type, int root) {
  (void)flags;
  mst_bcast(buf, off, count, ora_type_size(type), root, 0, P - 1);
  return 0;
}

/* FT_Allreduce (PureIntracomm.java:2267-2311): every rank starts from its own send and folds the
 * others in ascending rank order, so results may differ per rank for float. */
static void ft_allreduce(int P, unsigned flags, void *const *send, int soff, void *const *recv, int roff,
                         int count, int type, int op) {
  int esz = ora_type_size(type);
  for (int r = 0; r < P; r++) {
    jop o;
    jop_init(&o, op, type, flags, send[r], soff, count, maxi(soff, roff) + count);
    if (!(flags & ORA_FLAG_FAITHFUL) && soff != roff)
      memmove(E(o.arr, roff, esz), E(o.arr, soff, esz), (size_t)count * esz);
    for (int i = 0; i < P; i++) {
      if (i == r) continue;
      memcpy(E(recv[r], roff, esz), E(send[i], soff, esz), (size_t)count * esz);
      jop_perform(&o, recv[r], roff, count);
    }
    jop_result(&o, recv[r], roff, count);
    jop_free(&o);
  }
}

int ora_allreduce(int P, unsigned flags, void *const *send, int soff, void *const *recv, int roff,
                  int count, int type, int op) {
  int c = ora_check(op, type);
  if (c) return c;
  int esz = ora_type_size(type);
  if (flags & ORA_FLAG_OLD) {
    if (flags & ORA_FLAG_FAITHFUL) {
      ft_allreduce(P, flags, send, soff, recv, roff, count, type, op);
    } else {
      void **w = scratch_from(P, send, soff, count, esz);
      void **o = scratch_from(P, NULL, 0, count, esz);
      ft_allreduce(P, flags, w, 0, o, 0, count, type, op);
      for (int r = 0; r < P; r++) memcpy(E(recv[r], roff, esz), o[r], (size_t)count * esz);
      scratch_free(P, w);
      scratch_free(P, o);
    }
    return 0;
  }
  /* PureIntracomm.java:2180-2183: Reduce(root 0) + Bcast(root 0) */
  if (flags & ORA_FLAG_FAITHFUL) {
    ora_reduce(P, flags, send, soff, recv, roff, count, type, op, 0);
    mst_bcast(recv, roff, count, esz, 0, 0, P - 1);
  } else {
    void **w = scratch_from(P, send, soff, count, esz);
    mst_reduce(w, 0, count, type, op, flags, 0, 0, P - 1);
    mst_bcast(w, 0, count, esz, 0, 0, P - 1);
    for (int r = 0; r < P; r++) memcpy(E(recv[r], roff, esz), w[r], (size_t)count * esz);
    scratch_free(P, w);
  }
  return 0;
}

/* BKT_Reduce_scatter (PureIntracomm.java:2377-2439), simulated round by round. Correct for P <= 2;
 * for P >= 3 it reproduces defect A9 (same block resent every round, zero tmpbuf folded over the
 * whole vector, user's sendbuf overwritten). */
static void bkt_reduce_scatter(int P, unsigned flags, void *const *buf, int offset, void *const *recv,
                               int roff, const int *rc, int type, int op) {
  int esz = ora_type_size(type);
  int count = 0;
  for (int i = 0; i < P; i++) count += rc[i];
  jop *o = (jop *)calloc((size_t)P, sizeof(jop));
  char **tmp = (char **)calloc((size_t)P, sizeof(char *));
  char **msg = (char **)calloc((size_t)P, sizeof(char *));
  int *soffs = (int *)calloc((size_t)P, sizeof(int)), *roffs = (int *)calloc((size_t)P, sizeof(int));
  for (int r = 0; r < P; r++) {
    int prev = (r - 1 + P) % P;
    for (int i = 0; i < prev; i++) soffs[r] += rc[i];
    for (int i = 0; i < r; i++) roffs[r] += rc[i];
    jop_init(&o[r], op, type, flags, buf[r], offset, count, offset + count);
    tmp[r] = (char *)calloc((size_t)(count + offset + 1), (size_t)esz); /* createTemporaryBuffer */
    msg[r] = (char *)calloc((size_t)(count + 1), (size_t)esz);
  }
  for (int k = P - 2; k >= 0; k--) {
    for (int r = 0; r < P; r++) { /* isend(buf, isend_offset, recvcounts[prev], prev) */
      int prev = (r - 1 + P) % P;
      memcpy(msg[r], E(buf[r], soffs[r], esz), (size_t)rc[prev] * esz);
    }
    for (int r = 0; r < P; r++) { /* irecv(tmpbuf, irecv_offset, recvcounts[me], next).Wait() */
      int next = (r + 1) % P;
      memcpy(E(tmp[r], roffs[r], esz), msg[next], (size_t)rc[r] * esz);
      jop_perform(&o[r], tmp[r], offset, count);
      jop_result(&o[r], buf[r], offset, count);
    }
  }
  for (int r = 0; r < P; r++) {
    memcpy(E(recv[r], roff, esz), E(buf[r], roffs[r], esz), (size_t)rc[r] * esz);
    jop_free(&o[r]);
    free(tmp[r]);
    free(msg[r]);
  }
  free(o); free(tmp); free(msg); free(soffs); free(roffs);
}

int ora_reduce_scatter(int P, unsigned flags, void *const *send, int soff, void *const *recv, int roff,
                       const int *rc, int type, int op) {
  int c = ora_check(op, type);
  if (c) return c;
  int esz = ora_type_size(type);
  int count = 0;
  for (int i = 0; i < P; i++) count += rc[i];
  if ((flags & ORA_FLAG_FAITHFUL) && !is_pair(type)) {
    if (flags & ORA_FLAG_OLD) {
      /* FT_Reduce_scatter (:2441-2456) = Reduce(root 0) + FT_Scatter(:1132-1171) whose root strides
       * by its own sendcount = recvcounts[0] */
      ft_reduce(P, flags, send, soff, recv, roff, count, type, op, 0);
      char *tmp = (char *)malloc((size_t)(count + 1) * esz);
      memcpy(tmp, E(recv[0], roff, esz), (size_t)count * esz);
      for (int r = 0; r < P; r++) {
        int n = rc[r] < rc[0] ? rc[r] : rc[0];
        memcpy(E(recv[r], roff, esz), tmp + (size_t)r * rc[0] * esz, (size_t)n * esz);
      }
      free(tmp);
    } else {
      bkt_reduce_scatter(P, flags, send, soff, recv, roff, rc, type, op);
    }
    return 0;
  }
  void **w = scratch_from(P, send, soff, count, esz);
  if (flags & ORA_FLAG_OLD) {
    void **o = scratch_from(P, NULL, 0, count, esz);
    ft_reduce(P, flags, w, 0, o, 0, count, type, op, 0);
    int off = 0;
    for (int r = 0; r < P; r++) {
      memcpy(E(recv[r], roff, esz), E(o[0], off, esz), (size_t)rc[r] * esz);
      off += rc[r];
    }
    scratch_free(P, o);
  } else if (P <= 2 && !is_pair(type)) {
    bkt_reduce_scatter(P, flags, w, 0, recv, roff, rc, type, op);
  } else {
    /* MPI-correct replacement for the defective P >= 3 ring: block r of Reduce(root 0) (MST order) */
    mst_reduce(w, 0, count, type, op, flags, 0, 0, P - 1);
    int off = 0;
    for (int r = 0; r < P; r++) {
      memcpy(E(recv[r], roff, esz), E(w[0], off, esz), (size_t)rc[r] * esz);
      off += rc[r];
    }
  }
  scratch_free(P, w);
  return 0;
}

/* Scan (PureIntracomm.java:2526-2544): rank r starts from its own send, folds ranks 0..r-1 in order. */
int ora_scan(int P, unsigned flags, void *const *send, int soff, void *const *recv, int roff, int count,
             int type, int op) {
  int c = ora_check(op, type);
  if (c) return c;
  int esz = ora_type_size(type);
  for (int r = 0; r < P; r++) {
    jop o;
    jop_init(&o, op, type, flags, send[r], soff, count, maxi(soff, roff) + count);
    if (!(flags & ORA_FLAG_FAITHFUL) && soff != roff)
      memmove(E(o.arr, roff, esz), E(o.arr, soff, esz), (size_t)count * esz);
    for (int i = 0; i < r; i++) {
      memcpy(E(recv[r], roff, esz), E(send[i], soff, esz), (size_t)count * esz);
      jop_perform(&o, recv[r], roff, count);
    }
    jop_result(&o, recv[r], roff, count);
    jop_free(&o);
  }
  return 0;
}

/* ------------------------------------------------------------------------------------------- */
/* CPU baselines                                                                                 */

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}
static int cmp_d(const void *a, const void *b) {
  double x = *(const double *)a, y = *(const double *)b;
  return x < y ? -1 : x > y;
}
static double median(double *v, int n) {
  qsort(v, (size_t)n, sizeof(double), cmp_d);
  return v[n / 2];
}

static void fill_pattern(void *p, int64_t bytes, uint64_t seed) {
  uint64_t *q = (uint64_t *)p;
  for (int64_t i = 0; i < bytes / 8; i++) { /* splitmix64 -> doubles in [-1, 1) bit patterns */
    uint64_t z = (seed += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    double d = (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
    memcpy(&q[i], &d, 8);
  }
}

double ora_time_combine(int op, int type, int64_t n, int reps) {
  int esz = ora_type_size(type);
  if (!esz || reps < 1) return -1.0;
  char *in = (char *)malloc((size_t)n * esz), *buf = (char *)malloc((size_t)n * esz);
  char *arr = (char *)malloc((size_t)n * esz);
  fill_pattern(in, n * esz, 1);
  fill_pattern(buf, n * esz, 2);
  memset(arr, 0, (size_t)n * esz);
  double *t = (double *)malloc(sizeof(double) * (size_t)reps);
  for (int r = 0; r < reps; r++) {
    double t0 = now_s();
    memset(arr, 0, (size_t)n * esz);          /* new T[buf.length] (zeroed) */
    memcpy(arr, buf, (size_t)n * esz);        /* createInitialBuffer arraycopy */
    ora_apply(op, type, arr, in, 0, n);       /* perform loop */
    memcpy(buf, arr, (size_t)n * esz);        /* getResultant arraycopy */
    t[r] = now_s() - t0;
  }
  double m = median(t, reps);
  free(in); free(buf); free(arr); free(t);
  return m;
}

/* --- multicore Allreduce model: P threads, smpdev-style message copies, big-endian mpjbuf --- */

typedef struct {
  pthread_mutex_t mu;
  pthread_cond_t cv;
  const char *payload; /* sender's packed mpjbuf (big-endian) */
  int64_t bytes;
  int full, taken;
} mailbox;

typedef struct {
  int P, me, pin;
  int64_t n;
  int reps;
  double *times;
  mailbox *mb; /* [P*P], index dst*P + src */
  pthread_barrier_t *bar;
} ar_ctx;

static void bswap_copy64(char *dst, const char *src, int64_t n) { /* NIOBuffer big-endian put/get */
  const uint64_t *s = (const uint64_t *)src;
  uint64_t *d = (uint64_t *)dst;
  for (int64_t i = 0; i < n; i++) d[i] = __builtin_bswap64(s[i]);
}

static void mb_send(ar_ctx *c, int dst, const double *data, int64_t n, char *packbuf) {
  /* Comm.send: createWriteBuffer + SimplePackerDouble.pack -> NIOBuffer.write (big-endian) */
  memset(packbuf, 0, 8); /* section header: type code + count */
  bswap_copy64(packbuf + 8, (const char *)data, n);
  mailbox *m = &c->mb[dst * c->P + c->me];
  pthread_mutex_lock(&m->mu);
  m->payload = packbuf;
  m->bytes = n * 8 + 8;
  m->full = 1;
  m->taken = 0;
  pthread_cond_broadcast(&m->cv);
  while (!m->taken) pthread_cond_wait(&m->cv, &m->mu); /* blocking send */
  pthread_mutex_unlock(&m->mu);
}

static void mb_recv(ar_ctx *c, int src, double *data, int64_t n, char *rbuf) {
  mailbox *m = &c->mb[c->me * c->P + src];
  pthread_mutex_lock(&m->mu);
  while (!m->full) pthread_cond_wait(&m->cv, &m->mu);
  memcpy(rbuf, m->payload, (size_t)m->bytes); /* smpdev: ByteBuffer.put into the receiver's buffer */
  m->full = 0;
  m->taken = 1;
  pthread_cond_broadcast(&m->cv);
  pthread_mutex_unlock(&m->mu);
  bswap_copy64((char *)data, rbuf + 8, n); /* unpack: NIOBuffer.read */
}

static void mst_reduce_thr(ar_ctx *c, double *buf, double *arr, char *pk, char *rb, int root, int left,
                           int right) {
  if (left == right) return;
  int mid = (left + right) / 2, me = c->me;
  int srce = (root <= mid) ? right : left;
  if (me <= mid && root <= mid) mst_reduce_thr(c, buf, arr, pk, rb, root, left, mid);
  else if (me <= mid && root > mid) mst_reduce_thr(c, buf, arr, pk, rb, srce, left, mid);
  else if (me > mid && root <= mid) mst_reduce_thr(c, buf, arr, pk, rb, srce, mid + 1, right);
  else mst_reduce_thr(c, buf, arr, pk, rb, root, mid + 1, right);
  if (me == srce) mb_send(c, root, buf, c->n, pk);
  if (me == root) {
    memset(arr, 0, (size_t)c->n * 8);
    memcpy(arr, buf, (size_t)c->n * 8);
    mb_recv(c, srce, buf, c->n, rb);
    ora_apply(ORA_SUM, ORA_DOUBLE, arr, buf, 0, c->n);
    memcpy(buf, arr, (size_t)c->n * 8);
  }
}

static void mst_bcast_thr(ar_ctx *c, double *buf, char *pk, char *rb, int root, int left, int right) {
  if (left == right) return;
  int mid = (left + right) / 2, me = c->me;
  int dest = (root <= mid) ? right : left;
  if (me == root) mb_send(c, dest, buf, c->n, pk);
  if (me == dest) mb_recv(c, root, buf, c->n, rb);
  if (me <= mid && root <= mid) mst_bcast_thr(c, buf, pk, rb, root, left, mid);
  else if (me <= mid && root > mid) mst_bcast_thr(c, buf, pk, rb, dest, left, mid);
  else if (me > mid && root <= mid) mst_bcast_thr(c, buf, pk, rb, dest, mid + 1, right);
  else mst_bcast_thr(c, buf, pk, rb, root, mid + 1, right);
}

static void *ar_thread(void *arg) {
  ar_ctx *c = (ar_ctx *)arg;
  if (c->pin >= 0) {
    cpu_set_t allowed, one;
    CPU_ZERO(&allowed);
    sched_getaffinity(0, sizeof(allowed), &allowed);
    int k = -1, want = c->me;
    for (int cpu = 0; cpu < CPU_SETSIZE; cpu++)
      if (CPU_ISSET(cpu, &allowed) && ++k == want) {
        CPU_ZERO(&one);
        CPU_SET(cpu, &one);
        pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
        break;
      }
  }
  int64_t n = c->n;
  double *send = (double *)malloc((size_t)n * 8), *recv = (double *)malloc((size_t)n * 8);
  double *arr = (double *)malloc((size_t)n * 8);
  char *pk = (char *)malloc((size_t)n * 8 + 8), *rb = (char *)malloc((size_t)n * 8 + 8);
  fill_pattern(send, n * 8, 0x4D504A00ull + 1000 + c->me);
  memset(recv, 0, (size_t)n * 8);
  memset(arr, 0, (size_t)n * 8);
  memset(pk, 0, (size_t)n * 8 + 8);
  memset(rb, 0, (size_t)n * 8 + 8);
  for (int r = -1; r < c->reps; r++) { /* r = -1: warm-up */
    pthread_barrier_wait(c->bar);
    double t0 = now_s();
    memcpy(recv, send, (size_t)n * 8); /* Reduce: arraycopy send -> recv (:1937) */
    mst_reduce_thr(c, recv, arr, pk, rb, 0, 0, c->P - 1);
    mst_bcast_thr(c, recv, pk, rb, 0, 0, c->P - 1);
    pthread_barrier_wait(c->bar);
    if (r >= 0 && c->me == 0) c->times[r] = now_s() - t0;
  }
  free(send); free(recv); free(arr); free(pk); free(rb);
  return NULL;
}

double ora_time_allreduce_mst(int P, int64_t n, int reps, int pin_cores) {
  if (P < 1 || reps < 1) return -1.0;
  mailbox *mb = (mailbox *)calloc((size_t)P * P, sizeof(mailbox));
  for (int i = 0; i < P * P; i++) {
    pthread_mutex_init(&mb[i].mu, NULL);
    pthread_cond_init(&mb[i].cv, NULL);
  }
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)P);
  double *times = (double *)calloc((size_t)reps, sizeof(double));
  ar_ctx *cs = (ar_ctx *)calloc((size_t)P, sizeof(ar_ctx));
  pthread_t *th = (pthread_t *)calloc((size_t)P, sizeof(pthread_t));
  for (int r = 0; r < P; r++) {
    cs[r] = (ar_ctx){P, r, pin_cores ? 1 : -1, n, reps, times, mb, &bar};
    pthread_create(&th[r], NULL, ar_thread, &cs[r]);
  }
  for (int r = 0; r < P; r++) pthread_join(th[r], NULL);
  double m = median(times, reps);
  pthread_barrier_destroy(&bar);
  for (int i = 0; i < P * P; i++) {
    pthread_mutex_destroy(&mb[i].mu);
    pthread_cond_destroy(&mb[i].cv);
  }
  free(mb); free(times); free(cs); free(th);
  return m;
}
