/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see mpjx_oracle.h). Never linked into libmpjx.
 *
 * The application side of the reference's Java Grande Forum SparseMatmult benchmark, the one
 * reference-held double-precision result on the Allreduce(DOUBLE, SUM) path:
 *   test/jgf_mpj_benchmarks/section2/sparsematmult/JGFSparseMatmultBench.java
 *     :33           RANDOM_SEED = 10101010, one java.util.Random for all draws (:41)
 *     :35-37        size A: M = N = 50,000, nz = 250,000; SPARSE_NUM_ITER = 200 (:38)
 *     :73-80        per-rank share ceil(nz/P), remainder on the last rank
 *     :84,182-190   x[i] = R.nextDouble() * 1e-6, drawn first
 *     :104-124      then, for every nonzero in rank order: row = Math.abs(R.nextInt()) % M,
 *                   col = Math.abs(R.nextInt()) % N, val = R.nextDouble()
 *     :148-150      refval[A] = 75.02484945753453, |ytotal - refval| <= 1e-12
 *   test/jgf_mpj_benchmarks/section2/sparsematmult/SparseMatmult.java
 *     :239-247      200 reps of { p_y[row[i]] += x[col[i]] * val[i]  (p_y never reset);
 *                                 Allreduce(p_y, 0, y, 0, M, DOUBLE, SUM) }
 *     :255-259      ytotal = sum over i of y[buf_row[i]] (rank 0, all nz rows in draw order)
 *
 * java.util.Random is restated from its specification in the Java SE API documentation (the
 * reference ships no copy of it): a 48-bit LCG, seed' = seed * 0x5DEECE66D + 0xB mod 2^48,
 * scrambled at construction with 0x5DEECE66D; next(bits) = (int)(seed' >>> (48 - bits));
 * nextInt() = next(32); nextDouble() = ((long)next(26) << 27 | next(27)) * 2^-53.
 * Java's `%` truncates toward zero and Math.abs(Integer.MIN_VALUE) stays negative, which would
 * make the reference throw ArrayIndexOutOfBoundsException; ora_jgf_sparse_gen reports that as -1.
 *
 * Compiled with -ffp-contract=off: `p_y += x * val` is a rounded multiply then a rounded add in
 * Java, never a fused multiply-add.
 */
#include <stdint.h>

#include "mpjx_oracle.h"

#define JR_MULT 0x5DEECE66DULL
#define JR_ADD 0xBULL
#define JR_MASK ((1ULL << 48) - 1)

void ora_jrandom_seed(uint64_t *state, int64_t seed) { *state = ((uint64_t)seed ^ JR_MULT) & JR_MASK; }

static int32_t jr_next(uint64_t *s, int bits) {
  *s = (*s * JR_MULT + JR_ADD) & JR_MASK;
  return (int32_t)(uint32_t)(*s >> (48 - bits));
}

int32_t ora_jrandom_next_int(uint64_t *state) { return jr_next(state, 32); }

double ora_jrandom_next_double(uint64_t *state) {
  int64_t hi = (int64_t)jr_next(state, 26), lo = (int64_t)jr_next(state, 27);
  return (double)((hi << 27) + lo) * 0x1.0p-53;
}

/* Math.abs(int) % m with Java semantics (m > 0): truncating remainder, MIN_VALUE stays negative */
static int32_t java_abs_mod(int32_t v, int32_t m) {
  int32_t a = (v == INT32_MIN) ? v : (v < 0 ? -v : v);
  return a % m; /* C99 `%` truncates toward zero, as Java's does */
}

int ora_jgf_sparse_gen(int64_t seed, int M, int N, int nz, double *x, int32_t *row, int32_t *col,
                       double *val) {
  uint64_t s;
  ora_jrandom_seed(&s, seed);
  for (int i = 0; i < N; i++) x[i] = ora_jrandom_next_double(&s) * 1e-6; /* RandomVector */
  int bad = 0;
  /* the draw order is the same for every P: rank 0's share first, then ranks 1..P-1 in turn
   * (JGFSparseMatmultBench.java:104-124), i.e. nonzeros 0..nz-1 in index order */
  for (int i = 0; i < nz; i++) {
    row[i] = java_abs_mod(ora_jrandom_next_int(&s), M);
    col[i] = java_abs_mod(ora_jrandom_next_int(&s), N);
    val[i] = ora_jrandom_next_double(&s);
    if (row[i] < 0 || col[i] < 0) bad = 1;
  }
  return bad ? -1 : 0;
}

void ora_jgf_sparse_rep(double *p_y, const double *x, const int32_t *row, const int32_t *col,
                        const double *val, int lo, int hi) {
  for (int i = lo; i < hi; i++) p_y[row[i]] += x[col[i]] * val[i]; /* SparseMatmult.java:241-244 */
}

double ora_jgf_ytotal(const double *y, const int32_t *row, int nz) {
  double t = 0.0;
  for (int i = 0; i < nz; i++) t += y[row[i]]; /* SparseMatmult.java:256-258 */
  return t;
}
