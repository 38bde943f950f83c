/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C) of the MPJ Express 0.44 reduction path: the typed element-wise
 * Op classes and the pure-Java collective algorithms of src/mpi/PureIntracomm.java. It is the
 * checker the parity tests compare the HIP path against, and the CPU baseline bench.py times.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product
 * library (libmpjx) never links, calls or falls back to it.
 *
 * Parity pinning: the reference is Java and no JVM exists in this image, so the reference itself
 * cannot be run. The oracle is pinned by the reference's own known-answer tests
 * (test/mpi/ccl/{allreduce,reduce,reduce2,scan,reduce_scatter}.java, restated as fixtures under
 * tests/golden/) for INT SUM/PROD; every other (op, type) row is pinned by source reading only
 * (see DESIGN.md "Parity").
 */
#ifndef MPJX_ORACLE_H
#define MPJX_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* mpi.Datatype base types, src/mpi/Datatype.java:57-66 */
enum { ORA_BYTE = 1, ORA_CHAR = 2, ORA_SHORT = 3, ORA_BOOLEAN = 4, ORA_INT = 5, ORA_LONG = 6,
       ORA_FLOAT = 7, ORA_DOUBLE = 8 };
/* mpjdev.Constants op codes, src/mpjdev/Constants.java:53-62 */
enum { ORA_MAX = 1, ORA_MIN = 2, ORA_SUM = 3, ORA_PROD = 4, ORA_LAND = 5, ORA_BAND = 6,
       ORA_LOR = 7, ORA_BOR = 8, ORA_LXOR = 9, ORA_BXOR = 10, ORA_MAXLOC = 11, ORA_MINLOC = 12 };
/* (value, index) pair types MPI.SHORT2..DOUBLE2 = Datatype.Contiguous(2, base), src/mpi/MPI.java:110-114 */
enum { ORA_SHORT2 = 0x103, ORA_INT2 = 0x105, ORA_LONG2 = 0x106, ORA_FLOAT2 = 0x107, ORA_DOUBLE2 = 0x108 };

/* flags */
#define ORA_FLAG_OLD      1u /* conf mpjexpress.mpi.old.collectives=true (MPI.isOldSelected) */
#define ORA_FLAG_FAITHFUL 2u /* reproduce the reference's observable defects */

int ora_type_size(int type);
/* 0 = valid, 1 = worker throws MPIException, 2 = no worker (unknown type) */
int ora_check(int op, int type);

/* acc[i] = in[i] (op) acc[i] for i in [lo, hi): the body of the typed perform() loop */
void ora_apply(int op, int type, void *acc, const void *in, int64_t lo, int64_t hi);

/*
 * Collectives over P simulated ranks (pointer arrays indexed by rank). Offsets and counts are in
 * elements, as in the mpiJava API. Without ORA_FLAG_FAITHFUL the MPI-semantics result is produced
 * (correct offsets, BOR/BXOR applied, correct Reduce_scatter for P >= 3), with the reference's
 * combine ORDER kept. Returns 0 or the ora_check() code.
 */
int ora_reduce(int P, unsigned flags, void *const *send, int soff, void *const *recv, int roff,
               int count, int type, int op, int root);
int ora_allreduce(int P, unsigned flags, void *const *send, int soff, void *const *recv, int roff,
                  int count, int type, int op);
int ora_reduce_scatter(int P, unsigned flags, void *const *send, int soff, void *const *recv,
                       int roff, const int *recvcounts, int type, int op);
int ora_scan(int P, unsigned flags, void *const *send, int soff, void *const *recv, int roff,
             int count, int type, int op);
int ora_bcast(int P, unsigned flags, void *const *buf, int off, int count, int type, int root);

/*
 * CPU baselines (timed restatements of the reference's host cost structure).
 * ora_time_combine: one Op.perform round trip on the host as the typed class does it —
 *   createInitialBuffer (new T[len] + arraycopy), perform loop, getResultant arraycopy
 *   (src/mpi/SumDouble.java:49-67) — over n elements; returns seconds per call (median).
 * ora_time_allreduce_mst: Allreduce = MST_Reduce(root 0) + MST_Broadcast with P ranks as P
 *   threads (multicore/smpdev mode), every hop paying mpjbuf pack + unpack with big-endian
 *   byte swap (src/mpjbuf/NIOBuffer.java:42,520-563); returns seconds per Allreduce (median).
 */
double ora_time_combine(int op, int type, int64_t n, int reps);
double ora_time_allreduce_mst(int P, int64_t n, int reps, int pin_cores);

/*
 * JGF SparseMatmult (oracle/jgf_sparsematmult.c): java.util.Random restated from the Java API
 * specification, the benchmark's input generation in draw order, one rep of its per-rank sparse
 * product and its ytotal check sum. Returns -1 from ora_jgf_sparse_gen if a drawn index would be
 * negative (the reference would throw).
 */
void ora_jrandom_seed(uint64_t *state, int64_t seed);
int32_t ora_jrandom_next_int(uint64_t *state);
double ora_jrandom_next_double(uint64_t *state);
int ora_jgf_sparse_gen(int64_t seed, int M, int N, int nz, double *x, int32_t *row, int32_t *col,
                       double *val);
void ora_jgf_sparse_rep(double *p_y, const double *x, const int32_t *row, const int32_t *col,
                        const double *val, int lo, int hi);
double ora_jgf_ytotal(const double *y, const int32_t *row, int nz);

/*
 * JGF MolDyn (oracle/jgf_moldyn.c): one simulated rank's particle state. Per move: ora_md_forces
 * (move + this rank's cyclic share of the forces -> partial forces, epot/vir, interaction count),
 * the caller's in-place Allreduce(SUM) of those, ora_md_finish (the rest of the move). size 0 = A.
 */
typedef struct ora_md ora_md;
ora_md *ora_md_new(int size);
void ora_md_free(ora_md *m);
int ora_md_mdsize(const ora_md *m);
void ora_md_forces(ora_md *m, int rank, int P, double *xf, double *yf, double *zf, double *ev, int32_t *inter);
void ora_md_finish(ora_md *m, const double *xf, const double *yf, const double *zf, const double *ev,
                   int32_t inter);
double ora_md_ek(const ora_md *m);
int32_t ora_md_interactions(const ora_md *m);
int ora_md_moves(void);
/* StrictMath.log (fdlibm 5.3 __ieee754_log) as restated in jgf_moldyn.c */
double ora_java_log(double x);


/* JGF RayTracer (oracle/jgf_raytracer.c): the checksum contribution of every row of the size x size
 * picture (rows[0..size)), and rank `rank`'s partial at P ranks (rows rank, rank + P, ...), the value
 * each rank feeds to the reference's in-place Reduce(DOUBLE, SUM, root 0) (RayTracer.java:275-279). */
int ora_jgf_raytracer_rows(int size, int64_t *rows);
int64_t ora_jgf_raytracer_partial(const int64_t *rows, int size, int rank, int P);

#ifdef __cplusplus
}
#endif
#endif
