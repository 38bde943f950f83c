/*
 * ORACLE CROSS-CHECK — TEST INFRASTRUCTURE ONLY (this container; never shipped or linked into libmpjx).
 *
 * Runs MPICH's MPI_Allreduce / MPI_Reduce / MPI_Reduce_scatter / MPI_Scan on seeded integer and
 * logical data for the ops whose results do not depend on combine order (integer SUM/PROD/MAX/MIN
 * and the bitwise/logical ops, all wrapping or exact), so the oracle's MPI-semantics mode can be
 * checked against an independent MPI implementation — MPICH is also the arithmetic behind the
 * reference's `native` device (src/mpjdev/natmpjdev/lib/mpjdev_natmpjdev_Intracomm.c:428-516).
 * Java types map to byte=MPI_INT8_T, short=MPI_INT16_T, char=MPI_UINT16_T, int=MPI_INT32_T,
 * long=MPI_INT64_T, boolean=MPI_UINT8_T (0/1).
 *
 * usage: mpiexec -n P mpich_xcheck <outdir> <n>
 * writes <outdir>/in_<rank>_<case>.bin and <outdir>/<coll>_<rank>_<case>.bin
 */
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t sm(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

typedef struct { const char *name; int jtype; MPI_Datatype dt; int esz; } T;
typedef struct { const char *name; int code; MPI_Op op; } O;

static void dump(const char *dir, const char *what, int rank, const char *cname, const void *p, size_t bytes) {
  char path[512];
  snprintf(path, sizeof path, "%s/%s_%d_%s.bin", dir, what, rank, cname);
  FILE *f = fopen(path, "wb");
  if (!f) { perror(path); MPI_Abort(MPI_COMM_WORLD, 2); }
  fwrite(p, 1, bytes, f);
  fclose(f);
}

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int rank, P;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &P);
  const char *dir = argv[1];
  const int n = atoi(argv[2]);  /* multiple of P */
  T types[] = {{"BYTE", 1, MPI_INT8_T, 1}, {"CHAR", 2, MPI_UINT16_T, 2}, {"SHORT", 3, MPI_INT16_T, 2},
               {"INT", 5, MPI_INT32_T, 4}, {"LONG", 6, MPI_INT64_T, 8}, {"BOOLEAN", 4, MPI_UINT8_T, 1}};
  O ops[] = {{"MAX", 1, MPI_MAX}, {"MIN", 2, MPI_MIN}, {"SUM", 3, MPI_SUM}, {"PROD", 4, MPI_PROD},
             {"BAND", 6, MPI_BAND}, {"BOR", 8, MPI_BOR}, {"BXOR", 10, MPI_BXOR},
             {"LAND", 5, MPI_LAND}, {"LOR", 7, MPI_LOR}, {"LXOR", 9, MPI_LXOR}};
  int *rc = (int *)malloc(sizeof(int) * P);
  for (int j = 0; j < P; j++) rc[j] = n / P;
  for (size_t ti = 0; ti < sizeof types / sizeof *types; ti++) {
    for (size_t oi = 0; oi < sizeof ops / sizeof *ops; oi++) {
      const T *t = &types[ti];
      const O *o = &ops[oi];
      const int logical = (o->code == 5 || o->code == 7 || o->code == 9);
      if (logical != (t->jtype == 4)) continue; /* the reference's worker table */
      char cname[64];
      snprintf(cname, sizeof cname, "%s_%s", o->name, t->name);
      size_t bytes = (size_t)n * t->esz;
      unsigned char *in = malloc(bytes), *out = malloc(bytes), *rs = malloc(bytes / P + 8);
      uint64_t s = 0x4D504A00ull + 77 * ti + 1000 * oi + rank;
      for (size_t i = 0; i < bytes; i++) in[i] = (unsigned char)sm(&s);
      if (t->jtype == 4) for (int i = 0; i < n; i++) in[i] &= 1;
      if (o->code == 4) /* PROD: small magnitudes so products of P values stay interesting */
        for (int i = 0; i < n; i++) { if (t->esz == 1) in[i] = (unsigned char)(in[i] % 5); }
      dump(dir, "in", rank, cname, in, bytes);
      MPI_Allreduce(in, out, n, t->dt, o->op, MPI_COMM_WORLD);
      dump(dir, "allreduce", rank, cname, out, bytes);
      memset(out, 0, bytes);
      MPI_Reduce(in, out, n, t->dt, o->op, P / 2, MPI_COMM_WORLD);
      if (rank == P / 2) dump(dir, "reduce", rank, cname, out, bytes);
      MPI_Scan(in, out, n, t->dt, o->op, MPI_COMM_WORLD);
      dump(dir, "scan", rank, cname, out, bytes);
      MPI_Reduce_scatter(in, rs, rc, t->dt, o->op, MPI_COMM_WORLD);
      dump(dir, "rs", rank, cname, rs, bytes / P);
      free(in); free(out); free(rs);
    }
  }
  free(rc);
  MPI_Finalize();
  return 0;
}
