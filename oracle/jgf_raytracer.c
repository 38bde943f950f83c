/*
 * jgf_raytracer.c — ORACLE (test infrastructure only; never linked into libmpjx).
 *
 * Restatement of the reference's JGF RayTracer benchmark (test/jgf_mpj_benchmarks/section3/raytracer/,
 * MPJ Version 1.0 of the Java Grande Forum suite), the one application in the reference's test tree
 * that ends in a Reduce on DOUBLE (not an Allreduce) checked EXACTLY:
 *   RayTracer.java:275-279   tmp_checksum[0] = (double) checksum;
 *                            MPI.COMM_WORLD.Reduce(tmp_checksum,0,tmp_checksum,0,1,MPI.DOUBLE,MPI.SUM,0);
 *                            rank 0: checksum = (long) tmp_checksum[0];
 *   JGFRayTracerBench.java:87-88  refval = {2676692, 29827635} for sizes A (150 x 150), B (500 x 500).
 * Every rank's partial checksum is an integer below 2^53, so the Reduce is exact in any combine order:
 * rank 0 must hold refval at every P.
 *
 * Followed line by line (file:line in the reference's raytracer directory):
 *   scene        RayTracer.java:102-161 (4x4x4 spheres of radius 3, colour (0, 0, (i+j)/6), shine 15,
 *                ks = kt = 1.5 - 1.0; five lights; view from (0,20,-30) at (0,0,0), up (0,1,0),
 *                dist 1, angle 35*3.14159265/180, aspect 1); Surface.java defaults (kd 1, ior 1)
 *   render       RayTracer.java:187-271: rows y = rank, rank + P, ... (:240); per pixel the ray
 *                direction comb(xlen, leftVec, ylen, upVec) + viewVec, normalised; colour channels
 *                (int)(c * 255.0) clamped at 255 (Java's saturating double->int cast), summed
 *   intersect    RayTracer.java:302-320 (the global Isect `inter`: t reset to 1e9, fields replaced on
 *                every closer hit); Sphere.java intersect/normal
 *   shadow       RayTracer.java:327-331 (ANY hit blocks: the tmax argument is unused)
 *   shade        RayTracer.java:368-433, trace :438-458, SpecularDirection :338-343, TransDir :348-361
 *   Vec          Vec.java (every expression in Java's left-to-right order; no FMA contraction: build
 *                with -ffp-contract=off)
 * Java reference semantics that change results are kept: the one global temporary ray `tRay` is
 * shared by every recursion level, so the transmission ray of a shade() call starts at whatever point
 * the nested specular trace() left in tRay.P (RayTracer.java:413-425), not necessarily at this hit's P.
 * The other shared temporaries (L, inter, each Sphere's v) are rewritten before every read that
 * matters, and `hit.enter` selects between two TransDir calls that are identical for ior = 1; they are
 * modelled as Java has them anyway. No state crosses pixels, so a row's checksum does not depend on
 * which rank renders it; the per-rank partial is the sum of its rows (:240, :262-264).
 * Math.sqrt is IEEE-exact; Math.tan and Math.pow are the C library's (Java allows them 1 ulp; the
 * channels are truncated to integers, and refval is met exactly — tests/test_oracle.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "mpjx_oracle.h"

typedef struct {
  double x, y, z;
} Vec;

static Vec vec(double a, double b, double c) {
  Vec v = {a, b, c};
  return v;
}
static Vec vsub(Vec a, Vec b) { return vec(a.x - b.x, a.y - b.y, a.z - b.z); }
static double vdot(Vec a, Vec b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static Vec vcross(Vec a, Vec b) { return vec(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static Vec vcomb(double a, Vec A, double b, Vec B) {
  return vec(a * A.x + b * B.x, a * A.y + b * B.y, a * A.z + b * B.z);
}
static void vscale(Vec* v, double t) {
  v->x *= t;
  v->y *= t;
  v->z *= t;
}
static void vadd(Vec* v, Vec a) {
  v->x += a.x;
  v->y += a.y;
  v->z += a.z;
}
static void vadds(Vec* v, double s, Vec b) {  // Vec.adds(double, Vec): x += s * b.x
  v->x += s * b.x;
  v->y += s * b.y;
  v->z += s * b.z;
}
static double vnormalize(Vec* v) {  // Vec.normalize: returns the length before normalising
  const double len = sqrt(v->x * v->x + v->y * v->y + v->z * v->z);
  if (len > 0.0) {
    v->x /= len;
    v->y /= len;
    v->z /= len;
  }
  return len;
}

typedef struct {
  Vec color;
  double kd, ks, shine, kt, ior;
} Surface;

typedef struct {
  Vec c;
  double r, r2;
  Surface surf;
} Sphere;

typedef struct {
  double t;
  int enter;
  const Sphere* prim;
  const Surface* surf;
} Isect;

typedef struct {
  Vec pos;
  double brightness;
} Light;

enum { NSPH = 64, NLIGHT = 5 };

typedef struct {
  Sphere prim[NSPH];
  Light lights[NLIGHT];
  Vec from, at, up;
  double dist, angle, aspect;
  Isect inter;     /* RayTracer.inter: ONE Isect for every intersect() */
  Vec tRayP, tRayD; /* RayTracer.tRay: ONE temporary ray shared by every recursion level */
} Tracer;

/* RayTracer.createScene (:102-161) */
static void create_scene(Tracer* T) {
  const int nx = 4, ny = 4, nz = 4;
  int o = 0;
  for (int i = 0; i < nx; i++)
    for (int j = 0; j < ny; j++)
      for (int k = 0; k < nz; k++) {
        const double xx = 20.0 / (nx - 1) * i - 10.0;
        const double yy = 20.0 / (ny - 1) * j - 10.0;
        const double zz = 20.0 / (nz - 1) * k - 10.0;
        Sphere* p = &T->prim[o++];
        p->c = vec(xx, yy, zz);
        p->r = 3;
        p->r2 = p->r * p->r;
        /* Surface() defaults (Surface.java), then setColor and the three assignments */
        p->surf.kd = 1.0;
        p->surf.ior = 1.0;
        p->surf.color = vec(0, 0, (i + j) / (double)(nx + ny - 2));
        p->surf.shine = 15.0;
        p->surf.ks = 1.5 - 1.0;
        p->surf.kt = 1.5 - 1.0;
      }
  const double lp[NLIGHT][3] = {{100, 100, -50}, {-100, 100, -50}, {100, -100, -50}, {-100, -100, -50}, {200, 200, 0}};
  for (int l = 0; l < NLIGHT; l++) {
    T->lights[l].pos = vec(lp[l][0], lp[l][1], lp[l][2]);
    T->lights[l].brightness = 1.0;
  }
  T->from = vec(0, 20, -30);
  T->at = vec(0, 0, 0);
  T->up = vec(0, 1, 0);
  T->dist = 1.0;
  T->angle = 35.0 * 3.14159265 / 180.0;
  T->aspect = 1.0;
  T->inter.t = 0;
  T->inter.enter = 0;
  T->inter.prim = NULL;
  T->inter.surf = NULL;
  T->tRayP = vec(0, 0, 0);
  T->tRayD = vec(0, 0, 0);
}

/* Sphere.intersect: 1 and *ip filled on a hit (Java returns a new Isect), 0 for null */
static int sphere_intersect(const Sphere* s, Vec P, Vec D, Isect* ip) {
  const Vec v = vsub(s->c, P);
  const double b = vdot(v, D);
  double disc = b * b - vdot(v, v) + s->r2;
  if (disc < 0.0) return 0;
  disc = sqrt(disc);
  const double t = (b - disc < 1e-6) ? b + disc : b - disc;
  if (t < 1e-6) return 0;
  ip->t = t;
  ip->enter = vdot(v, v) > s->r2 + 1e-6 ? 1 : 0;
  ip->prim = s;
  ip->surf = &s->surf;
  return 1;
}

/* RayTracer.intersect (:302-320): the global inter keeps its old prim/surf/enter when nothing hits */
static int intersect(Tracer* T, Vec P, Vec D) {
  int nhits = 0;
  T->inter.t = 1e9;
  for (int i = 0; i < NSPH; i++) {
    Isect tp;
    if (sphere_intersect(&T->prim[i], P, D, &tp) && tp.t < T->inter.t) {
      T->inter.t = tp.t;
      T->inter.prim = tp.prim;
      T->inter.surf = tp.surf;
      T->inter.enter = tp.enter;
      nhits++;
    }
  }
  return nhits > 0;
}

static Vec specular_direction(Vec I, Vec N) {  /* :338-343 */
  Vec r = vcomb(1.0 / fabs(vdot(I, N)), I, 2.0, N);
  vnormalize(&r);
  return r;
}

static Vec trans_dir(const Surface* m1, const Surface* m2, Vec I, Vec N) {  /* :348-361 (never null: ior 1) */
  const double n1 = m1 == NULL ? 1.0 : m1->ior;
  const double n2 = m2 == NULL ? 1.0 : m2->ior;
  const double eta = n1 / n2;
  const double c1 = -vdot(I, N);
  const double cs2 = 1.0 - eta * eta * (1.0 - c1 * c1);
  Vec r = vcomb(eta, I, eta * c1 - sqrt(cs2), N);
  vnormalize(&r);
  return r;
}

static Vec trace(Tracer* T, int level, double weight, Vec rP, Vec rD);

/* RayTracer.shade (:368-433); `hit` is the global inter, read where Java reads it */
static Vec shade(Tracer* T, int level, double weight, Vec P, Vec N, Vec I) {
  Vec col = vec(0, 0, 0), R = vec(0, 0, 0);
  const Surface* surf = T->inter.surf;
  if (surf->shine > 1e-6) R = specular_direction(I, N);
  for (int l = 0; l < NLIGHT; l++) {
    Vec L = vsub(T->lights[l].pos, P); /* the shared temporary RayTracer.L */
    if (vdot(N, L) >= 0.0) {
      const double t = vnormalize(&L);
      (void)t;  /* Shadow's tmax: unused by the reference (:327-331) */
      T->tRayP = P;
      T->tRayD = L;
      if (!intersect(T, T->tRayP, T->tRayD)) { /* Shadow(tRay, t) > 0 */
        const double diff = vdot(N, L) * surf->kd * T->lights[l].brightness;
        vadds(&col, diff, surf->color);
        if (surf->shine > 1e-6) {
          double spec = vdot(R, L);
          if (spec > 1e-6) {
            spec = pow(spec, surf->shine);
            col.x += spec;
            col.y += spec;
            col.z += spec;
          }
        }
      }
    }
  }
  T->tRayP = P;
  if (surf->ks * weight > 1e-3) {
    T->tRayD = specular_direction(I, N);
    const Vec tcol = trace(T, level + 1, surf->ks * weight, T->tRayP, T->tRayD);
    vadds(&col, surf->ks, tcol);
  }
  if (surf->kt * weight > 1e-3) {
    /* hit.enter: the global inter as the shadow rays and the nested trace left it */
    if (T->inter.enter > 0) T->tRayD = trans_dir(NULL, surf, I, N);
    else T->tRayD = trans_dir(surf, NULL, I, N);
    /* tRay.P: still this hit's P only if the nested specular trace did not move it (:413, :391) */
    const Vec tcol = trace(T, level + 1, surf->kt * weight, T->tRayP, T->tRayD);
    vadds(&col, surf->kt, tcol);
  }
  return col;
}

/* RayTracer.trace (:438-458) */
static Vec trace(Tracer* T, int level, double weight, Vec rP, Vec rD) {
  if (level > 6) return vec(0, 0, 0);
  if (intersect(T, rP, rD)) {
    const Vec P = vec(rP.x + rD.x * T->inter.t, rP.y + rD.y * T->inter.t, rP.z + rD.z * T->inter.t); /* Ray.point */
    Vec N = vsub(P, T->inter.prim->c); /* Sphere.normal */
    vnormalize(&N);
    if (vdot(rD, N) >= 0.0) N = vec(-N.x, -N.y, -N.z);
    return shade(T, level, weight, P, N, rD);
  }
  return vec(0, 0, 0); /* voidVec */
}

/* Java's (int) cast of a double: NaN -> 0, saturating at the int range, else truncation */
static int32_t java_d2i(double d) {
  if (d != d) return 0;
  if (d >= 2147483647.0) return INT32_MAX;
  if (d <= -2147483648.0) return INT32_MIN;
  return (int32_t)d;
}

/* The checksum contribution (red + green + blue, RayTracer.java:252-264) of every row of the
 * size x size picture into rows[0..size): the render loop (:210-271) over each row in turn. */
int ora_jgf_raytracer_rows(int size, int64_t* rows) {
  if (size <= 0 || !rows) return -1;
  Tracer* T = (Tracer*)calloc(1, sizeof(Tracer));
  if (!T) return -1;
  create_scene(T);
  const int width = size;
  Vec viewVec = vsub(T->at, T->from);
  vnormalize(&viewVec);
  Vec tmpVec = viewVec;
  vscale(&tmpVec, vdot(T->up, viewVec));
  Vec upVec = vsub(T->up, tmpVec);
  vnormalize(&upVec);
  Vec leftVec = vcross(T->up, viewVec);
  vnormalize(&leftVec);
  const double frustrumwidth = T->dist * tan(T->angle);
  vscale(&upVec, -frustrumwidth);
  vscale(&leftVec, T->aspect * frustrumwidth);
  const Vec rP = T->from; /* new Ray(view.from, voidVec): P copied, never moved */
  for (int y = 0; y < size; y++) {
    const double ylen = (double)(2.0 * y) / (double)width - 1.0;
    int64_t sum = 0;
    for (int x = 0; x < width; x++) {
      const double xlen = (double)(2.0 * x) / (double)width - 1.0;
      Vec D = vcomb(xlen, leftVec, ylen, upVec);
      vadd(&D, viewVec);
      vnormalize(&D);
      const Vec col = trace(T, 0, 1.0, rP, D);
      int32_t red = java_d2i(col.x * 255.0);
      if (red > 255) red = 255;
      int32_t green = java_d2i(col.y * 255.0);
      if (green > 255) green = 255;
      int32_t blue = java_d2i(col.z * 255.0);
      if (blue > 255) blue = 255;
      sum += red;
      sum += green;
      sum += blue;
    }
    rows[y] = sum;
  }
  free(T);
  return 0;
}

/* Rank `rank`'s partial checksum at P ranks: its rows y = rank, rank + P, ... (RayTracer.java:240). */
int64_t ora_jgf_raytracer_partial(const int64_t* rows, int size, int rank, int P) {
  int64_t s = 0;
  for (int y = rank; y < size; y += P) s += rows[y];
  return s;
}
