/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see mpjx_oracle.h). Never linked into libmpjx.
 *
 * The application side of the reference's Java Grande Forum MolDyn benchmark, whose every time step
 * ends in in-place Allreduce(DOUBLE, SUM) calls of the per-rank partial forces (and of the potential
 * energy, the virial and an INT interaction count):
 *   test/jgf_mpj_benchmarks/section3/moldyn/md.java
 *     :37-76       constants; size A: mm = 8, mdsize = 4 mm^3 = 2048 particles; movemx = 50 moves
 *     :81-216      initialise(): fcc lattice, velocities from the benchmark's own `random` class
 *                  (:475-532, a Park-Miller 16807 generator and a polar Box-Muller), velocity scaling
 *     :220-318     runiters(): domove, the rank's cyclic share of force() (i = rank, rank + P, ...),
 *                  Allreduce of x/y/z forces (:248-250), epot, vir (:262-263), interactions (:264,
 *                  INT, never reset — it wraps), mkekin, velavg, temperature scaling, ek every 10 moves
 *     :321-470     class particle: domove, force (pairs i < j within rcoff, minimum image), mkekin,
 *                  velavg, dscal
 *   test/jgf_mpj_benchmarks/section3/moldyn/JGFMolDynBench.java:72-73
 *                  refval[A] = 1731.4306625334357, |ek - refval| <= 1e-12
 *
 * One state per simulated rank (each rank of the reference holds the whole particle set and repeats
 * every step; the statics epot/vir/interactions/count are per rank: every multicore rank thread
 * loads its own copy of the classes). The Allreduce between md_forces() and md_finish() is the
 * caller's — the oracle's restatement in CPU tests, libmpjx in the GPU tests.
 * Compiled with -ffp-contract=off (Java never fuses a multiply-add). Math.sqrt is IEEE sqrt. Math.log
 * is restated as fdlibm's __ieee754_log (java_log below; StrictMath.log is specified as fdlibm 5.3):
 * glibc's log rounds 208 of the 3,072 Box-Muller arguments of size A differently, and with it the
 * chaotic trajectory ends 9 ulps from refval; with fdlibm's the final ek IS refval, for A and for B.
 * Math.pow is called once (the box side); the C library's result gives refval there.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "mpjx_oracle.h"

typedef struct {
  double x, y, z, vx, vy, vz, fx, fy, fz;
} particle;

struct ora_md {
  int mm, mdsize, move;
  double side, rcoff, hsq, hsq2, tscale, vaverh, h, tref, den;
  double epot, vir, count, ekin, ek, vel;
  int32_t interactions;
  particle *one;
};

/* fdlibm 5.3 e_log.c (__ieee754_log), the algorithm java.lang.StrictMath.log is specified by: x =
 * 2^k (1 + f) with sqrt(2)/2 < 1 + f < sqrt(2), log(1 + f) = f - s (f - R) with s = f / (2 + f) and R a
 * degree-14 minimax polynomial in s (Lg1..Lg7), k ln2 split into ln2_hi + ln2_lo. Restated for
 * finite positive arguments (every call here has 0 < x < 1). */
static double java_log(double x) {
  static const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                      two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
                      Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                      Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
                      Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
  uint64_t u;
  memcpy(&u, &x, 8);
  int32_t hx = (int32_t)(u >> 32), k = 0;
  if (hx < 0x00100000) { /* subnormal: scale up */
    k -= 54;
    x *= two54;
    memcpy(&u, &x, 8);
    hx = (int32_t)(u >> 32);
  }
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  int32_t i = (hx + 0x95f64) & 0x100000;
  u = (u & 0xffffffffull) | ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32); /* normalize x or x/2 */
  memcpy(&x, &u, 8);
  k += (i >> 20);
  const double f = x - 1.0;
  double dk, R;
  if ((0x000fffff & (2 + hx)) < 3) { /* |f| < 2^-20 */
    if (f == 0.0) {
      if (k == 0) return 0.0;
      dk = (double)k;
      return dk * ln2_hi + dk * ln2_lo;
    }
    R = f * f * (0.5 - 0.33333333333333333 * f);
    if (k == 0) return f - R;
    dk = (double)k;
    return dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  const double s = f / (2.0 + f);
  dk = (double)k;
  const double z = s * s;
  i = hx - 0x6147a;
  const double w = z * z;
  const int32_t j = 0x6b851 - hx;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  i |= j;
  R = t2 + t1;
  if (i > 0) {
    const double hfsq = 0.5 * f * f;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  if (k == 0) return f - s * (f - R);
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

double ora_java_log(double x) { return java_log(x); }

/* class random (md.java:475-532): iseed as a Java int, all arithmetic in int */
typedef struct {
  int32_t iseed;
  double v1, v2;
} md_random;

static double md_update(md_random *r) {
  const double scale = 4.656612875e-10;
  const int32_t imult = 16807, imod = 2147483647;
  if (r->iseed <= 0) r->iseed = 1;
  int32_t is2 = r->iseed % 32768;
  int32_t is1 = (r->iseed - is2) / 32768;
  int32_t iss2 = is2 * imult; /* < 2^31: no overflow */
  is2 = iss2 % 32768;
  is1 = (int32_t)(((int64_t)is1 * imult + (iss2 - is2) / 32768) % 65536);
  r->iseed = (is1 * 32768 + is2) % imod;
  return scale * r->iseed;
}

static double md_seed(md_random *r) {
  double s = 1.0, u1, u2;
  do {
    u1 = md_update(r);
    u2 = md_update(r);
    r->v1 = 2.0 * u1 - 1.0;
    r->v2 = 2.0 * u2 - 1.0;
    s = r->v1 * r->v1 + r->v2 * r->v2;
  } while (s >= 1.0);
  return sqrt(-2.0 * java_log(s) / s); /* Math.log = fdlibm */
}

ora_md *ora_md_new(int size) {
  static const int datasizes[] = {8, 13};
  if (size < 0 || size > 1) return NULL;
  ora_md *m = (ora_md *)calloc(1, sizeof *m);
  m->mm = datasizes[size];
  m->mdsize = m->mm * m->mm * m->mm * 4;
  m->one = (particle *)calloc((size_t)m->mdsize, sizeof(particle));
  m->den = 0.83134;
  m->tref = 0.722;
  m->h = 0.064;
  const int mm = m->mm, mdsize = m->mdsize;
  m->side = pow(mdsize / m->den, 0.3333333);
  m->rcoff = mm / 4.0;
  const double a = m->side / mm;
  m->hsq = m->h * m->h;
  m->hsq2 = m->hsq * 0.5;
  m->tscale = 16.0 / (1.0 * mdsize - 1.0);
  const double vaver = 1.13 * sqrt(m->tref / 24.0);
  m->vaverh = vaver * m->h;
  int ijk = 0;
  for (int lg = 0; lg <= 1; lg++)
    for (int i = 0; i < mm; i++)
      for (int j = 0; j < mm; j++)
        for (int k = 0; k < mm; k++) {
          particle *p = &m->one[ijk++];
          p->x = i * a + lg * a * 0.5;
          p->y = j * a + lg * a * 0.5;
          p->z = k * a;
        }
  for (int lg = 1; lg <= 2; lg++)
    for (int i = 0; i < mm; i++)
      for (int j = 0; j < mm; j++)
        for (int k = 0; k < mm; k++) {
          particle *p = &m->one[ijk++];
          p->x = i * a + (2 - lg) * a * 0.5;
          p->y = j * a + (lg - 1) * a * 0.5;
          p->z = k * a + a * 0.5;
        }
  md_random rnd = {0, 0.0, 0.0};
  for (int i = 0; i < mdsize; i += 2) {
    double r = md_seed(&rnd);
    m->one[i].vx = r * rnd.v1;
    m->one[i + 1].vx = r * rnd.v2;
  }
  for (int i = 0; i < mdsize; i += 2) {
    double r = md_seed(&rnd);
    m->one[i].vy = r * rnd.v1;
    m->one[i + 1].vy = r * rnd.v2;
  }
  for (int i = 0; i < mdsize; i += 2) {
    double r = md_seed(&rnd);
    m->one[i].vz = r * rnd.v1;
    m->one[i + 1].vz = r * rnd.v2;
  }
  double ekin = 0.0, sp = 0.0;
  for (int i = 0; i < mdsize; i++) sp = sp + m->one[i].vx;
  sp = sp / mdsize;
  for (int i = 0; i < mdsize; i++) {
    m->one[i].vx = m->one[i].vx - sp;
    ekin = ekin + m->one[i].vx * m->one[i].vx;
  }
  sp = 0.0;
  for (int i = 0; i < mdsize; i++) sp = sp + m->one[i].vy;
  sp = sp / mdsize;
  for (int i = 0; i < mdsize; i++) {
    m->one[i].vy = m->one[i].vy - sp;
    ekin = ekin + m->one[i].vy * m->one[i].vy;
  }
  sp = 0.0;
  for (int i = 0; i < mdsize; i++) sp = sp + m->one[i].vz;
  sp = sp / mdsize;
  for (int i = 0; i < mdsize; i++) {
    m->one[i].vz = m->one[i].vz - sp;
    ekin = ekin + m->one[i].vz * m->one[i].vz;
  }
  const double ts = m->tscale * ekin;
  const double sc = m->h * sqrt(m->tref / ts);
  for (int i = 0; i < mdsize; i++) {
    m->one[i].vx = m->one[i].vx * sc;
    m->one[i].vy = m->one[i].vy * sc;
    m->one[i].vz = m->one[i].vz * sc;
  }
  return m;
}

void ora_md_free(ora_md *m) {
  if (!m) return;
  free(m->one);
  free(m);
}

int ora_md_mdsize(const ora_md *m) { return m->mdsize; }

static void md_domove(particle *p, double side) { /* md.java:346-369 */
  p->x = p->x + p->vx + p->fx;
  p->y = p->y + p->vy + p->fy;
  p->z = p->z + p->vz + p->fz;
  if (p->x < 0) p->x = p->x + side;
  if (p->x > side) p->x = p->x - side;
  if (p->y < 0) p->y = p->y + side;
  if (p->y > side) p->y = p->y - side;
  if (p->z < 0) p->z = p->z + side;
  if (p->z > side) p->z = p->z - side;
  p->vx = p->vx + p->fx;
  p->vy = p->vy + p->fy;
  p->vz = p->vz + p->fz;
  p->fx = 0.0;
  p->fy = 0.0;
  p->fz = 0.0;
}

static void md_force(ora_md *m, int x) { /* md.java:371-434 */
  particle *one = m->one;
  const double side = m->side, sideh = 0.5 * side, rcoffs = m->rcoff * m->rcoff;
  const double xi = one[x].x, yi = one[x].y, zi = one[x].z;
  double fxi = 0.0, fyi = 0.0, fzi = 0.0;
  for (int i = x + 1; i < m->mdsize; i++) {
    double xx = xi - one[i].x, yy = yi - one[i].y, zz = zi - one[i].z;
    if (xx < (-sideh)) xx = xx + side;
    if (xx > (sideh)) xx = xx - side;
    if (yy < (-sideh)) yy = yy + side;
    if (yy > (sideh)) yy = yy - side;
    if (zz < (-sideh)) zz = zz + side;
    if (zz > (sideh)) zz = zz - side;
    const double rd = xx * xx + yy * yy + zz * zz;
    if (rd <= rcoffs) {
      const double rrd = 1.0 / rd, rrd2 = rrd * rrd, rrd3 = rrd2 * rrd, rrd4 = rrd2 * rrd2;
      const double rrd6 = rrd2 * rrd4, rrd7 = rrd6 * rrd;
      m->epot = m->epot + (rrd6 - rrd3);
      const double r148 = rrd7 - 0.5 * rrd4;
      m->vir = m->vir - rd * r148;
      const double forcex = xx * r148;
      fxi = fxi + forcex;
      one[i].fx = one[i].fx - forcex;
      const double forcey = yy * r148;
      fyi = fyi + forcey;
      one[i].fy = one[i].fy - forcey;
      const double forcez = zz * r148;
      fzi = fzi + forcez;
      one[i].fz = one[i].fz - forcez;
      m->interactions = (int32_t)((uint32_t)m->interactions + 1u); /* Java int++ wraps */
    }
  }
  one[x].fx = one[x].fx + fxi;
  one[x].fy = one[x].fy + fyi;
  one[x].fz = one[x].fz + fzi;
}

/* runiters() up to the Allreduces (md.java:222-244): every move, then this rank's cyclic share of
 * the forces; the partial forces go out in xf/yf/zf, epot/vir in ev[0..1], the count in *inter. */
void ora_md_forces(ora_md *m, int rank, int P, double *xf, double *yf, double *zf, double *ev, int32_t *inter) {
  for (int i = 0; i < m->mdsize; i++) md_domove(&m->one[i], m->side);
  m->epot = 0.0;
  m->vir = 0.0;
  for (int i = rank; i < m->mdsize; i += P) md_force(m, i);
  for (int i = 0; i < m->mdsize; i++) {
    xf[i] = m->one[i].fx;
    yf[i] = m->one[i].fy;
    zf[i] = m->one[i].fz;
  }
  ev[0] = m->epot;
  ev[1] = m->vir;
  *inter = m->interactions;
}

/* The rest of the move after the Allreduces (md.java:252-318), with the reduced values. */
void ora_md_finish(ora_md *m, const double *xf, const double *yf, const double *zf, const double *ev,
                   int32_t inter) {
  const int mdsize = m->mdsize;
  for (int i = 0; i < mdsize; i++) {
    m->one[i].fx = xf[i];
    m->one[i].fy = yf[i];
    m->one[i].fz = zf[i];
  }
  m->epot = ev[0];
  m->vir = ev[1];
  m->interactions = inter;
  double sum = 0.0;
  for (int i = 0; i < mdsize; i++) { /* mkekin, md.java:436-451 */
    particle *p = &m->one[i];
    p->fx = p->fx * m->hsq2;
    p->fy = p->fy * m->hsq2;
    p->fz = p->fz * m->hsq2;
    p->vx = p->vx + p->fx;
    p->vy = p->vy + p->fy;
    p->vz = p->vz + p->fz;
    sum = sum + ((p->vx * p->vx) + (p->vy * p->vy) + (p->vz * p->vz));
  }
  m->ekin = sum / m->hsq;
  double vel = 0.0;
  m->count = 0.0;
  for (int i = 0; i < mdsize; i++) { /* velavg, md.java:453-465 */
    const particle *p = &m->one[i];
    const double sq = sqrt(p->vx * p->vx + p->vy * p->vy + p->vz * p->vz);
    if (sq > m->vaverh) m->count = m->count + 1.0;
    vel = vel + sq;
  }
  m->vel = vel / m->h;
  const int istop = 19, irep = 10, iprint = 10, move = m->move;
  if ((move < istop) && (((move + 1) % irep) == 0)) {
    const double sc = sqrt(m->tref / (m->tscale * m->ekin));
    for (int i = 0; i < mdsize; i++) { /* dscal */
      m->one[i].vx = m->one[i].vx * sc;
      m->one[i].vy = m->one[i].vy * sc;
      m->one[i].vz = m->one[i].vz * sc;
    }
    m->ekin = m->tref / m->tscale;
  }
  if (((move + 1) % iprint) == 0) {
    m->ek = 24.0 * m->ekin;
    m->epot = 4.0 * m->epot;
  }
  m->move++;
}

double ora_md_ek(const ora_md *m) { return m->ek; }
int32_t ora_md_interactions(const ora_md *m) { return m->interactions; }
int ora_md_moves(void) { return 50; } /* movemx, md.java:77 */
