// jgf_tests.cpp — the reference's two JGF benchmarks whose kernels are Allreduce(DOUBLE, SUM) calls,
// run through the C++ host mirror (include/mpjx.hpp) in a NATIVE process, i.e. bound to /opt/rocm's
// HIP runtime and RCCL as a JVM loading libmpjx would be (Python processes bind torch's bundled
// runtime). Multicore ranks are threads (MulticoreStarter), the arrays host vectors (Java heap arrays:
// mpjx_allreduce_host), the application side is the oracle's restatement (test infrastructure):
//   SparseMatmult  test/jgf_mpj_benchmarks/section2/sparsematmult (200 Allreduce per run)
//                  refval A = 75.02484945753453 (JGFSparseMatmultBench.java:148)
//   MolDyn         test/jgf_mpj_benchmarks/section3/moldyn (6 in-place Allreduce per move, 50 moves)
//                  refval A = 1731.4306625334357 (JGFMolDynBench.java:72)
//   RayTracer      test/jgf_mpj_benchmarks/section3/raytracer (one in-place Reduce(DOUBLE, SUM, root 0)
//                  of the pixel checksum), refval A = 2676692 (JGFRayTracerBench.java:87), exact at every P
// P = 1 must give refval exactly; every P must give the oracle's own restatement of the reference's
// reduction order (ora_allreduce) bit for bit. Prints "ALL JGF TESTS PASSED" or the failures.
//   build: make -C mpjexpress_amd tests      run: tests/cpp/jgf_tests [P ...]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#include "../../oracle/mpjx_oracle.h"
#include "mpjx.hpp"

using mpi::MPI;

static int g_fail = 0;

static void run_ranks(std::vector<mpi::Intracomm>& w, const std::function<void(mpi::Intracomm&)>& fn) {
  std::vector<std::thread> th;
  std::vector<std::string> err(w.size());
  for (size_t r = 0; r < w.size(); r++)
    th.emplace_back([&, r] {
      try {
        (void)hipSetDevice(0);
        fn(w[r]);
      } catch (const std::exception& e) {
        err[r] = e.what();
      }
    });
  for (auto& t : th) t.join();
  for (size_t r = 0; r < w.size(); r++)
    if (!err[r].empty()) {
      printf("rank %zu: %s\n", r, err[r].c_str());
      g_fail++;
    }
}

// ---- SparseMatmult -------------------------------------------------------------------------------
struct Sparse {
  int M = 50000, N = 50000, nz = 250000;
  std::vector<double> x, val;
  std::vector<int32_t> row, col;
  Sparse() : x(N), val(nz), row(nz), col(nz) {
    if (ora_jgf_sparse_gen(10101010, M, N, nz, x.data(), row.data(), col.data(), val.data())) abort();
  }
  void share(int r, int P, int* lo, int* hi) const {  // JGFSparseMatmultBench.java:73-80
    const int p = (nz + P - 1) / P, rem = p - (p * P - nz);
    *lo = r * p;
    *hi = r * p + ((r == P - 1 && p * (r + 1) > nz) ? rem : p);
  }
};

static double sparse_oracle(const Sparse& S, int P) {
  std::vector<std::vector<double>> py(P, std::vector<double>(S.M)), y(P, std::vector<double>(S.M));
  std::vector<void*> sp(P), rp(P);
  for (int it = 0; it < 200; it++) {
    for (int r = 0; r < P; r++) {
      int lo, hi;
      S.share(r, P, &lo, &hi);
      ora_jgf_sparse_rep(py[r].data(), S.x.data(), S.row.data(), S.col.data(), S.val.data(), lo, hi);
      sp[r] = py[r].data();
      rp[r] = y[r].data();
    }
    ora_allreduce(P, 0, sp.data(), 0, rp.data(), 0, S.M, ORA_DOUBLE, ORA_SUM);
  }
  return ora_jgf_ytotal(y[0].data(), S.row.data(), S.nz);
}

static void sparse_test(const Sparse& S, int P) {
  auto w = mpi::smp_world(P, std::vector<int>(P, 0));
  std::vector<double> ytot(P);
  run_ranks(w, [&](mpi::Intracomm& c) {
    const int r = c.Rank();
    int lo, hi;
    S.share(r, P, &lo, &hi);
    std::vector<double> p_y(S.M, 0.0), y(S.M, 0.0);
    for (int it = 0; it < 200; it++) {  // SparseMatmult.java:239-247
      ora_jgf_sparse_rep(p_y.data(), S.x.data(), S.row.data(), S.col.data(), S.val.data(), lo, hi);
      c.Allreduce(p_y, 0, y, 0, S.M, MPI::DOUBLE, MPI::SUM);
    }
    ytot[r] = ora_jgf_ytotal(y.data(), S.row.data(), S.nz);
  });
  const double exp = sparse_oracle(S, P), ref = 75.02484945753453;
  const bool ok = ytot[0] == exp && (P > 1 || ytot[0] == ref) && std::fabs(ytot[0] - ref) <= 1e-12;
  printf("SparseMatmult P=%d: ytotal %.17g oracle %.17g refval %.17g -> %s\n", P, ytot[0], exp, ref,
         ok ? "ok" : "FAILED");
  if (!ok) g_fail++;
}

// ---- MolDyn ----------------------------------------------------------------------------------------
static void md_step_allreduce_oracle(std::vector<ora_md*>& ranks, int P) {
  const int n = ora_md_mdsize(ranks[0]);
  std::vector<std::vector<double>> xf(P, std::vector<double>(n)), yf(xf), zf(xf), ev(P, std::vector<double>(2));
  std::vector<int32_t> in(P);
  for (int r = 0; r < P; r++) ora_md_forces(ranks[r], r, P, xf[r].data(), yf[r].data(), zf[r].data(), ev[r].data(), &in[r]);
  auto red = [&](std::vector<std::vector<double>>& v, int off, int cnt) {
    std::vector<void*> sp(P), rp(P);
    std::vector<std::vector<double>> out(P, std::vector<double>(cnt));
    for (int r = 0; r < P; r++) {
      sp[r] = v[r].data() + off;
      rp[r] = out[r].data();
    }
    ora_allreduce(P, 0, sp.data(), 0, rp.data(), 0, cnt, ORA_DOUBLE, ORA_SUM);
    for (int r = 0; r < P; r++) memcpy(v[r].data() + off, out[r].data(), cnt * sizeof(double));
  };
  red(xf, 0, n);
  red(yf, 0, n);
  red(zf, 0, n);
  red(ev, 0, 1);
  red(ev, 1, 1);
  std::vector<void*> sp(P), rp(P);
  std::vector<int32_t> inr(P);
  for (int r = 0; r < P; r++) {
    sp[r] = &in[r];
    rp[r] = &inr[r];
  }
  ora_allreduce(P, 0, sp.data(), 0, rp.data(), 0, 1, ORA_INT, ORA_SUM);
  for (int r = 0; r < P; r++) ora_md_finish(ranks[r], xf[r].data(), yf[r].data(), zf[r].data(), ev[r].data(), inr[r]);
}

static void moldyn_test(int P) {
  std::vector<ora_md*> ora(P);
  for (int r = 0; r < P; r++) ora[r] = ora_md_new(0);
  for (int m = 0; m < ora_md_moves(); m++) md_step_allreduce_oracle(ora, P);
  const double exp = ora_md_ek(ora[0]);
  std::vector<int32_t> exp_inter(P);
  for (int r = 0; r < P; r++) {
    exp_inter[r] = ora_md_interactions(ora[r]);
    ora_md_free(ora[r]);
  }
  auto w = mpi::smp_world(P, std::vector<int>(P, 0));
  std::vector<double> ek(P);
  std::vector<int32_t> inter(P);
  run_ranks(w, [&](mpi::Intracomm& c) {
    const int r = c.Rank();
    ora_md* md = ora_md_new(0);
    const int n = ora_md_mdsize(md);
    std::vector<double> xf(n), yf(n), zf(n), ev(2), ep(1), vi(1);
    std::vector<int32_t> it(1);
    for (int m = 0; m < ora_md_moves(); m++) {
      ora_md_forces(md, r, P, xf.data(), yf.data(), zf.data(), ev.data(), it.data());
      ep[0] = ev[0];
      vi[0] = ev[1];
      c.Allreduce(xf, 0, xf, 0, n, MPI::DOUBLE, MPI::SUM);  // md.java:248-264, in place
      c.Allreduce(yf, 0, yf, 0, n, MPI::DOUBLE, MPI::SUM);
      c.Allreduce(zf, 0, zf, 0, n, MPI::DOUBLE, MPI::SUM);
      c.Allreduce(ep, 0, ep, 0, 1, MPI::DOUBLE, MPI::SUM);
      c.Allreduce(vi, 0, vi, 0, 1, MPI::DOUBLE, MPI::SUM);
      c.Allreduce(it, 0, it, 0, 1, MPI::INT, MPI::SUM);
      ev[0] = ep[0];
      ev[1] = vi[0];
      ora_md_finish(md, xf.data(), yf.data(), zf.data(), ev.data(), it[0]);
    }
    ek[r] = ora_md_ek(md);
    inter[r] = ora_md_interactions(md);
    ora_md_free(md);
  });
  const double ref = 1731.4306625334357;
  const bool ok = ek[0] == exp && inter == exp_inter && (P > 1 || ek[0] == ref);
  printf("MolDyn P=%d: ek %.17g oracle %.17g refval %.17g interactions %d -> %s\n", P, ek[0], exp, ref, inter[0],
         ok ? "ok" : "FAILED");
  if (!ok) g_fail++;
}

// ---- RayTracer -------------------------------------------------------------------------------------
static void raytracer_test(const std::vector<int64_t>& rows, int P) {
  auto w = mpi::smp_world(P, std::vector<int>(P, 0));
  std::vector<int64_t> checksum(P);
  run_ranks(w, [&](mpi::Intracomm& c) {
    const int r = c.Rank();
    std::vector<double> tmp(1, (double)ora_jgf_raytracer_partial(rows.data(), (int)rows.size(), r, P));
    c.Reduce(tmp, 0, tmp, 0, 1, MPI::DOUBLE, MPI::SUM, 0);  // RayTracer.java:275-279, in place
    checksum[r] = (int64_t)tmp[0];
  });
  const int64_t ref = 2676692;
  const bool ok = checksum[0] == ref;
  printf("RayTracer P=%d: checksum %lld refval %lld -> %s\n", P, (long long)checksum[0], (long long)ref,
         ok ? "ok" : "FAILED");
  if (!ok) g_fail++;
}

int main(int argc, char** argv) {
  std::vector<int> Ps;
  for (int i = 1; i < argc; i++) Ps.push_back(atoi(argv[i]));
  if (Ps.empty()) Ps = {1, 2, 4, 8};
  int rt = 0, rc = 0;
  mpjx_runtime_versions(&rt, &rc);
  printf("HIP runtime %d, RCCL %d\n", rt, rc);
  Sparse S;
  std::vector<int64_t> rt_rows(150);
  if (ora_jgf_raytracer_rows(150, rt_rows.data())) abort();
  for (int P : Ps) {
    sparse_test(S, P);
    moldyn_test(P);
    raytracer_test(rt_rows, P);
  }
  if (g_fail) {
    printf("%d JGF TEST(S) FAILED\n", g_fail);
    return 1;
  }
  printf("ALL JGF TESTS PASSED\n");
  return 0;
}
