// ASan + UBSan driver for the host C++ of libplagnn.so (csrc/graph.cpp, csrc/cpu_backend.cpp)
// and the oracle's C restatement (oracle/*.c) — SURVEY.md §5 "ASan/UBSan on the C++ CPU
// oracle". Built by tests/sanitize/Makefile with -fsanitize=address,undefined and run by
// tests/test_sanitize.py (CPU suite). Exercises the graph build (COO -> in-CSR, transpose,
// schedules) and the _cpu message-passing entry points on random multigraphs with empty
// rows, duplicate edges, explicit self-loops and a hub row that the schedule splits, and
// checks them against the oracle (bit-exact max / argmax, backward within summation order);
// then the oracle's ECC and perturbation loops on small inputs. Any sanitizer report aborts
// the process with a non-zero status.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../include/plagnn.h"

extern "C" {
int oracle_csc_build(const int64_t* src, const int64_t* dst, int64_t nnz, int64_t n_dst, int64_t* indptr,
                     int64_t* indices, int64_t* eids);
void oracle_spmm_max(const int64_t* indptr, const int64_t* indices, const int64_t* eids, const float* w,
                     const float* X, int64_t n_dst, int64_t F, float* out, int64_t* argx, int64_t* arge);
void oracle_spmm_max_omp(const int64_t* indptr, const int64_t* indices, const int64_t* eids, const float* w,
                         const float* X, int64_t n_dst, int64_t F, float* out, int64_t* argx, int64_t* arge);
void oracle_spmm_max_bwd(const int64_t* argx, const int64_t* arge, const float* w, const float* dZ,
                         const uint8_t* has_in, int64_t n_dst, int64_t n_src, int64_t F, float* dX);
void oracle_spmm_sum(const int64_t* indptr, const int64_t* indices, const int64_t* eids, const float* w,
                     const float* X, int64_t n_dst, int64_t F, int mean, float* out);
int64_t oracle_spmm_max_align(const int64_t* indptr, const int64_t* indices, const int64_t* eids, const float* w,
                              const float* X, int64_t n_dst, int64_t F, const int32_t* hint, const double* S,
                              double band, float* out, int64_t* argx, int64_t* arge, int64_t* hard,
                              double* max_gap);
int64_t oracle_ecc(const int64_t* indptr, const int64_t* indices, const double* data, int64_t n, double epsilon,
                   int64_t* rows, int64_t* cols, double* vals);
void oracle_perturb_sd(const double* xc, int64_t n, int S, double inv_fact, double* sd);
double oracle_perturb_sum(const double* xn, const double* xi, const double* sdn, const double* sdi, int64_t n, int S,
                          double inv_fact, int squared, double mean, int64_t r0, int64_t r1);
int64_t oracle_perturb_rows(const double* xn, const double* xi, const double* sdn, const double* sdi, int64_t n,
                            int S, double inv_fact, const int64_t* ptr, const int64_t* col, const int64_t* val,
                            double lo_thr, double hi_thr, int64_t r0, int64_t r1, int64_t* out_row, int64_t* out_col,
                            int64_t* out_val, int64_t cap);
}

static int failures = 0;
#define CHECK(c, ...)                 \
  do {                                \
    if (!(c)) {                       \
      std::printf("FAIL: " __VA_ARGS__); \
      std::printf("\n");              \
      ++failures;                     \
    }                                 \
  } while (0)

struct Graph {
  int64_t n, E;
  std::vector<int64_t> src, dst;
};

static Graph random_graph(int64_t n, int64_t e, int64_t hub, uint32_t seed) {
  std::mt19937_64 rng(seed);
  Graph g{n, 0, {}, {}};
  // node n-1 has no in-edges (an empty row) unless a self-loop is added below
  std::uniform_int_distribution<int64_t> any(0, n - 1), some(0, n - 2);
  for (int64_t i = 0; i < e; ++i) {
    g.src.push_back(any(rng));
    g.dst.push_back(some(rng));
  }
  for (int64_t i = 0; i < hub; ++i) {  // hub row 0 (split by the schedule), duplicates allowed
    g.src.push_back(any(rng));
    g.dst.push_back(0);
  }
  g.src.push_back(3);  // explicit self-loop + its duplicate (PPI_inter diagonal)
  g.dst.push_back(3);
  g.src.push_back(3);
  g.dst.push_back(3);
  g.E = (int64_t)g.src.size();
  return g;
}

static void run_case(int64_t n, int64_t e, int64_t hub, int64_t F, int chunk, bool weighted, uint32_t seed) {
  Graph g = random_graph(n, e, hub, seed);
  const int64_t E = g.E;
  std::vector<int32_t> ptr(n + 1), col(E), eid(E);
  CHECK(pg_csr_from_coo(g.src.data(), g.dst.data(), E, n, n, ptr.data(), col.data(), eid.data()) == 0, "csr");
  std::vector<int32_t> tptr(n + 1), tcol(E), tslot(E), tpos(E);
  CHECK(pg_csr_transpose(ptr.data(), col.data(), n, n, E, tptr.data(), tcol.data(), tslot.data(), tpos.data()) == 0,
        "transpose");
  auto sched = [&](const std::vector<int32_t>& p, std::vector<int32_t>& items, std::vector<int32_t>& merges,
                   int64_t& ni, int64_t& nm, int64_t& ns, int32_t& md) {
    CHECK(pg_schedule_count(p.data(), n, chunk, &ni, &nm, &ns, &md) == 0, "schedule count");
    items.assign(4 * (ni > 0 ? ni : 1), 0);
    merges.assign(4 * (nm > 0 ? nm : 1), 0);
    CHECK(pg_schedule_build(p.data(), n, chunk, items.data(), merges.data()) == 0, "schedule build");
  };
  std::vector<int32_t> fi, fm, bi, bm;
  int64_t fni, fnm, fns, bni, bnm, bns;
  int32_t fmd, bmd;
  sched(ptr, fi, fm, fni, fnm, fns, fmd);
  sched(tptr, bi, bm, bni, bnm, bns, bmd);
  std::mt19937_64 rng(seed + 1);
  std::normal_distribution<float> nd;
  std::uniform_real_distribution<float> ud(0.f, 1.f);
  std::vector<float> X(n * F), dZ(n * F), w_eid(E), w_slot(E);
  for (auto& v : X) v = std::max(0.f, nd(rng));  // relu-like: many exact ties at 0
  for (auto& v : dZ) v = nd(rng);
  for (int64_t k = 0; k < E; ++k) w_eid[k] = ud(rng);
  for (int64_t k = 0; k < E; ++k) w_slot[k] = w_eid[eid[k]];
  pg_csr_t fwd{n, n, E, ptr.data(), col.data(), nullptr, nullptr, weighted ? w_slot.data() : nullptr,
               fi.data(), fni, fnm ? fm.data() : nullptr, fnm, fns, fmd, chunk};
  pg_csr_t bwd{n, n, E, tptr.data(), tcol.data(), tslot.data(), tpos.data(), nullptr,
               bi.data(), bni, bnm ? bm.data() : nullptr, bnm, bns, bmd, chunk};
  std::vector<float> out(n * F), dx(n * F), sum(n * F);
  std::vector<int32_t> arg(n * F);
  std::vector<int64_t> argx(n * F), argx_o(n * F), arge_o(n * F);
  CHECK(pg_spmm_max_fwd_cpu(&fwd, X.data(), F, F, out.data(), F, arg.data(), F, PG_ARG_I32) == 0, "max fwd: %s",
        pg_last_error_string());
  CHECK(pg_argpos_to_src_cpu(&fwd, arg.data(), F, PG_ARG_I32, F, argx.data(), F) == 0, "argpos_to_src");
  CHECK(pg_spmm_max_bwd_cpu(&fwd, &bwd, arg.data(), F, PG_ARG_I32, dZ.data(), F, F, X.data(), F, dx.data(), F) == 0,
        "max bwd: %s", pg_last_error_string());
  CHECK(pg_spmm_sum_cpu(&fwd, X.data(), F, F, 1, nullptr, sum.data(), F) == 0, "sum: %s", pg_last_error_string());
  // oracle
  std::vector<int64_t> optr(n + 1), oind(E), oeid(E);
  CHECK(oracle_csc_build(g.src.data(), g.dst.data(), E, n, optr.data(), oind.data(), oeid.data()) == 0, "csc");
  std::vector<float> oout(n * F), oout2(n * F), odx(n * F), osum(n * F);
  const float* w = weighted ? w_eid.data() : nullptr;
  oracle_spmm_max(optr.data(), oind.data(), oeid.data(), w, X.data(), n, F, oout.data(), argx_o.data(),
                  arge_o.data());
  std::vector<int64_t> ax2(n * F), ae2(n * F);
  oracle_spmm_max_omp(optr.data(), oind.data(), oeid.data(), w, X.data(), n, F, oout2.data(), ax2.data(), ae2.data());
  std::vector<uint8_t> has_in(n);
  for (int64_t v = 0; v < n; ++v) has_in[v] = optr[v + 1] > optr[v];
  oracle_spmm_max_bwd(argx_o.data(), arge_o.data(), w, dZ.data(), has_in.data(), n, n, F, odx.data());
  oracle_spmm_sum(optr.data(), oind.data(), oeid.data(), w, X.data(), n, F, 1, osum.data());
  std::vector<int32_t> hint(n * F, -1);
  for (int64_t v = 0; v < n; ++v)  // every row's hint: its first in-edge (real mismatches mostly)
    for (int64_t f = 0; f < F; ++f) hint[v * F + f] = optr[v + 1] > optr[v] ? 0 : -1;
  std::vector<double> S(n * F);
  for (int64_t i = 0; i < n * F; ++i) S[i] = std::fabs((double)X[i]);
  std::vector<float> oout3(oout2);
  std::vector<int64_t> ax3(ax2), ae3(ae2);
  int64_t hard = -1;
  double gap = -1.0;
  const int64_t changed = oracle_spmm_max_align(optr.data(), oind.data(), oeid.data(), w, X.data(), n, F, hint.data(),
                                                S.data(), 0.0, oout3.data(), ax3.data(), ae3.data(), &hard, &gap);
  CHECK(changed >= 0 && hard >= 0 && gap == 0.0, "align counts");
  for (int64_t i = 0; i < n * F; ++i) CHECK(oout3[i] <= oout2[i], "align never raises a maximum (%ld)", (long)i);
  for (int64_t i = 0; i < n * F; ++i) {
    const int64_t v = i / F;
    CHECK(out[i] == oout[i] && out[i] == oout2[i], "max value (%ld)", (long)i);
    if (has_in[v]) CHECK(argx[i] == argx_o[i], "argmax (%ld)", (long)i);
    const float ref = X[i] > 0.f ? odx[i] : 0.f;
    CHECK(std::fabs(dx[i] - ref) <= 1e-5f * (1.f + std::fabs(ref)), "max bwd (%ld) %g vs %g", (long)i, dx[i], ref);
    CHECK(std::fabs(sum[i] - osum[i]) <= 1e-5f * (1.f + std::fabs(osum[i])), "mean (%ld)", (long)i);
  }
}

static void run_ecc_perturb() {
  // triangle {0,1,2} + pendant 0-3 + a 6-clique 4..9, symmetric, no diagonal
  std::vector<std::vector<int64_t>> adj(10);
  auto add = [&](int a, int b) { adj[a].push_back(b); adj[b].push_back(a); };
  add(0, 1); add(1, 2); add(0, 2); add(0, 3);
  for (int a = 4; a < 10; ++a)
    for (int b = a + 1; b < 10; ++b) add(a, b);
  std::vector<int64_t> ptr(11, 0), col;
  std::vector<double> data;
  for (int i = 0; i < 10; ++i) {
    std::sort(adj[i].begin(), adj[i].end());
    for (int64_t j : adj[i]) { col.push_back(j); data.push_back(1.0); }
    ptr[i + 1] = (int64_t)col.size();
  }
  const int64_t nnz = (int64_t)col.size();
  std::vector<int64_t> r(2 * nnz), c(2 * nnz);
  std::vector<double> v(2 * nnz);
  const int64_t m = oracle_ecc(ptr.data(), col.data(), data.data(), 10, 0.0, r.data(), c.data(), v.data());
  CHECK(m > 0, "ecc entries");
  for (int64_t k = 0; k < m; ++k)
    if ((r[k] == 0 && c[k] == 3) || (r[k] == 3 && c[k] == 0)) CHECK(v[k] == 0.0, "pendant ecc");
  const int S = 3;
  std::mt19937_64 rng(9);
  std::normal_distribution<double> nd;
  std::vector<double> xn(10 * S), xi(10 * S), sdn(10), sdi(10);
  for (auto& t : xn) t = nd(rng);
  for (auto& t : xi) t = nd(rng);
  for (int i = 0; i < 10; ++i) {  // centre rows as np.cov does
    double mn = 0, mi = 0;
    for (int s = 0; s < S; ++s) { mn += xn[i * S + s]; mi += xi[i * S + s]; }
    for (int s = 0; s < S; ++s) { xn[i * S + s] -= mn / S; xi[i * S + s] -= mi / S; }
  }
  oracle_perturb_sd(xn.data(), 10, S, 0.5, sdn.data());
  oracle_perturb_sd(xi.data(), 10, S, 0.5, sdi.data());
  const double mean = oracle_perturb_sum(xn.data(), xi.data(), sdn.data(), sdi.data(), 10, S, 0.5, 0, 0.0, 0, 10) / 100.0;
  const double var = oracle_perturb_sum(xn.data(), xi.data(), sdn.data(), sdi.data(), 10, S, 0.5, 1, mean, 0, 10) / 100.0;
  std::vector<int64_t> orow(100), ocol(100), oval(100);
  const int64_t k = oracle_perturb_rows(xn.data(), xi.data(), sdn.data(), sdi.data(), 10, S, 0.5, ptr.data(),
                                        col.data(), nullptr, mean - std::sqrt(var), mean + std::sqrt(var), 0, 10,
                                        orow.data(), ocol.data(), oval.data(), 100);
  CHECK(k >= 0 && k <= 100, "perturb rows");
}

int main() {
  run_case(300, 2000, 0, 7, 256, false, 1);
  run_case(500, 4000, 900, 64, 64, true, 2);    // hub row split by the forward schedule
  run_case(200, 1500, 300, 33, 32, false, 3);   // odd F, tiny chunk: many split rows
  run_case(5, 0, 0, 4, 256, false, 4);          // only the explicit self-loops: empty rows
  run_ecc_perturb();
  if (failures) {
    std::printf("%d failures\n", failures);
    return 1;
  }
  std::printf("sanitize ok\n");
  return 0;
}
