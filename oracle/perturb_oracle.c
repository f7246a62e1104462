/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into or called by the product path.
 *
 * Streaming plain-C restatement of the reference's topology perturbation, without the
 * N x N matrices (used for large-N checks and as the timed CPU baseline):
 *   construct_gcn_matrix (code/data_preprocess.py:165-170):
 *     pcc = np.corrcoef(expr): xc = x - mean(x) (caller, numpy), c = dot(xc_i, xc_j) /
 *     (S - 1), c /= sd_i, c /= sd_j, clip(c, -1, 1); fill_diagonal(pcc, 0); pcc[nan] = 0
 *     (the dot in OpenBLAS dgemm's order: a fused multiply-add chain over the samples)
 *   modify_network_topology (code/data_preprocess.py:217-257):
 *     diff = pcc_inter - pcc_normal; mean, std over all n*n entries;
 *     ppi' = 0 where ppi == 1 and diff < mean - thr*std; 1 where ppi == 0 and diff > mean + thr*std
 * Sums are compensated (Neumaier) in row order. The dense numpy restatement in
 * oracle.py (np.corrcoef / np.mean / np.std verbatim) pins this one and the GPU path on
 * the reference's own outputs (tests/golden/perturb.npz).
 */
#include <math.h>
#include <stdint.h>

static double po_dot(const double* a, const double* b, int S) {
  double d = a[0] * b[0];
  for (int s = 1; s < S; ++s) d = fma(a[s], b[s], d);
  return d;
}

static double po_pcc(const double* xa, double sda, const double* xb, double sdb, int S,
                     double inv_fact, int diag) {
  double c = po_dot(xa, xb, S) * inv_fact;
  c = c / sda;
  c = c / sdb;
  if (c < -1.0) c = -1.0;
  else if (c > 1.0) c = 1.0;
  if (diag || c != c) c = 0.0;
  return c;
}

void oracle_perturb_sd(const double* xc, int64_t n, int S, double inv_fact, double* sd) {
  for (int64_t i = 0; i < n; ++i) sd[i] = sqrt(po_dot(xc + i * S, xc + i * S, S) * inv_fact);
}

static double po_diff(const double* xn, const double* xi, const double* sdn, const double* sdi,
                      int S, double inv_fact, int64_t i, int64_t j) {
  const int diag = i == j;
  return po_pcc(xi + i * S, sdi[i], xi + j * S, sdi[j], S, inv_fact, diag) -
         po_pcc(xn + i * S, sdn[i], xn + j * S, sdn[j], S, inv_fact, diag);
}

static void kadd(double* s, double* c, double x) {
  const double t = *s + x;
  if (fabs(*s) >= fabs(x)) *c += (*s - t) + x;
  else *c += (x - t) + *s;
  *s = t;
}

/* sum over rows [r0, r1) x all columns of diff (squared = 0) or (diff - mean)^2 */
double oracle_perturb_sum(const double* xn, const double* xi, const double* sdn, const double* sdi,
                          int64_t n, int S, double inv_fact, int squared, double mean, int64_t r0,
                          int64_t r1) {
  double s = 0.0, c = 0.0;
  for (int64_t i = r0; i < r1; ++i)
    for (int64_t j = 0; j < n; ++j) {
      double d = po_diff(xn, xi, sdn, sdi, S, inv_fact, i, j);
      if (squared) {
        d = d - mean;
        d = d * d;
      }
      kadd(&s, &c, d);
    }
  return s + c;
}

/* rows [r0, r1) of the perturbed adjacency. ptr/col/val: CSR of the original (sorted
 * unique columns; val NULL = ones). Writes (row, col, val) of the non-zeros row-major
 * into the outputs (capacity cap); returns the count, or -1 when cap is exceeded. */
int64_t oracle_perturb_rows(const double* xn, const double* xi, const double* sdn, const double* sdi,
                            int64_t n, int S, double inv_fact, const int64_t* ptr, const int64_t* col,
                            const int64_t* val, double lo_thr, double hi_thr, int64_t r0, int64_t r1,
                            int64_t* out_row, int64_t* out_col, int64_t* out_val, int64_t cap) {
  int64_t m = 0;
  for (int64_t i = r0; i < r1; ++i) {
    int64_t k = ptr[i];
    for (int64_t j = 0; j < n; ++j) {
      int64_t v = 0;
      while (k < ptr[i + 1] && col[k] < j) ++k;
      if (k < ptr[i + 1] && col[k] == j) v = val ? val[k] : 1;
      if (v == 0 || v == 1) {
        const double d = po_diff(xn, xi, sdn, sdi, S, inv_fact, i, j);
        if (v == 1 && d < lo_thr) v = 0;
        else if (v == 0 && d > hi_thr) v = 1;
      }
      if (v != 0) {
        if (m >= cap) return -1;
        out_row[m] = i;
        out_col[m] = j;
        out_val[m] = v;
        ++m;
      }
    }
  }
  return m;
}
