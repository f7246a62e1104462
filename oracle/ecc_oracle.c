/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into or called by the product path.
 *
 * Plain-C restatement of the reference's edge clustering coefficient
 * (code/data_preprocess.py:175-214, edge_clustering_coefficients):
 *   ppi = ppi_net.tocsr()                      (duplicates summed, as scipy does)
 *   for every row i, for every neighbour j > i of i in row order:
 *     triangles = |{k : ppi[i,k] != 0 and ppi[j,k] != 0}|   (logical_and of dense rows)
 *     possible  = min(degree_i, degree_j) - 1,  degree = row sum of the stored data
 *     value     = epsilon if possible == 0 else triangles / possible   (float64)
 *     emit (i, j, value) and (j, i, value)
 * The dense-row logical_and is restated with a per-row marker array (same count).
 * Pinned by tests/golden/ecc.npz, produced by running the reference function itself
 * (tests/golden/gen_golden.py).
 *
 * indptr[n+1], indices[nnz], data[nnz] (f64; a row's degree is its sum). Outputs are
 * written to rows/cols/vals (capacity >= 2 * nnz); returns the number of entries, or -1.
 */
#include <stdint.h>
#include <stdlib.h>

int64_t oracle_ecc(const int64_t* indptr, const int64_t* indices, const double* data, int64_t n,
                   double epsilon, int64_t* rows, int64_t* cols, double* vals) {
  unsigned char* mark = (unsigned char*)calloc((size_t)(n > 0 ? n : 1), 1);
  double* deg = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
  if (!mark || !deg) {
    free(mark);
    free(deg);
    return -1;
  }
  for (int64_t i = 0; i < n; ++i) {
    double s = 0.0;
    for (int64_t k = indptr[i]; k < indptr[i + 1]; ++k) s += data[k];
    deg[i] = s;
  }
  int64_t m = 0;
  for (int64_t i = 0; i < n; ++i) {
    for (int64_t k = indptr[i]; k < indptr[i + 1]; ++k)
      if (data[k] != 0.0) mark[indices[k]] = 1;
    for (int64_t k = indptr[i]; k < indptr[i + 1]; ++k) {
      const int64_t j = indices[k];
      if (j <= i) continue;
      int64_t tri = 0;
      for (int64_t q = indptr[j]; q < indptr[j + 1]; ++q)
        if (data[q] != 0.0 && mark[indices[q]]) ++tri;
      const double a = deg[i], b = deg[j];
      const double possible = (a < b ? a : b) - 1.0;
      const double value = possible == 0.0 ? epsilon : (double)tri / possible;
      rows[m] = i; cols[m] = j; vals[m] = value; ++m;
      rows[m] = j; cols[m] = i; vals[m] = value; ++m;
    }
    for (int64_t k = indptr[i]; k < indptr[i + 1]; ++k) mark[indices[k]] = 0;
  }
  free(mark);
  free(deg);
  return m;
}
