/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into or called by the product path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and
 * only as the checker / the timed CPU baseline.
 *
 * Plain-C, single-threaded restatement of the native operations DGL 0.8.2.post1
 * (the reference's pinned third-party dependency, README.md:27; not vendored in
 * /root/reference and not installed here) runs under the reference's call sites:
 *
 *   oracle_csc_build   dgl.graph((start, end), num_nodes) + dgl.add_self_loop
 *                      (code/utils.py:44-45) and the lazily built CSC that update_all
 *                      walks (first use at code/model.py:20): in-edges of each
 *                      destination in ascending edge id, self-loop ids E..E+N-1 last.
 *   oracle_spmm_max    SpMMCmpCsr<copy_lhs|u_mul_e, Max> reached from SAGEConv('pool')'s
 *                      update_all(copy_u('h','m'), max('m','neigh')) (code/model.py:20,
 *                      22, 24): out starts at -inf, argX at 0; an entry replaces the
 *                      running value only when strictly greater (first max wins);
 *                      argX = source node id, argE = edge id; afterwards +-inf -> 0
 *                      (DGL _gspmm replace_inf_with_zero).
 *   oracle_spmm_max_bwd  GSpMM.backward for max: dX = zeros; dX.scatter_add_(0, argX,
 *                      dZ [* w[argE]]) visiting destinations in ascending order
 *                      (train_loss.backward(), code/train.py:204).
 *   oracle_spmm_sum    SpMMCsr<copy_lhs|u_mul_e, Sum> and mean (= sum / in-degree):
 *                      the aggregator variants the reference does not run
 *                      (reference-unpinned).
 *
 * Parity of these restatements against DGL itself is UNPINNED: the reference has no
 * tests or fixtures for this path and DGL cannot be run here.
 * They are pinned by hand-built known-answer tests (tests/test_oracle.py) that encode
 * the semantics above. Compile: see oracle/Makefile (gcc -O2 -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Stable order of edges by destination: insertion sort within buckets keyed by dst.
 * Deliberately a different algorithm from the product's counting sort. */
typedef struct {
  int64_t dst;
  int64_t eid;
} edge_key;

static int cmp_key(const void* a, const void* b) {
  const edge_key* x = (const edge_key*)a;
  const edge_key* y = (const edge_key*)b;
  if (x->dst != y->dst) return x->dst < y->dst ? -1 : 1;
  if (x->eid != y->eid) return x->eid < y->eid ? -1 : 1;
  return 0;
}

/* indptr[n_dst+1], indices[nnz] (source ids), eids[nnz] (edge ids). Returns 0 / -1. */
int oracle_csc_build(const int64_t* src, const int64_t* dst, int64_t nnz, int64_t n_dst,
                     int64_t* indptr, int64_t* indices, int64_t* eids) {
  edge_key* keys = (edge_key*)malloc(sizeof(edge_key) * (size_t)(nnz > 0 ? nnz : 1));
  if (!keys) return -1;
  for (int64_t e = 0; e < nnz; ++e) {
    if (dst[e] < 0 || dst[e] >= n_dst) {
      free(keys);
      return -1;
    }
    keys[e].dst = dst[e];
    keys[e].eid = e;
  }
  qsort(keys, (size_t)nnz, sizeof(edge_key), cmp_key);
  for (int64_t v = 0; v <= n_dst; ++v) indptr[v] = 0;
  for (int64_t e = 0; e < nnz; ++e) indptr[keys[e].dst + 1]++;
  for (int64_t v = 0; v < n_dst; ++v) indptr[v + 1] += indptr[v];
  for (int64_t k = 0; k < nnz; ++k) {
    indices[k] = src[keys[k].eid];
    eids[k] = keys[k].eid;
  }
  free(keys);
  return 0;
}

/* X: n_src x F (row-major, contiguous). w: per-edge weights indexed by edge id, or NULL.
 * out: n_dst x F; argx, arge: n_dst x F (int64). */
void oracle_spmm_max(const int64_t* indptr, const int64_t* indices, const int64_t* eids,
                     const float* w, const float* X, int64_t n_dst, int64_t F, float* out,
                     int64_t* argx, int64_t* arge) {
  for (int64_t v = 0; v < n_dst; ++v) {
    float* o = out + v * F;
    int64_t* ax = argx + v * F;
    int64_t* ae = arge + v * F;
    for (int64_t f = 0; f < F; ++f) {
      o[f] = -INFINITY;
      ax[f] = 0;
      ae[f] = 0;
    }
    for (int64_t j = indptr[v]; j < indptr[v + 1]; ++j) {
      const int64_t u = indices[j];
      const int64_t e = eids[j];
      for (int64_t f = 0; f < F; ++f) {
        const float val = w ? X[u * F + f] * w[e] : X[u * F + f];
        if (o[f] < val) { /* Cmp = Max: replace only when strictly greater */
          o[f] = val;
          ax[f] = u;
          ae[f] = e;
        }
      }
    }
    for (int64_t f = 0; f < F; ++f)
      if (isinf(o[f])) o[f] = 0.f;
  }
}

/* dX (n_src x F) = scatter_add over destinations in ascending order. The zero-in-degree
 * rows of DGL would scatter into node 0 through their argX = 0; `has_in` (n_dst flags)
 * lets the caller exclude them (unreachable with self-loops). */
void oracle_spmm_max_bwd(const int64_t* argx, const int64_t* arge, const float* w,
                         const float* dZ, const uint8_t* has_in, int64_t n_dst, int64_t n_src,
                         int64_t F, float* dX) {
  memset(dX, 0, sizeof(float) * (size_t)(n_src * F));
  for (int64_t v = 0; v < n_dst; ++v) {
    if (has_in && !has_in[v]) continue;
    for (int64_t f = 0; f < F; ++f) {
      const float g = w ? dZ[v * F + f] * w[arge[v * F + f]] : dZ[v * F + f];
      dX[argx[v * F + f] * F + f] += g;
    }
  }
}

/* mean = 1: out row divided by in-degree (rows with no in-edges stay 0). */
void oracle_spmm_sum(const int64_t* indptr, const int64_t* indices, const int64_t* eids,
                     const float* w, const float* X, int64_t n_dst, int64_t F, int mean,
                     float* out) {
  for (int64_t v = 0; v < n_dst; ++v) {
    float* o = out + v * F;
    for (int64_t f = 0; f < F; ++f) o[f] = 0.f;
    for (int64_t j = indptr[v]; j < indptr[v + 1]; ++j) {
      const int64_t u = indices[j];
      const int64_t e = eids[j];
      for (int64_t f = 0; f < F; ++f) o[f] += w ? X[u * F + f] * w[e] : X[u * F + f];
    }
    const int64_t d = indptr[v + 1] - indptr[v];
    if (mean && d > 0)
      for (int64_t f = 0; f < F; ++f) o[f] = o[f] / (float)d;
  }
}

/* The same SpMMCmpCsr<copy_lhs|u_mul_e, Max> loop, row-parallel with OpenMP as DGL's CPU
 * backend runs it (runtime::parallel_for over destination rows): the CPU BASELINE timed
 * by bench.py's cpu_baseline leg. Each row is computed exactly as in oracle_spmm_max, so
 * the results are identical. */
void oracle_spmm_max_omp(const int64_t* indptr, const int64_t* indices, const int64_t* eids,
                         const float* w, const float* X, int64_t n_dst, int64_t F, float* out,
                         int64_t* argx, int64_t* arge) {
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t v = 0; v < n_dst; ++v) {
    float* o = out + v * F;
    int64_t* ax = argx + v * F;
    int64_t* ae = arge + v * F;
    for (int64_t f = 0; f < F; ++f) {
      o[f] = -INFINITY;
      ax[f] = 0;
      ae[f] = 0;
    }
    for (int64_t j = indptr[v]; j < indptr[v + 1]; ++j) {
      const int64_t u = indices[j];
      const int64_t e = eids[j];
      for (int64_t f = 0; f < F; ++f) {
        const float val = w ? X[u * F + f] * w[e] : X[u * F + f];
        if (o[f] < val) {
          o[f] = val;
          ax[f] = u;
          ae[f] = e;
        }
      }
    }
    for (int64_t f = 0; f < F; ++f)
      if (isinf(o[f])) o[f] = 0.f;
  }
}

/* float64 form of the same loop (copy_lhs|u_mul_e, Max): the exact-arithmetic yardstick
 * the full-size parity tests use where two float32 computations differ by more than the
 * 1e-4 bar. Row-parallel; each row is independent. */
void oracle_spmm_max_f64(const int64_t* indptr, const int64_t* indices, const int64_t* eids,
                         const double* w, const double* X, int64_t n_dst, int64_t F, double* out,
                         int64_t* argx, int64_t* arge) {
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t v = 0; v < n_dst; ++v) {
    double* o = out + v * F;
    int64_t* ax = argx + v * F;
    int64_t* ae = arge + v * F;
    for (int64_t f = 0; f < F; ++f) {
      o[f] = -INFINITY;
      ax[f] = 0;
      ae[f] = 0;
    }
    for (int64_t j = indptr[v]; j < indptr[v + 1]; ++j) {
      const int64_t u = indices[j];
      const int64_t e = eids[j];
      for (int64_t f = 0; f < F; ++f) {
        const double val = w ? X[u * F + f] * w[e] : X[u * F + f];
        if (o[f] < val) {
          o[f] = val;
          ax[f] = u;
          ae[f] = e;
        }
      }
    }
    for (int64_t f = 0; f < F; ++f)
      if (isinf(o[f])) o[f] = 0.0;
  }
}

/* Decision alignment for parity tests: after oracle_spmm_max[_f64] has run, entries where
 * another computation picked a different winning edge (`hint`: in-row positions of the
 * in-CSR, n_dst x F, -1 = none) take that winner when the two candidates lie within the
 * rounding band of each other: m - val <= band * max(S[u_own, f] w_own, S[u_hint, f] w_hint),
 * S (n_src x F) being the float64 running-error scale of X (the sum of |terms| X was formed
 * from, propagated through the layers: oracle.py) — a few ulp of the magnitudes that
 * formed THESE candidates. Which of two candidates this close wins is decided by float32
 * rounding, not by the algorithm. Returns the number of changed entries; *hard counts the
 * entries where the hint names a different winner OUTSIDE the band (a real disagreement),
 * *max_gap the largest (m - val) / max(scale) among the changed entries. */
static inline double cand_scale(const double* S, const float* w, int64_t u, int64_t e, int64_t F, int64_t f) {
  return S[u * F + f] * (w ? fabs((double)w[e]) : 1.0);
}

int64_t oracle_spmm_max_align(const int64_t* indptr, const int64_t* indices, const int64_t* eids,
                              const float* w, const float* X, int64_t n_dst, int64_t F,
                              const int32_t* hint, const double* S, double band, float* out,
                              int64_t* argx, int64_t* arge, int64_t* hard, double* max_gap) {
  int64_t changed = 0, nhard = 0;
  double gap_max = 0.0;
  for (int64_t v = 0; v < n_dst; ++v) {
    for (int64_t f = 0; f < F; ++f) {
      const int32_t p = hint[v * F + f];
      if (p < 0 || p >= indptr[v + 1] - indptr[v]) continue;
      const int64_t j = indptr[v] + p;
      const int64_t u = indices[j], e = eids[j];
      if (u == argx[v * F + f] && e == arge[v * F + f]) continue;
      const float val = w ? X[u * F + f] * w[e] : X[u * F + f];
      const float m = out[v * F + f];
      const double s0 = cand_scale(S, w, argx[v * F + f], arge[v * F + f], F, f);
      const double s1 = cand_scale(S, w, u, e, F, f);
      const double smax = s0 > s1 ? s0 : s1;
      if ((double)m - (double)val <= band * smax) {
        if (smax > 0.0 && ((double)m - (double)val) / smax > gap_max) gap_max = ((double)m - (double)val) / smax;
        out[v * F + f] = val;
        argx[v * F + f] = u;
        arge[v * F + f] = e;
        ++changed;
      } else {
        ++nhard;
      }
    }
  }
  if (hard) *hard = nhard;
  if (max_gap) *max_gap = gap_max;
  return changed;
}

int64_t oracle_spmm_max_align_f64(const int64_t* indptr, const int64_t* indices, const int64_t* eids,
                                  const double* w, const double* X, int64_t n_dst, int64_t F,
                                  const int32_t* hint, const double* S, double band, double* out,
                                  int64_t* argx, int64_t* arge, int64_t* hard, double* max_gap) {
  int64_t changed = 0, nhard = 0;
  double gap_max = 0.0;
  for (int64_t v = 0; v < n_dst; ++v) {
    for (int64_t f = 0; f < F; ++f) {
      const int32_t p = hint[v * F + f];
      if (p < 0 || p >= indptr[v + 1] - indptr[v]) continue;
      const int64_t j = indptr[v] + p;
      const int64_t u = indices[j], e = eids[j];
      if (u == argx[v * F + f] && e == arge[v * F + f]) continue;
      const double val = w ? X[u * F + f] * w[e] : X[u * F + f];
      const double m = out[v * F + f];
      const int64_t uo = argx[v * F + f], eo = arge[v * F + f];
      const double s0 = S[uo * F + f] * (w ? fabs(w[eo]) : 1.0);
      const double s1 = S[u * F + f] * (w ? fabs(w[e]) : 1.0);
      const double smax = s0 > s1 ? s0 : s1;
      if (m - val <= band * smax) {
        if (smax > 0.0 && (m - val) / smax > gap_max) gap_max = (m - val) / smax;
        out[v * F + f] = val;
        argx[v * F + f] = u;
        arge[v * F + f] = e;
        ++changed;
      } else {
        ++nhard;
      }
    }
  }
  if (hard) *hard = nhard;
  if (max_gap) *max_gap = gap_max;
  return changed;
}
