// Host (CPU-device) implementations of the message-passing entry points.
//
// These serve tensors the caller keeps on the CPU device, the role DGL's CPU backend
// plays when the reference runs with `-d cpu` (code/main_normal.py:30, 66). They are a
// device choice made by the caller, never a fallback for a failed GPU call.
// Row-parallel over destinations with OpenMP, entries in CSR order, like DGL's
// SpMMCmpCsr CPU loop.
#include <cmath>
#include <limits>

#include "common.hpp"

namespace {

template <typename A>
inline A none_val();
template <>
inline uint16_t none_val<uint16_t>() { return 0xFFFF; }
template <>
inline int32_t none_val<int32_t>() { return -1; }

template <typename A>
void max_fwd(const pg_csr_t* g, const float* X, int64_t ldx, int64_t F, float* out, int64_t ldo,
             A* arg, int64_t lda) {
  const float ninf = -std::numeric_limits<float>::infinity();
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t v = 0; v < g->n_rows; ++v) {
    float* o = out + v * ldo;
    A* a = arg + v * lda;
    const int32_t b = g->ptr[v], e = g->ptr[v + 1];
    if (b == e) {
      for (int64_t f = 0; f < F; ++f) {
        o[f] = 0.f;
        a[f] = none_val<A>();
      }
      continue;
    }
    for (int64_t f = 0; f < F; ++f) {
      o[f] = ninf;
      a[f] = none_val<A>();
    }
    for (int32_t k = b; k < e; ++k) {
      const float* x = X + (int64_t)g->col[k] * ldx;
      const float w = g->ew ? g->ew[g->eslot ? g->eslot[k] : k] : 1.f;
      const A pos = (A)(k - b);
      for (int64_t f = 0; f < F; ++f) {
        const float m = g->ew ? x[f] * w : x[f];
        if (m > o[f]) {
          o[f] = m;
          a[f] = pos;
        }
      }
    }
    // DGL's _gspmm masks +-inf of a min/max reduce to 0 (replace_inf_with_zero)
    for (int64_t f = 0; f < F; ++f)
      if (std::isinf(o[f])) o[f] = 0.f;
  }
}

template <typename A>
void max_bwd(const pg_csr_t* g, const pg_csr_t* gt, const A* arg, int64_t lda, const float* dout,
             int64_t ldd, int64_t F, const float* mask, int64_t ldm, float* dx, int64_t ldx) {
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t u = 0; u < gt->n_rows; ++u) {
    float* d = dx + u * ldx;
    for (int64_t f = 0; f < F; ++f) d[f] = 0.f;
    for (int32_t t = gt->ptr[u]; t < gt->ptr[u + 1]; ++t) {
      const int32_t v = gt->col[t];
      const int32_t j = gt->eslot ? gt->eslot[t] : t;
      const A pos = (A)(j - g->ptr[v]);
      const float w = g->ew ? g->ew[j] : 1.f;
      const A* a = arg + (int64_t)v * lda;
      const float* go = dout + (int64_t)v * ldd;
      for (int64_t f = 0; f < F; ++f)
        if (a[f] == pos) d[f] += g->ew ? w * go[f] : go[f];
    }
    if (mask) {
      const float* m = mask + u * ldm;
      for (int64_t f = 0; f < F; ++f)
        if (!(m[f] > 0.f)) d[f] = 0.f;
    }
  }
}

}  // namespace

extern "C" {

int pg_spmm_max_fwd_cpu(const pg_csr_t* g, const float* X, int64_t ldx, int64_t F, float* out,
                        int64_t ldo, void* argpos, int64_t lda, int arg_kind) {
  PG_TRY(pg::check_csr(g, "pg_spmm_max_fwd_cpu", false));
  if (!pg::valid_arg_kind(arg_kind))
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_fwd_cpu: bad arg_kind %d", arg_kind);
  if (F < 0 || ldx < F || ldo < F || lda < F)
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_fwd_cpu: bad F/leading dims");
  if (arg_kind == PG_ARG_U16 && g->max_deg >= 0xFFFF)
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_fwd_cpu: degree too large for u16");
  if (arg_kind == PG_ARG_U16)
    max_fwd<uint16_t>(g, X, ldx, F, out, ldo, (uint16_t*)argpos, lda);
  else
    max_fwd<int32_t>(g, X, ldx, F, out, ldo, (int32_t*)argpos, lda);
  return pg::ok();
}

int pg_spmm_max_bwd_cpu(const pg_csr_t* g, const pg_csr_t* gt, const void* argpos, int64_t lda,
                        int arg_kind, const float* dout, int64_t ldd, int64_t F,
                        const float* mask_src, int64_t ldm, float* dx, int64_t ldx) {
  PG_TRY(pg::check_csr(g, "pg_spmm_max_bwd_cpu", false));
  PG_TRY(pg::check_csr(gt, "pg_spmm_max_bwd_cpu", false));
  if (!pg::valid_arg_kind(arg_kind))
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_bwd_cpu: bad arg_kind %d", arg_kind);
  if (F < 0 || ldd < F || ldx < F || lda < F || (mask_src && ldm < F))
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_bwd_cpu: bad F/leading dims");
  if (arg_kind == PG_ARG_U16)
    max_bwd<uint16_t>(g, gt, (const uint16_t*)argpos, lda, dout, ldd, F, mask_src, ldm, dx, ldx);
  else
    max_bwd<int32_t>(g, gt, (const int32_t*)argpos, lda, dout, ldd, F, mask_src, ldm, dx, ldx);
  return pg::ok();
}

int pg_spmm_sum_cpu(const pg_csr_t* g, const float* X, int64_t ldx, int64_t F, int norm_mode,
                    const int32_t* norm_ptr, float* out, int64_t ldo) {
  PG_TRY(pg::check_csr(g, "pg_spmm_sum_cpu", false));
  if (F < 0 || ldx < F || ldo < F)
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_sum_cpu: bad F/leading dims");
  if (norm_mode < 0 || norm_mode > 2 || (norm_mode == 2 && !norm_ptr))
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_sum_cpu: bad norm_mode");
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t r = 0; r < g->n_rows; ++r) {
    float* o = out + r * ldo;
    for (int64_t f = 0; f < F; ++f) o[f] = 0.f;
    const int32_t b = g->ptr[r], e = g->ptr[r + 1];
    for (int32_t k = b; k < e; ++k) {
      const int32_t c = g->col[k];
      const float* x = X + (int64_t)c * ldx;
      const float w = g->ew ? g->ew[g->eslot ? g->eslot[k] : k] : 1.f;
      const float dc = norm_mode == 2 ? (float)(norm_ptr[c + 1] - norm_ptr[c]) : 1.f;
      for (int64_t f = 0; f < F; ++f) {
        float t = g->ew ? x[f] * w : x[f];
        if (norm_mode == 2) t = t / dc;
        o[f] += t;
      }
    }
    if (norm_mode == 1 && e > b) {
      const float d = (float)(e - b);
      for (int64_t f = 0; f < F; ++f) o[f] = o[f] / d;
    }
  }
  return pg::ok();
}

int pg_argpos_to_src_cpu(const pg_csr_t* g, const void* argpos, int64_t lda, int arg_kind,
                         int64_t F, int64_t* argx, int64_t ldx) {
  PG_TRY(pg::check_csr(g, "pg_argpos_to_src_cpu", false));
  if (!pg::valid_arg_kind(arg_kind))
    return pg::set_error(PG_ERR_INVALID, "pg_argpos_to_src_cpu: bad arg_kind %d", arg_kind);
#pragma omp parallel for
  for (int64_t v = 0; v < g->n_rows; ++v) {
    for (int64_t f = 0; f < F; ++f) {
      int64_t p;
      if (arg_kind == PG_ARG_U16) {
        const uint16_t a = ((const uint16_t*)argpos)[v * lda + f];
        p = a == 0xFFFF ? -1 : (int64_t)a;
      } else {
        p = ((const int32_t*)argpos)[v * lda + f];
      }
      argx[v * ldx + f] = p < 0 ? -1 : (int64_t)g->col[g->ptr[v] + p];
    }
  }
  return pg::ok();
}

}  // extern "C"
