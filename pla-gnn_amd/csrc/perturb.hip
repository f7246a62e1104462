// Topology perturbation on the GPU: the reference's
//   construct_gcn_matrix   (code/data_preprocess.py:128-172): Pearson correlation of the
//                           expression rows, np.corrcoef + fill_diagonal(0) + nan -> 0
//   modify_network_topology(code/data_preprocess.py:217-257): diff = pcc_inter - pcc_normal
//                           over all N x N entries, its mean / std, then
//                           drop edge (i, j) if ppi == 1 and diff < mean - thr * std,
//                           add  edge (i, j) if ppi == 0 and diff > mean + thr * std
// fused: the two N x N float64 correlation matrices (2 x 4.6 GB at N = 24 041) and their
// difference are never materialised. Every pass recomputes diff(i, j) from the centred
// expression rows (N x S, S samples: the whole working set is ~1.5 MB and stays in L2),
// so the kernels are f64-VALU bound, not memory bound.
//
// Pearson entry, as numpy computes it (np.cov -> dot -> corrcoef, numpy 2.2 + OpenBLAS):
//   xc   = x - mean(x)                   mean = ((x0 + x1) + x2 ...) / S   (host side)
//   dot  = fma(a[S-1], b[S-1], ... fma(a[1], b[1], a[0] * b[0]))  (OpenBLAS dgemm order)
//   c    = dot * (1 / (S - 1)); c = c / sd_i; c = c / sd_j;  clip to [-1, 1] (NaN kept)
//   c    = 0 on the diagonal and where NaN (zero-variance rows)
//   sd_i = sqrt(dot(xc_i, xc_i) * (1 / (S - 1)))
// Passes (each one workgroup per row i, threads over j):
//   pg_perturb_prepare : sd of every row, both states
//   pg_perturb_sum     : per-row compensated sums of diff (pass 1: mean) or of
//                        (diff - mean)^2 (pass 2: variance), then one ordered final
//                        reduction (deterministic)
//   pg_perturb_count   : per-row count of non-zero entries of the perturbed adjacency
//   pg_perturb_fill    : the entries themselves, row-major with ascending columns (the
//                        order of scipy's coo_matrix(dense)), column ids + int64 values
// Row i's adjacency lives in an LDS bitmap (non-zero set); a stored value other than 1 is
// looked up in the row (binary search): both rules only fire on values 0 and 1.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "common.hpp"

namespace {

constexpr int kBlock = 256;
constexpr int kMaxS = 8;
constexpr int kMaxBitmapWords = 160 * 1024 / 4;

struct Rows {
  const double* xn;  // [n][S] centred expression, normal state
  const double* xi;  // [n][S] intervention state
  const double* sdn; // [n]
  const double* sdi; // [n]
};

template <int S>
__device__ __forceinline__ double dot_rows(const double* __restrict__ a, const double* __restrict__ b) {
  double d = a[0] * b[0];
#pragma unroll
  for (int s = 1; s < S; ++s) d = fma(a[s], b[s], d);
  return d;
}

template <int S>
__device__ __forceinline__ double pcc(const double* __restrict__ xa, double sda,
                                      const double* __restrict__ xb, double sdb, double inv_fact,
                                      bool diag) {
  double c = dot_rows<S>(xa, xb) * inv_fact;
  c = c / sda;
  c = c / sdb;
  if (c < -1.0) c = -1.0;
  else if (c > 1.0) c = 1.0;
  if (diag || c != c) c = 0.0;
  return c;
}

// diff(i, j) = pcc_inter(i, j) - pcc_normal(i, j): the sparse subtraction of the
// reference gives exactly the dense difference (x - 0 = x, 0 - y = -y)
template <int S>
__device__ __forceinline__ double diff_ij(const Rows& r, const double (&xni)[S], double sdni,
                                          const double (&xii)[S], double sdii, int i, int j,
                                          double inv_fact) {
  double xnj[S], xij[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    xnj[s] = r.xn[(int64_t)j * S + s];
    xij[s] = r.xi[(int64_t)j * S + s];
  }
  const bool diag = i == j;
  const double pn = pcc<S>(xni, sdni, xnj, r.sdn[j], inv_fact, diag);
  const double pi = pcc<S>(xii, sdii, xij, r.sdi[j], inv_fact, diag);
  return pi - pn;
}

template <int S>
__device__ __forceinline__ void load_row(const double* __restrict__ x, int i, double (&o)[S]) {
#pragma unroll
  for (int s = 0; s < S; ++s) o[s] = x[(int64_t)i * S + s];
}

// Neumaier compensated accumulation (s, c): s + c is the running sum
__device__ __forceinline__ void kadd(double& s, double& c, double x) {
  const double t = s + x;
  if (fabs(s) >= fabs(x)) c += (s - t) + x;
  else c += (x - t) + s;
  s = t;
}

template <int S>
__global__ __launch_bounds__(kBlock) void prepare_kernel(const double* __restrict__ xn,
                                                         const double* __restrict__ xi, int n,
                                                         double inv_fact, double* __restrict__ sdn,
                                                         double* __restrict__ sdi) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  double a[S];
  load_row<S>(xn, i, a);
  sdn[i] = sqrt(dot_rows<S>(a, a) * inv_fact);
  load_row<S>(xi, i, a);
  sdi[i] = sqrt(dot_rows<S>(a, a) * inv_fact);
}

// one workgroup per row: part[2 i + {0, 1}] = compensated sum over j of diff (SQ = false)
// or of (diff - mean)^2 (SQ = true)
template <int S, bool SQ>
__global__ __launch_bounds__(kBlock) void sum_kernel(Rows r, int n, double inv_fact, double mean,
                                                     double* __restrict__ part) {
  __shared__ double red[2][kBlock];
  const int i = blockIdx.x;
  double xni[S], xii[S];
  load_row<S>(r.xn, i, xni);
  load_row<S>(r.xi, i, xii);
  const double sdni = r.sdn[i], sdii = r.sdi[i];
  double s = 0.0, c = 0.0;
  for (int j = threadIdx.x; j < n; j += kBlock) {
    double d = diff_ij<S>(r, xni, sdni, xii, sdii, i, j, inv_fact);
    if constexpr (SQ) {
      d = d - mean;
      d = d * d;
    }
    kadd(s, c, d);
  }
  red[0][threadIdx.x] = s;
  red[1][threadIdx.x] = c;
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      double a = red[0][threadIdx.x], ac = red[1][threadIdx.x];
      kadd(a, ac, red[0][threadIdx.x + w]);
      ac += red[1][threadIdx.x + w];
      red[0][threadIdx.x] = a;
      red[1][threadIdx.x] = ac;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * (int64_t)i] = red[0][0];
    part[2 * (int64_t)i + 1] = red[1][0];
  }
}

// ordered final reduction of the per-row partials: out[0] = total (s + c)
__global__ __launch_bounds__(kBlock) void final_sum_kernel(const double* __restrict__ part, int n,
                                                           double* __restrict__ out) {
  __shared__ double red[2][kBlock];
  double s = 0.0, c = 0.0;
  // thread t sums a contiguous run of rows in order
  const int per = (n + kBlock - 1) / kBlock;
  const int a = threadIdx.x * per, b = min(n, a + per);
  for (int i = a; i < b; ++i) {
    kadd(s, c, part[2 * (int64_t)i]);
    c += part[2 * (int64_t)i + 1];
  }
  red[0][threadIdx.x] = s;
  red[1][threadIdx.x] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0, tc = 0.0;
    for (int k = 0; k < kBlock; ++k) {
      kadd(t, tc, red[0][k]);
      tc += red[1][k];
    }
    out[0] = t + tc;
  }
}

// row i's stored entries -> LDS bitmap of the non-zero columns
__device__ __forceinline__ void build_bitmap(uint32_t* bits, int words, const int32_t* __restrict__ ptr,
                                             const int32_t* __restrict__ col,
                                             const int64_t* __restrict__ val, int i) {
  for (int w = threadIdx.x; w < words; w += kBlock) bits[w] = 0u;
  __syncthreads();
  for (int k = ptr[i] + threadIdx.x; k < ptr[i + 1]; k += kBlock) {
    if (val && val[k] == 0) continue;
    const int c = col[k];
    atomicOr(&bits[c >> 5], 1u << (c & 31));
  }
  __syncthreads();
}

// the stored value of (i, j) (0 if absent): 1 unless a value array says otherwise
__device__ __forceinline__ int64_t ppi_value(const uint32_t* bits, const int32_t* __restrict__ ptr,
                                             const int32_t* __restrict__ col,
                                             const int64_t* __restrict__ val, int i, int j) {
  if (!((bits[j >> 5] >> (j & 31)) & 1u)) return 0;
  if (!val) return 1;
  int lo = ptr[i], hi = ptr[i + 1] - 1;  // sorted, unique columns
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (col[mid] < j) lo = mid + 1;
    else hi = mid;
  }
  return val[lo];
}

template <int S>
__device__ __forceinline__ int64_t new_value(const Rows& r, const uint32_t* bits,
                                             const int32_t* __restrict__ ptr,
                                             const int32_t* __restrict__ col,
                                             const int64_t* __restrict__ val, const double (&xni)[S],
                                             double sdni, const double (&xii)[S], double sdii, int i,
                                             int j, double inv_fact, double lo_thr, double hi_thr) {
  const int64_t v = ppi_value(bits, ptr, col, val, i, j);
  if (v != 0 && v != 1) return v;
  const double d = diff_ij<S>(r, xni, sdni, xii, sdii, i, j, inv_fact);
  if (v == 1 && d < lo_thr) return 0;  // res1 (data_preprocess.py:248)
  if (v == 0 && d > hi_thr) return 1;  // res2 (data_preprocess.py:249)
  return v;
}

template <int S>
__global__ __launch_bounds__(kBlock) void count_kernel(Rows r, const int32_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ col,
                                                       const int64_t* __restrict__ val, int n,
                                                       int words, double inv_fact, double lo_thr,
                                                       double hi_thr, int32_t* __restrict__ counts) {
  extern __shared__ uint32_t bits[];
  __shared__ int wsum[kBlock / 64];
  const int i = blockIdx.x;
  build_bitmap(bits, words, ptr, col, val, i);
  double xni[S], xii[S];
  load_row<S>(r.xn, i, xni);
  load_row<S>(r.xi, i, xii);
  const double sdni = r.sdn[i], sdii = r.sdi[i];
  int cnt = 0;
  for (int j = threadIdx.x; j < n; j += kBlock)
    cnt += new_value<S>(r, bits, ptr, col, val, xni, sdni, xii, sdii, i, j, inv_fact, lo_thr, hi_thr) != 0;
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += wsum[w];
    counts[i] = t;
  }
}

template <int S>
__global__ __launch_bounds__(kBlock) void fill_kernel(Rows r, const int32_t* __restrict__ ptr,
                                                      const int32_t* __restrict__ col,
                                                      const int64_t* __restrict__ val, int n,
                                                      int words, double inv_fact, double lo_thr,
                                                      double hi_thr, const int64_t* __restrict__ offs,
                                                      int32_t* __restrict__ out_col,
                                                      int64_t* __restrict__ out_val) {
  extern __shared__ uint32_t bits[];
  __shared__ int wcnt[kBlock / 64];
  const int i = blockIdx.x;
  build_bitmap(bits, words, ptr, col, val, i);
  double xni[S], xii[S];
  load_row<S>(r.xn, i, xni);
  load_row<S>(r.xi, i, xii);
  const double sdni = r.sdn[i], sdii = r.sdi[i];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t base = offs[i];
  // tiles of kBlock consecutive columns; entries are placed in column order
  for (int j0 = 0; j0 < n; j0 += kBlock) {
    const int j = j0 + threadIdx.x;
    int64_t v = 0;
    if (j < n) v = new_value<S>(r, bits, ptr, col, val, xni, sdni, xii, sdii, i, j, inv_fact, lo_thr, hi_thr);
    const unsigned long long m = __ballot(v != 0);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wcnt[wave] = __popcll(m);
    __syncthreads();
    int wbase = 0, tot = 0;
    for (int w = 0; w < kBlock / 64; ++w) {
      if (w < wave) wbase += wcnt[w];
      tot += wcnt[w];
    }
    if (v != 0) {
      out_col[base + wbase + before] = j;
      out_val[base + wbase + before] = v;
    }
    base += tot;
    __syncthreads();
  }
}

inline int check_s(int S) { return S >= 2 && S <= kMaxS; }

#define PG_S_DISPATCH(S_, CALL)             \
  switch (S_) {                             \
    case 2: { constexpr int S = 2; CALL; } break; \
    case 3: { constexpr int S = 3; CALL; } break; \
    case 4: { constexpr int S = 4; CALL; } break; \
    case 5: { constexpr int S = 5; CALL; } break; \
    case 6: { constexpr int S = 6; CALL; } break; \
    case 7: { constexpr int S = 7; CALL; } break; \
    default: { constexpr int S = 8; CALL; } break; \
  }

inline int launch_result(const char* who) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pg::set_error((int)e, "%s: launch failed: %s", who, hipGetErrorString(e));
  return pg::ok();
}

}  // namespace

extern "C" {

size_t pg_perturb_workspace(int64_t n) { return n <= 0 ? 0 : (size_t)(2 * n + 8) * sizeof(double); }

int pg_perturb_prepare(const double* xc_normal, const double* xc_inter, int64_t n, int32_t S,
                       double inv_fact, double* sd_normal, double* sd_inter, pg_stream_t stream) {
  if (n < 0 || n > INT32_MAX || !check_s(S))
    return pg::set_error(PG_ERR_INVALID, "pg_perturb_prepare: n in [0, 2^31), 2 <= S <= %d", kMaxS);
  if (n == 0) return pg::ok();
  if (!xc_normal || !xc_inter || !sd_normal || !sd_inter)
    return pg::set_error(PG_ERR_INVALID, "pg_perturb_prepare: NULL buffer");
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
  PG_S_DISPATCH(S, hipLaunchKernelGGL((prepare_kernel<S>), grid, dim3(kBlock), 0, st, xc_normal,
                                      xc_inter, (int)n, inv_fact, sd_normal, sd_inter));
  return launch_result("pg_perturb_prepare");
}

int pg_perturb_sum(const double* xc_normal, const double* xc_inter, const double* sd_normal,
                   const double* sd_inter, int64_t n, int32_t S, double inv_fact, int squared,
                   double mean, double* total, void* ws, size_t ws_bytes, pg_stream_t stream) {
  if (n < 0 || n > INT32_MAX || !check_s(S))
    return pg::set_error(PG_ERR_INVALID, "pg_perturb_sum: n in [0, 2^31), 2 <= S <= %d", kMaxS);
  if (!total) return pg::set_error(PG_ERR_INVALID, "pg_perturb_sum: NULL total");
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    (void)hipMemsetAsync(total, 0, sizeof(double), st);
    return launch_result("pg_perturb_sum");
  }
  if (!xc_normal || !xc_inter || !sd_normal || !sd_inter)
    return pg::set_error(PG_ERR_INVALID, "pg_perturb_sum: NULL buffer");
  if (!ws || ws_bytes < pg_perturb_workspace(n))
    return pg::set_error(PG_ERR_WORKSPACE, "pg_perturb_sum: workspace too small");
  const Rows r{xc_normal, xc_inter, sd_normal, sd_inter};
  double* part = (double*)ws;
  if (squared) {
    PG_S_DISPATCH(S, hipLaunchKernelGGL((sum_kernel<S, true>), dim3((unsigned)n), dim3(kBlock), 0, st, r,
                                        (int)n, inv_fact, mean, part));
  } else {
    PG_S_DISPATCH(S, hipLaunchKernelGGL((sum_kernel<S, false>), dim3((unsigned)n), dim3(kBlock), 0, st, r,
                                        (int)n, inv_fact, mean, part));
  }
  hipLaunchKernelGGL(final_sum_kernel, dim3(1), dim3(kBlock), 0, st, (const double*)part, (int)n, total);
  return launch_result("pg_perturb_sum");
}

int pg_perturb_count(const double* xc_normal, const double* xc_inter, const double* sd_normal,
                     const double* sd_inter, int64_t n, int32_t S, double inv_fact,
                     const int32_t* ptr, const int32_t* col, const int64_t* val, double lo_thr,
                     double hi_thr, int32_t* counts, pg_stream_t stream) {
  const int64_t words = (n + 31) / 32;
  if (n < 0 || n > INT32_MAX || !check_s(S) || words > kMaxBitmapWords)
    return pg::set_error(PG_ERR_INVALID, "pg_perturb_count: n in [0, %d], 2 <= S <= %d",
                         kMaxBitmapWords * 32, kMaxS);
  if (n == 0) return pg::ok();
  if (!xc_normal || !xc_inter || !sd_normal || !sd_inter || !ptr || !counts)
    return pg::set_error(PG_ERR_INVALID, "pg_perturb_count: NULL buffer");
  hipStream_t st = (hipStream_t)stream;
  const Rows r{xc_normal, xc_inter, sd_normal, sd_inter};
  const size_t lds = (size_t)words * 4;
  PG_S_DISPATCH(S, {
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)count_kernel<S>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
    hipLaunchKernelGGL((count_kernel<S>), dim3((unsigned)n), dim3(kBlock), lds, st, r, ptr, col, val,
                       (int)n, (int)words, inv_fact, lo_thr, hi_thr, counts);
  });
  return launch_result("pg_perturb_count");
}

int pg_perturb_fill(const double* xc_normal, const double* xc_inter, const double* sd_normal,
                    const double* sd_inter, int64_t n, int32_t S, double inv_fact,
                    const int32_t* ptr, const int32_t* col, const int64_t* val, double lo_thr,
                    double hi_thr, const int64_t* offsets, int32_t* out_col, int64_t* out_val,
                    pg_stream_t stream) {
  const int64_t words = (n + 31) / 32;
  if (n < 0 || n > INT32_MAX || !check_s(S) || words > kMaxBitmapWords)
    return pg::set_error(PG_ERR_INVALID, "pg_perturb_fill: n in [0, %d], 2 <= S <= %d",
                         kMaxBitmapWords * 32, kMaxS);
  if (n == 0) return pg::ok();
  if (!xc_normal || !xc_inter || !sd_normal || !sd_inter || !ptr || !offsets || !out_col || !out_val)
    return pg::set_error(PG_ERR_INVALID, "pg_perturb_fill: NULL buffer");
  hipStream_t st = (hipStream_t)stream;
  const Rows r{xc_normal, xc_inter, sd_normal, sd_inter};
  const size_t lds = (size_t)words * 4;
  PG_S_DISPATCH(S, {
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)fill_kernel<S>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
    hipLaunchKernelGGL((fill_kernel<S>), dim3((unsigned)n), dim3(kBlock), lds, st, r, ptr, col, val,
                       (int)n, (int)words, inv_fact, lo_thr, hi_thr, offsets, out_col, out_val);
  });
  return launch_result("pg_perturb_fill");
}

}  // extern "C"
