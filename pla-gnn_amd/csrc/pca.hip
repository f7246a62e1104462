// The PCA front end's heavy products (code/data_preprocess.py:475-487 `pca`, called at
// 528-546 on the ECC and GCN*PPI matrices): scikit-learn 1.1.1's PCA(n_components=250,
// random_state=42) takes the randomized-SVD path there (N = 24 041 >> 500, 250 < 0.8 N),
// whose cost is the power iteration Xc Q, Xc^T Q with Xc = X - 1 mean^T dense N x N
// (4.6 GB float64). X is sparse (<= the PPI's nonzeros), so each product is a float64
// CSR x dense SpMM plus a rank-1 centring term:
//   Y[r, :] = sum_{j in row r} val[j] * X[col[j], :]  -  u[r] * v[:]
// (u = 1, v = mean^T Q for Xc Q; u = mean, v = 1^T Q for Xc^T Q on the transposed CSR).
// One wave per row; each lane owns 2 consecutive columns (double2 when X is 16-B aligned
// with an even ldx) per 128-column chunk;
// the row's column ids / values come 64 at a time into VGPRs and are broadcast with
// v_readlane; 4 source rows in flight. The sum runs in CSR order (deterministic).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kMaxChunks = 4;  // k <= 512 columns

__device__ __forceinline__ int bcast_i(int v, int j) { return __builtin_amdgcn_readlane(v, j); }
__device__ __forceinline__ double bcast_d(double v, int j) {
  const int64_t b = __builtin_bit_cast(int64_t, v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), j);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), j);
  return __builtin_bit_cast(double, ((int64_t)hi << 32) | (uint32_t)lo);
}

template <int NCH>
__global__ __launch_bounds__(kBlock) void csr_spmm_f64_kernel(
    int64_t n_rows, const int32_t* __restrict__ ptr, const int32_t* __restrict__ col,
    const double* __restrict__ val, const double* __restrict__ X, int64_t ldx, int k,
    const double* __restrict__ u, const double* __restrict__ v, double* __restrict__ Y, int64_t ldy,
    bool vec) {
  constexpr int U = 4;
  const int64_t r = (int64_t)blockIdx.x * (kBlock / kWave) +
                    __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (r >= n_rows) return;
  const int lane = threadIdx.x & 63;
  const int k0 = ptr[r], k1 = ptr[r + 1];
  double acc[NCH][2];
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c][0] = acc[c][1] = 0.0;
  for (int kw = k0; kw < k1; kw += kWave) {
    const int nw = min(kWave, k1 - kw);
    const int kl = kw + min(lane, nw - 1);
    const int cv = col[kl];
    const double wv = val[kl];
    for (int j = 0; j < nw; j += U) {
      const int nv = min(U, nw - j);
      double x[U][NCH][2];
#pragma unroll
      for (int e = 0; e < U; ++e) {
        const double* xr = X + (int64_t)bcast_i(cv, j + min(e, nv - 1)) * ldx;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const int f = (c * kWave + lane) * 2;
          if (vec && f + 1 < k) {
            const double2 t = *reinterpret_cast<const double2*>(xr + f);
            x[e][c][0] = t.x;
            x[e][c][1] = t.y;
          } else {
            x[e][c][0] = f < k ? xr[f] : 0.0;
            x[e][c][1] = f + 1 < k ? xr[f + 1] : 0.0;
          }
        }
      }
#pragma unroll
      for (int e = 0; e < U; ++e) {
        if (e < nv) {
          const double w = bcast_d(wv, j + e);
#pragma unroll
          for (int c = 0; c < NCH; ++c) {
            acc[c][0] = fma(w, x[e][c][0], acc[c][0]);
            acc[c][1] = fma(w, x[e][c][1], acc[c][1]);
          }
        }
      }
    }
  }
  const double ur = u ? u[r] : 1.0;
  double* yr = Y + r * ldy;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int f = (c * kWave + lane) * 2;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      if (f + i < k) yr[f + i] = v ? acc[c][i] - ur * v[f + i] : acc[c][i];
  }
}

}  // namespace

extern "C" {

int pg_csr_spmm_f64(int64_t n_rows, const int32_t* ptr, const int32_t* col, const double* val,
                    const double* X, int64_t ldx, int64_t k, const double* u, const double* v,
                    double* Y, int64_t ldy, pg_stream_t stream) {
  if (n_rows < 0 || k < 0 || k > 2 * kWave * kMaxChunks || ldx < k || ldy < k)
    return pg::set_error(PG_ERR_INVALID, "pg_csr_spmm_f64: bad sizes (k <= %d)", 2 * kWave * kMaxChunks);
  if (n_rows == 0 || k == 0) return pg::ok();
  if (!ptr || !X || !Y) return pg::set_error(PG_ERR_INVALID, "pg_csr_spmm_f64: NULL buffer");
  const bool vec = ((uintptr_t)X & 15) == 0 && (ldx & 1) == 0;  // double2 loads
  const int nch = (int)((k + 2 * kWave - 1) / (2 * kWave));
  const unsigned blocks = (unsigned)((n_rows + 3) / 4);
  hipStream_t st = (hipStream_t)stream;
#define PG_L(N_)                                                                                    \
  hipLaunchKernelGGL(csr_spmm_f64_kernel<N_>, dim3(blocks), dim3(kBlock), 0, st, n_rows, ptr, col, \
                     val, X, ldx, (int)k, u, v, Y, ldy, vec)
  switch (nch) {
    case 1: PG_L(1); break;
    case 2: PG_L(2); break;
    case 3: PG_L(3); break;
    default: PG_L(4); break;
  }
#undef PG_L
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pg::set_error((int)e, "pg_csr_spmm_f64: launch failed: %s", hipGetErrorString(e));
  return pg::ok();
}

}  // extern "C"
