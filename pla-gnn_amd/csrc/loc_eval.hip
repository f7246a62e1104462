// Per-epoch evaluation of the reference on the GPU:
//   protein_loc_correction (code/train.py:19-39): column min-max normalisation, row-sum
//     normalisation, per-row threshold max - (max - min) * alpha, pred = new > threshold;
//   performances_record (code/train.py:42-86): per-row |T∩P|/|P| (aim), |T∩P|/|T|
//     (coverage), |T∩P|/|T∪P| (accuracy), summed over rows as float32 in row order and
//     divided by n, exactly as the reference's running torch float32 scalars.
// The reference runs both as Python loops over the N rows with a device->host copy each
// epoch; here they are three small kernels and one 3-double result.
// Float32 operation order follows the reference element-wise; the row sum of the 12
// normalised scores runs in column order (torch-CPU's vectorised sum may associate
// differently: the last bit of a normalised score can differ, never observed to flip a
// prediction on the reference fixtures).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "common.hpp"

namespace {

constexpr int kBlock = 256;
constexpr int kRowsPerPart = 256;

// per-column partial min / max over row chunks: part[b][c] = {min, max}
__global__ __launch_bounds__(kBlock) void col_minmax_part_kernel(const float* __restrict__ p,
                                                                 int64_t ldp, int64_t n, int C,
                                                                 float2* __restrict__ part) {
  __shared__ float smin[kBlock], smax[kBlock];
  const int c = threadIdx.x % C, g = threadIdx.x / C, G = kBlock / C;
  const int64_t r0 = (int64_t)blockIdx.x * kRowsPerPart;
  const int64_t r1 = std::min<int64_t>(n, r0 + kRowsPerPart);
  float mn = INFINITY, mx = -INFINITY;
  if (g < G) {
    // four rows' loads in flight per iteration (min / max are order-free)
    int64_t r = r0 + g;
    for (; r + 3 * G < r1; r += 4 * G) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = p[(r + e * G) * ldp + c];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        mn = fminf(mn, v[e]);
        mx = fmaxf(mx, v[e]);
      }
    }
    for (; r < r1; r += G) {
      const float v = p[r * ldp + c];
      mn = fminf(mn, v);
      mx = fmaxf(mx, v);
    }
  }
  smin[threadIdx.x] = mn;
  smax[threadIdx.x] = mx;
  __syncthreads();
  if ((int)threadIdx.x < C) {
    for (int q = 1; q < G; ++q) {
      mn = fminf(mn, smin[q * C + threadIdx.x]);
      mx = fmaxf(mx, smax[q * C + threadIdx.x]);
    }
    part[(int64_t)blockIdx.x * C + threadIdx.x] = make_float2(mn, mx);
  }
}

// CT: the class count at compile time (the per-row arrays then live in registers; with a
// run-time count they went to scratch memory), or 0
template <int CT>
__global__ __launch_bounds__(kBlock) void loc_correction_kernel(
    const float* __restrict__ p, int64_t ldp, int64_t n, int Cr, const float2* __restrict__ part,
    int nparts, float alpha, double* __restrict__ pred, int64_t ldpred) {
  const int C = CT > 0 ? CT : Cr;
  constexpr int VN = CT > 0 ? CT : 64;
  __shared__ float cmin[64], cmax[64];
  if ((int)threadIdx.x < C) {
    float mn = INFINITY, mx = -INFINITY;
    for (int b = 0; b < nparts; ++b) {
      const float2 t = part[(int64_t)b * C + threadIdx.x];
      mn = fminf(mn, t.x);
      mx = fmaxf(mx, t.y);
    }
    cmin[threadIdx.x] = mn;
    cmax[threadIdx.x] = mx;
  }
  __syncthreads();
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= n) return;
  float v[VN];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    v[c] = (p[r * ldp + c] - cmin[c]) / (cmax[c] - cmin[c]);
    s = s + v[c];
  }
  float rmax = -INFINITY, rmin = INFINITY;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    v[c] = v[c] / s;
    rmax = fmaxf(rmax, v[c]);
    rmin = fminf(rmin, v[c]);
  }
  const float th = rmax - (rmax - rmin) * alpha;
#pragma unroll
  for (int c = 0; c < C; ++c) pred[r * ldpred + c] = v[c] > th ? 1.0 : 0.0;
}

// per row: {aim_i, cov_i, acc_i} as the reference's float32 divisions (aim_i = 0 when
// nothing is predicted)
__global__ __launch_bounds__(kBlock) void loc_perf_rows_kernel(const float* __restrict__ t,
                                                               int64_t ldt,
                                                               const double* __restrict__ pr,
                                                               int64_t ldp, int64_t n, int C,
                                                               float* __restrict__ rows) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= n) return;
  int a = 0, pc = 0, tc = 0, o = 0;
  for (int c = 0; c < C; ++c) {
    // loc.long() == 1 (a float label / prediction truncated towards zero)
    const bool tt = (long long)t[r * ldt + c] == 1;
    const bool pp = (long long)pr[r * ldp + c] == 1;
    a += tt && pp;
    pc += pp;
    tc += tt;
    o += tt || pp;
  }
  const float fa = (float)a;
  rows[3 * r + 0] = pc == 0 ? 0.f : fa / (float)pc;
  rows[3 * r + 1] = fa / (float)tc;
  rows[3 * r + 2] = fa / (float)o;
}

// running float32 sums in row order (one lane per metric), then / n. The per-row values
// stream through LDS in chunks loaded by waves 1-3 (many loads in flight, the next chunk
// while the current one is summed); wave 0's lanes 0-2 keep the three dependent add chains
// (a chain fed straight from global memory waited out one load latency per 8 rows).
constexpr int kSumChunk = 2048;  // rows per LDS chunk (2 x 24 KB)
__global__ __launch_bounds__(256) void loc_perf_sum_kernel(const float* __restrict__ rows, int64_t n,
                                                           double* __restrict__ out) {
  __shared__ float buf[2][kSumChunk * 3];
  const int t = threadIdx.x;
  const int64_t nch = (n + kSumChunk - 1) / kSumChunk;
  auto load = [&](int64_t c) {
    if (t < 64) return;
    const int64_t r0 = c * kSumChunk;
    const int cnt = (int)min<int64_t>(kSumChunk, n - r0) * 3;
    float* b = buf[c & 1];
    for (int i = t - 64; i < cnt; i += 192) b[i] = rows[3 * r0 + i];
  };
  float s = 0.f;
  load(0);
  __syncthreads();
  for (int64_t c = 0; c < nch; ++c) {
    if (c + 1 < nch) load(c + 1);
    if (t < 3) {
      const float* b = buf[c & 1];
      const int cnt = (int)min<int64_t>(kSumChunk, n - c * kSumChunk);
      int i = 0;
      for (; i + 8 <= cnt; i += 8) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = b[3 * (i + e) + t];
#pragma unroll
        for (int e = 0; e < 8; ++e) s = s + v[e];
      }
      for (; i < cnt; ++i) s = s + b[3 * i + t];
    }
    __syncthreads();
  }
  if (t < 3) out[t] = (double)(s / (float)n);
}

}  // namespace

extern "C" {

size_t pg_loc_eval_workspace(int64_t n, int32_t C) {
  const int64_t parts = std::max<int64_t>(1, (n + kRowsPerPart - 1) / kRowsPerPart);
  return (size_t)(parts * std::max(C, 1) * 8 + 3 * std::max<int64_t>(n, 1) * 4 + 256);
}

int pg_loc_correction(const float* proba, int64_t ldp, int64_t n, int32_t C, double alpha,
                      double* pred, int64_t ldpred, void* ws, size_t ws_bytes, pg_stream_t stream) {
  if (n < 0 || C <= 0 || C > 64 || ldp < C || ldpred < C)
    return pg::set_error(PG_ERR_INVALID, "pg_loc_correction: bad shape");
  if (n == 0) return pg::ok();
  if (!proba || !pred || !ws) return pg::set_error(PG_ERR_INVALID, "pg_loc_correction: NULL buffer");
  if (ws_bytes < pg_loc_eval_workspace(n, C))
    return pg::set_error(PG_ERR_WORKSPACE, "pg_loc_correction: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int parts = (int)((n + kRowsPerPart - 1) / kRowsPerPart);
  float2* part = (float2*)ws;
  hipLaunchKernelGGL(col_minmax_part_kernel, dim3(parts), dim3(kBlock), 0, st, proba, ldp, n, (int)C, part);
  // torch multiplies a float32 tensor by the Python float alpha in float32
  const dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
  if (C == 12)  // the reference's 12 subcellular locations
    hipLaunchKernelGGL(loc_correction_kernel<12>, grid, dim3(kBlock), 0, st, proba, ldp, n, (int)C,
                       (const float2*)part, parts, (float)alpha, pred, ldpred);
  else
    hipLaunchKernelGGL(loc_correction_kernel<0>, grid, dim3(kBlock), 0, st, proba, ldp, n, (int)C,
                       (const float2*)part, parts, (float)alpha, pred, ldpred);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pg::set_error((int)e, "pg_loc_correction: %s", hipGetErrorString(e));
  return pg::ok();
}

int pg_loc_performance(const float* loc_true, int64_t ldt, const double* loc_pred, int64_t ldp,
                       int64_t n, int32_t C, double* out3, void* ws, size_t ws_bytes,
                       pg_stream_t stream) {
  if (n <= 0 || C <= 0 || C > 64 || ldt < C || ldp < C)
    return pg::set_error(PG_ERR_INVALID, "pg_loc_performance: bad shape");
  if (!loc_true || !loc_pred || !out3 || !ws)
    return pg::set_error(PG_ERR_INVALID, "pg_loc_performance: NULL buffer");
  if (ws_bytes < pg_loc_eval_workspace(n, C))
    return pg::set_error(PG_ERR_WORKSPACE, "pg_loc_performance: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* rows = (float*)ws;
  hipLaunchKernelGGL(loc_perf_rows_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                     loc_true, ldt, loc_pred, ldp, n, (int)C, rows);
  hipLaunchKernelGGL(loc_perf_sum_kernel, dim3(1), dim3(256), 0, st, (const float*)rows, n, out3);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pg::set_error((int)e, "pg_loc_performance: %s", hipGetErrorString(e));
  return pg::ok();
}

}  // extern "C"
