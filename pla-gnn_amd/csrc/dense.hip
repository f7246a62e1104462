// Dense helpers of the PLA-GNN training step on gfx950: fused bias + activation
// (nn.Linear bias, F.relu of SAGEConv's fc_pool, F.leaky_relu of code/model.py:21-27),
// activation backward, deterministic column sums (bias gradients), the fused
// sigmoid + multi_loss forward/backward (code/model.py:29, code/train.py:89-108), and
// Adam (code/train.py:180, 205; torch 1.10 update order).
// Everything is written to be capturable in a HIP graph: no host sync, no allocation,
// the Adam step counter lives in device memory.
#include <hip/hip_runtime.h>

#include <cmath>

#include "adam_step.hpp"
#include "common.hpp"

namespace {

constexpr int kBlock = 256;

inline int hip_status(const char* who) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return pg::set_error((int)e, "%s: launch failed: %s", who, hipGetErrorString(e));
  return pg::ok();
}

inline int grid_1d(int64_t n, int cap = 8192) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(cap, (n + kBlock - 1) / kBlock));
}

template <int ACT>
__device__ __forceinline__ float act_fwd(float x, float slope) {
  if constexpr (ACT == PG_ACT_RELU) return x > 0.f ? x : 0.f;
  else if constexpr (ACT == PG_ACT_LEAKY) return x > 0.f ? x : x * slope;
  else return x;
}

template <int ACT>
__global__ __launch_bounds__(kBlock) void bias_act_kernel(float* __restrict__ y, int64_t ldy,
                                                          int64_t rows, int cols,
                                                          const float* __restrict__ bias,
                                                          float slope) {
  const int64_t n = rows * (int64_t)cols;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t r = i / cols;
    const int c = (int)(i - r * cols);
    float v = y[r * ldy + c];
    if (bias) v = v + bias[c];
    y[r * ldy + c] = act_fwd<ACT>(v, slope);
  }
}

template <int ACT>
__global__ __launch_bounds__(kBlock) void act_bwd_kernel(float* __restrict__ dy, int64_t lddy,
                                                         const float* __restrict__ y, int64_t ldy,
                                                         int64_t rows, int cols, float slope) {
  const int64_t n = rows * (int64_t)cols;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t r = i / cols;
    const int c = (int)(i - r * cols);
    const float yy = y[r * ldy + c];
    float g = dy[r * lddy + c];
    if constexpr (ACT == PG_ACT_RELU) g = yy > 0.f ? g : 0.f;
    else if constexpr (ACT == PG_ACT_LEAKY) g = yy > 0.f ? g : g * slope;
    dy[r * lddy + c] = g;
  }
}

// column sums, pass 1: block (cx, ry) owns 64 columns x one chunk of rows; its 4 waves
// take interleaved rows with 8 loads in flight per lane, then combine in wave order.
constexpr int kColRowChunks = 128;
__global__ __launch_bounds__(kBlock) void col_sum_part_kernel(const float* __restrict__ x,
                                                              int64_t ldx, int64_t rows,
                                                              int cols,
                                                              float* __restrict__ part) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  const int64_t per = (rows + gridDim.y - 1) / gridDim.y;
  const int64_t r0 = (int64_t)blockIdx.y * per;
  const int64_t r1 = min(rows, r0 + per);
  float s = 0.f;
  if (c < cols) {
    int64_t r = r0 + g;
    for (; r + 28 < r1; r += 32) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = x[(r + 4 * e) * ldx + c];
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[e];
    }
    for (; r < r1; r += 4) s += x[r * ldx + c];
  }
  red[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0 && c < cols) {
    const int l = threadIdx.x & 63;
    part[(int64_t)blockIdx.y * cols + c] = ((red[0][l] + red[1][l]) + red[2][l]) + red[3][l];
  }
}

__global__ __launch_bounds__(kBlock) void col_sum_final_kernel(const float* __restrict__ part,
                                                               int R, int cols,
                                                               float* __restrict__ out,
                                                               int accumulate) {
  const int c = blockIdx.x * kBlock + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
  for (int r = 0; r < R; r += 8) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = r + e < R ? part[(int64_t)(r + e) * cols + c] : 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[e];
  }
  out[c] = accumulate ? out[c] + s : s;
}

// ---- sigmoid + multi_loss -----------------------------------------------------------
// pass 1: prob = sigmoid(z) everywhere, dz = 0 everywhere
__global__ __launch_bounds__(kBlock) void sigmoid_zero_kernel(const float* __restrict__ z,
                                                              int64_t ldz, int64_t rows, int C,
                                                              float* __restrict__ prob,
                                                              int64_t ldp, float* __restrict__ dz,
                                                              int64_t lddz) {
  const int64_t n = rows * (int64_t)C;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t r = i / C;
    const int c = (int)(i - r * C);
    if (prob) prob[r * ldp + c] = 1.f / (1.f + expf(-z[r * ldz + c]));
    if (dz) dz[r * lddz + c] = 0.f;
  }
}

// pass 2: block b owns indexed rows [b*R, b*R+R), R = 256 / C; one thread per (row, class)
// pair writes the pair's loss term into LDS and its gradient into dz; then thread c < C
// sums its class over the block's rows in row order (deterministic), giving part[b][c].
// Mirrors the autograd graph of code/train.py:103-104 operation by operation.
inline __host__ __device__ int loss_rows(int C) { return C >= kBlock ? 1 : kBlock / C; }
__global__ __launch_bounds__(kBlock) void multi_loss_kernel(
    const float* __restrict__ z, int64_t ldz, int C, const float* __restrict__ labels,
    int64_t ldl, const float* __restrict__ cw, const int32_t* __restrict__ index, int64_t n_index,
    float* __restrict__ part, float* __restrict__ dz, int64_t lddz) {
  __shared__ float terms[kBlock];
  const int R = loss_rows(C);
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int nr = (int)min<int64_t>(R, n_index - r0);
  const float inv_n = 1.0f / (float)n_index;
  const int p = threadIdx.x;
  if (p < nr * C) {
    const int ri = p / C;
    const int c = p - ri * C;
    const int64_t r = index[r0 + ri];
    const float zz = z[r * ldz + c];
    const float pr = 1.f / (1.f + expf(-zz));
    const float t = labels[r * ldl + c];
    const float w = cw[2 * c];        // (float)w_c
    const float w1 = cw[2 * c + 1];   // (float)(w_c + 1)
    const float cp = fminf(fmaxf(pr, 1e-9f), 10.f);
    const float q = 1.f - pr;
    const float cq = fminf(fmaxf(q, 1e-9f), 10.f);
    const float la = logf(cp), lb = logf(cq);
    terms[p] = ((t * la) * w + (1.f - t) * lb) / w1 * 2.f;
    if (dz) {
      // d(-sum/n)/d term = -(1/n); then *2, /(w+1)
      float g = -inv_n;
      g = g * 2.f;
      g = g / w1;
      float ga = (g * w) * t;         // through (t * log(cp)) * w
      ga = ga / cp;                   // log'
      if (!(pr >= 1e-9f && pr <= 10.f)) ga = 0.f;  // clamp'
      float gb = g * (1.f - t);
      gb = gb / cq;
      if (!(q >= 1e-9f && q <= 10.f)) gb = 0.f;
      const float dp = ga + (-gb);
      dz[r * lddz + c] = (dp * (1.f - pr)) * pr;  // sigmoid_backward(grad, out)
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < C) {
    float s = 0.f;
    for (int ri = 0; ri < nr; ++ri) s += terms[ri * C + threadIdx.x];
    part[(int64_t)blockIdx.x * C + threadIdx.x] = s;
  }
}

// pass 3, one workgroup: G = 256 / C thread groups per class; group g sums blocks
// [nb g / G, nb (g+1) / G) in order, then thread c adds the G group sums in order and
// thread 0 the classes in order.
__global__ __launch_bounds__(kBlock) void multi_loss_final_kernel(const float* __restrict__ part,
                                                                  int nb, int C, int64_t n_index,
                                                                  float* __restrict__ loss) {
  __shared__ float gs[kBlock];
  __shared__ float cls[64];
  const int G = kBlock / C;
  const int c = threadIdx.x % C, g = threadIdx.x / C;
  float s = 0.f;
  if (g < G) {
    const int b0 = (int)((int64_t)nb * g / G), b1 = (int)((int64_t)nb * (g + 1) / G);
    for (int b = b0; b < b1; ++b) s += part[(int64_t)b * C + c];
  }
  gs[threadIdx.x] = s;
  __syncthreads();
  if ((int)threadIdx.x < C) {
    float t = 0.f;
    for (int q = 0; q < G; ++q) t += gs[q * C + threadIdx.x];
    cls[threadIdx.x] = -t / (float)n_index;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float total = 0.f;
    for (int k = 0; k < C; ++k) total += cls[k];
    loss[0] = total;
  }
}

// ---- Adam ---------------------------------------------------------------------------
__global__ void adam_prepare_kernel(float* state, double lr, double beta1, double beta2) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  pg_adam::step_scalars(state, lr, beta1, beta2);
}

__global__ __launch_bounds__(kBlock) void adam_apply_kernel(
    float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
    float* __restrict__ v, int64_t n, const float* __restrict__ state, float beta1, float beta2,
    float a1, float a2, float eps, float wd) {
  const float step_size = state[1];
  const float bc2s = state[2];
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock)
    pg_adam::elem(p, g, m, v, i, step_size, bc2s, beta1, beta2, a1, a2, eps, wd);
}

// bf16 storage helpers: dst[i] = bf16(src[map ? map[i] : i]) (round to nearest even;
// map[i] < 0 writes 0), and the widening copy back.
__global__ __launch_bounds__(kBlock) void cast_bf16_kernel(const float* __restrict__ src,
                                                           const int32_t* __restrict__ map, int64_t n,
                                                           uint16_t* __restrict__ dst) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    float v = 0.f;
    if (map) {
      const int32_t j = map[i];
      if (j >= 0) v = src[j];
    } else {
      v = src[i];
    }
    dst[i] = __builtin_bit_cast(uint16_t, static_cast<__bf16>(v));
  }
}

__global__ __launch_bounds__(kBlock) void widen_bf16_kernel(const uint16_t* __restrict__ src, int64_t n,
                                                            float* __restrict__ dst) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
    dst[i] = __uint_as_float((uint32_t)src[i] << 16);
}

}  // namespace

extern "C" {

int pg_bias_act(float* y, int64_t ldy, int64_t rows, int64_t cols, const float* bias, int act,
                float slope, pg_stream_t stream) {
  if (rows < 0 || cols < 0 || ldy < cols)
    return pg::set_error(PG_ERR_INVALID, "pg_bias_act: bad shape");
  if (rows * cols == 0) return pg::ok();
  hipStream_t st = (hipStream_t)stream;
  const int g = grid_1d(rows * cols);
  switch (act) {
    case PG_ACT_NONE:
      hipLaunchKernelGGL((bias_act_kernel<PG_ACT_NONE>), dim3(g), dim3(kBlock), 0, st, y, ldy, rows, (int)cols, bias, slope);
      break;
    case PG_ACT_RELU:
      hipLaunchKernelGGL((bias_act_kernel<PG_ACT_RELU>), dim3(g), dim3(kBlock), 0, st, y, ldy, rows, (int)cols, bias, slope);
      break;
    case PG_ACT_LEAKY:
      hipLaunchKernelGGL((bias_act_kernel<PG_ACT_LEAKY>), dim3(g), dim3(kBlock), 0, st, y, ldy, rows, (int)cols, bias, slope);
      break;
    default:
      return pg::set_error(PG_ERR_INVALID, "pg_bias_act: bad act %d", act);
  }
  return hip_status("pg_bias_act");
}

int pg_act_bwd(float* dy, int64_t lddy, const float* y, int64_t ldy, int64_t rows, int64_t cols,
               int act, float slope, pg_stream_t stream) {
  if (rows < 0 || cols < 0 || lddy < cols || ldy < cols)
    return pg::set_error(PG_ERR_INVALID, "pg_act_bwd: bad shape");
  if (rows * cols == 0 || act == PG_ACT_NONE) return pg::ok();
  hipStream_t st = (hipStream_t)stream;
  const int g = grid_1d(rows * cols);
  if (act == PG_ACT_RELU)
    hipLaunchKernelGGL((act_bwd_kernel<PG_ACT_RELU>), dim3(g), dim3(kBlock), 0, st, dy, lddy, y, ldy, rows, (int)cols, slope);
  else if (act == PG_ACT_LEAKY)
    hipLaunchKernelGGL((act_bwd_kernel<PG_ACT_LEAKY>), dim3(g), dim3(kBlock), 0, st, dy, lddy, y, ldy, rows, (int)cols, slope);
  else
    return pg::set_error(PG_ERR_INVALID, "pg_act_bwd: bad act %d", act);
  return hip_status("pg_act_bwd");
}

size_t pg_col_sum_workspace(int64_t rows, int64_t cols) {
  (void)rows;
  return (size_t)kColRowChunks * (size_t)std::max<int64_t>(cols, 0) * 4;
}

int pg_col_sum(const float* x, int64_t ldx, int64_t rows, int64_t cols, float* out,
               int accumulate, void* ws, size_t ws_bytes, pg_stream_t stream) {
  if (rows < 0 || cols < 0 || ldx < cols)
    return pg::set_error(PG_ERR_INVALID, "pg_col_sum: bad shape");
  if (cols == 0) return pg::ok();
  if (ws_bytes < pg_col_sum_workspace(rows, cols))
    return pg::set_error(PG_ERR_WORKSPACE, "pg_col_sum: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int R = (int)std::max<int64_t>(1, std::min<int64_t>(kColRowChunks, (rows + 63) / 64));
  hipLaunchKernelGGL(col_sum_part_kernel, dim3((cols + 63) / 64, R), dim3(kBlock), 0,
                     st, x, ldx, rows, (int)cols, (float*)ws);
  hipLaunchKernelGGL(col_sum_final_kernel, dim3((cols + kBlock - 1) / kBlock), dim3(kBlock), 0, st,
                     (const float*)ws, R, (int)cols, out, accumulate);
  return hip_status("pg_col_sum");
}

size_t pg_sigmoid_multi_loss_workspace(int64_t n_index, int32_t C) {
  const int64_t nb = std::max<int64_t>(1, (n_index + loss_rows(C) - 1) / loss_rows(C));
  return (size_t)(nb * std::max(C, 1) * 4 + 2 * 64 * 4);
}

int pg_sigmoid_multi_loss(const float* z, int64_t ldz, int64_t n_rows, int32_t C,
                          const float* labels, int64_t ldl, const float* class_w,
                          const int32_t* index, int64_t n_index, float* prob, int64_t ldp,
                          float* loss, float* dz, int64_t lddz, void* ws, size_t ws_bytes,
                          pg_stream_t stream) {
  if (C <= 0 || C > 64 || n_rows < 0 || ldz < C || ldl < C || (prob && ldp < C) ||
      (dz && lddz < C) || n_index < 0)
    return pg::set_error(PG_ERR_INVALID, "pg_sigmoid_multi_loss: bad shape");
  if (!z || !labels || !class_w || (n_index > 0 && !index))
    return pg::set_error(PG_ERR_INVALID, "pg_sigmoid_multi_loss: NULL buffer");
  if (ws_bytes < pg_sigmoid_multi_loss_workspace(n_index, C))
    return pg::set_error(PG_ERR_WORKSPACE, "pg_sigmoid_multi_loss: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if ((prob || dz) && n_rows > 0)
    hipLaunchKernelGGL(sigmoid_zero_kernel, dim3(grid_1d(n_rows * C)), dim3(kBlock), 0, st, z, ldz,
                       n_rows, (int)C, prob, ldp, dz, lddz);
  const int nb = (int)std::max<int64_t>(1, (n_index + loss_rows(C) - 1) / loss_rows(C));
  float* part = (float*)ws;
  if (n_index > 0) {
    hipLaunchKernelGGL(multi_loss_kernel, dim3(nb), dim3(kBlock), 0, st, z, ldz, (int)C, labels, ldl,
                       class_w, index, n_index, part, dz, lddz);
    if (loss)
      hipLaunchKernelGGL(multi_loss_final_kernel, dim3(1), dim3(kBlock), 0, st, (const float*)part, nb,
                         (int)C, n_index, loss);
  }
  return hip_status("pg_sigmoid_multi_loss");
}

int pg_adam_prepare(float* state, double lr, double beta1, double beta2, pg_stream_t stream) {
  if (!state) return pg::set_error(PG_ERR_INVALID, "pg_adam_prepare: NULL state");
  hipLaunchKernelGGL(adam_prepare_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, state, lr,
                     beta1, beta2);
  return hip_status("pg_adam_prepare");
}

int pg_adam_apply(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                  const float* state, double beta1, double beta2, double eps,
                  double weight_decay, pg_stream_t stream) {
  if (n < 0 || !state) return pg::set_error(PG_ERR_INVALID, "pg_adam_apply: bad arguments");
  if (n == 0) return pg::ok();
  if (!param || !grad || !exp_avg || !exp_avg_sq)
    return pg::set_error(PG_ERR_INVALID, "pg_adam_apply: NULL buffer");
  // one element per thread (up to 2^15 blocks): every thread's four loads are in flight at
  // once instead of 2-3 dependent grid-stride rounds
  hipLaunchKernelGGL(adam_apply_kernel, dim3(grid_1d(n, 32768)), dim3(kBlock), 0, (hipStream_t)stream,
                     param, grad, exp_avg, exp_avg_sq, n, state, (float)beta1, (float)beta2,
                     (float)(1.0 - beta1), (float)(1.0 - beta2), (float)eps, (float)weight_decay);
  return hip_status("pg_adam_apply");
}

}  // extern "C"

namespace {
// One launch for several zero-padded 2-D copies: part p owns the workgroups
// [first[p], first[p+1]); each thread writes one element of dst (drows x dcols), the
// source element or 0 past rows x cols.
struct Pad2dGroup {
  pg_pad2d_t p[PG_PAD2D_MAX];
  int64_t first[PG_PAD2D_MAX + 1];
  int n;
};

__global__ __launch_bounds__(kBlock) void pad2d_group_kernel(Pad2dGroup g) {
  int k = 0;
  while (k + 1 < g.n && (int64_t)blockIdx.x >= g.first[k + 1]) ++k;
  const pg_pad2d_t& p = g.p[k];
  const int64_t i = ((int64_t)blockIdx.x - g.first[k]) * kBlock + threadIdx.x;
  if (i >= p.drows * p.dcols) return;
  const int64_t r = i / p.dcols, c = i % p.dcols;
  p.dst[r * p.ldd + c] = (r < p.rows && c < p.cols) ? p.src[r * p.lds + c] : 0.f;
}
}  // namespace

extern "C" {

int pg_pad2d_group(const pg_pad2d_t* parts, int n, pg_stream_t stream) {
  if (n < 0 || n > PG_PAD2D_MAX || (n > 0 && !parts))
    return pg::set_error(PG_ERR_INVALID, "pg_pad2d_group: n = %d (at most %d parts)", n, PG_PAD2D_MAX);
  Pad2dGroup g{};
  g.n = n;
  int64_t blocks = 0;
  for (int k = 0; k < n; ++k) {
    const pg_pad2d_t& p = parts[k];
    if (p.rows < 0 || p.cols < 0 || p.drows < 0 || p.dcols < 0 || p.rows > p.drows || p.cols > p.dcols ||
        p.ldd < p.dcols ||
        (p.rows > 0 && p.cols > 0 && (!p.src || p.lds < p.cols)) || (p.drows * p.dcols > 0 && !p.dst))
      return pg::set_error(PG_ERR_INVALID, "pg_pad2d_group: bad part %d", k);
    g.p[k] = p;
    g.first[k] = blocks;
    blocks += (p.drows * p.dcols + kBlock - 1) / kBlock;
  }
  g.first[n] = blocks;
  if (blocks == 0) return pg::ok();
  if (blocks > INT32_MAX) return pg::set_error(PG_ERR_UNSUPPORTED, "pg_pad2d_group: too large");
  hipLaunchKernelGGL(pad2d_group_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream, g);
  return hip_status("pg_pad2d_group");
}

int pg_cast_f32_bf16(const float* src, const int32_t* map, int64_t n, void* dst,
                     pg_stream_t stream) {
  if (n < 0) return pg::set_error(PG_ERR_INVALID, "pg_cast_f32_bf16: n < 0");
  if (n == 0) return pg::ok();
  if (!src || !dst) return pg::set_error(PG_ERR_INVALID, "pg_cast_f32_bf16: NULL buffer");
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid_1d(n, 4096)), dim3(kBlock), 0, (hipStream_t)stream, src,
                     map, n, (uint16_t*)dst);
  return hip_status("pg_cast_f32_bf16");
}

int pg_cast_bf16_f32(const void* src, int64_t n, float* dst, pg_stream_t stream) {
  if (n < 0) return pg::set_error(PG_ERR_INVALID, "pg_cast_bf16_f32: n < 0");
  if (n == 0) return pg::ok();
  if (!src || !dst) return pg::set_error(PG_ERR_INVALID, "pg_cast_bf16_f32: NULL buffer");
  hipLaunchKernelGGL(widen_bf16_kernel, dim3(grid_1d(n, 4096)), dim3(kBlock), 0, (hipStream_t)stream,
                     (const uint16_t*)src, n, dst);
  return hip_status("pg_cast_bf16_f32");
}

}  // extern "C"
