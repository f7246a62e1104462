// The model head after liner1, fused into one pass over the nodes (f32 or bf16 storage):
//   z    = A4 W2^T + b2                         liner2              (code/model.py:28)
//   prob = sigmoid(z)                                               (code/model.py:29)
//   per-row terms of multi_loss for the train rows and the val rows (code/train.py:89-108,
//        199-200 and 206-207: the val loss on the same pre-step logits)
//   dz   = d train_loss / dz (train rows; 0 elsewhere)              (train.py:204)
//   dA4  = (dz W2) * leaky'(A4)   liner2's input gradient with liner1's activation backward
// Before, these were a liner2 GEMM (N = 12 columns), two loss launches per set and a
// dgrad GEMM of N x 12 x 100: five launches that each streamed A4 / z / dz through HBM
// for a few hundred MFLOP. Here one workgroup owns 32 rows: W2 and the rows of A4 sit in
// LDS, z / dz live in LDS, and A4 is read once.
// Loss terms follow the autograd graph of train.py:103-104 operation by operation (as
// pg_sigmoid_multi_loss); each workgroup sums its rows per class in row order, and one
// final workgroup sums the blocks in a fixed order: deterministic.
#include <hip/hip_runtime.h>

#include <cmath>

#include "common.hpp"

namespace {

constexpr int kBlock = 256;
constexpr int kRows = 32;    // rows per workgroup
constexpr int kMaxK = 128;   // liner1 width (padded)
constexpr int kMaxC = 16;    // classes (padded)

__device__ __forceinline__ float ld_elem(const float* p, int64_t i) { return p[i]; }
__device__ __forceinline__ float ld_elem(const uint16_t* p, int64_t i) {
  return __uint_as_float((uint32_t)p[i] << 16);
}
__device__ __forceinline__ void st_elem(float* p, int64_t i, float v) { p[i] = v; }
__device__ __forceinline__ void st_elem(uint16_t* p, int64_t i, float v) {
  p[i] = __builtin_bit_cast(uint16_t, static_cast<__bf16>(v));
}

// 4 consecutive elements k .. k+3 of a row (zero past K), widened to f32
__device__ __forceinline__ float4 ld4(const float* p, int64_t row, int k, int K) {
  if (k + 3 < K && ((row + k) & 3) == 0) return *reinterpret_cast<const float4*>(p + row + k);
  float4 r;
  r.x = k < K ? p[row + k] : 0.f;
  r.y = k + 1 < K ? p[row + k + 1] : 0.f;
  r.z = k + 2 < K ? p[row + k + 2] : 0.f;
  r.w = k + 3 < K ? p[row + k + 3] : 0.f;
  return r;
}
__device__ __forceinline__ float4 ld4(const uint16_t* p, int64_t row, int k, int K) {
  float4 r;
  if (k + 3 < K && ((row + k) & 3) == 0) {
    const uint2 t = *reinterpret_cast<const uint2*>(p + row + k);
    r.x = __uint_as_float(t.x << 16); r.y = __uint_as_float(t.x & 0xFFFF0000u);
    r.z = __uint_as_float(t.y << 16); r.w = __uint_as_float(t.y & 0xFFFF0000u);
    return r;
  }
  r.x = k < K ? ld_elem(p, row + k) : 0.f;
  r.y = k + 1 < K ? ld_elem(p, row + k + 1) : 0.f;
  r.z = k + 2 < K ? ld_elem(p, row + k + 2) : 0.f;
  r.w = k + 3 < K ? ld_elem(p, row + k + 3) : 0.f;
  return r;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void head_kernel(
    const T* __restrict__ a4, int64_t lda, int n, int K, const float* __restrict__ w2,
    int64_t ldw, const float* __restrict__ b2, int C, const float* __restrict__ labels,
    int64_t ldl, const float* __restrict__ cw, const int8_t* __restrict__ row_set,
    float inv_n_train, float* __restrict__ prob, int64_t ldp, float* __restrict__ dz,
    int64_t lddz, uint16_t* __restrict__ dz_bf16, T* __restrict__ da4, int64_t ldg, float slope,
    float* __restrict__ part, int nb) {
  // [row][k] images with a 16-B aligned row stride (K4 = K rounded up to 4, + 4)
  __shared__ __attribute__((aligned(16))) float w[kMaxC * (kMaxK + 4)];
  __shared__ __attribute__((aligned(16))) float a[kRows * (kMaxK + 4)];
  __shared__ float g[kRows][kMaxC];
  __shared__ float terms[2][kRows][kMaxC];
  const int K4 = (K + 3) / 4 * 4, S = K4 + 4;
  const int r0 = blockIdx.x * kRows;
  const int nr = min(kRows, n - r0);
  // A4 rows and W2 into LDS in 4-element units: every unit's load is issued before any LDS
  // store (a load-store loop would wait out one memory latency per iteration)
  {
    constexpr int kUnits = (kRows + kMaxC) * (kMaxK / 4);
    constexpr int kPer = (kUnits + kBlock - 1) / kBlock;
    const int ua = kRows * (K4 / 4), uw = C * (K4 / 4);
    float4 v[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int u = threadIdx.x + q * kBlock;
      v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (u < ua) {
        const int ri = u / (K4 / 4), k = (u - ri * (K4 / 4)) * 4;
        if (ri < nr) v[q] = ld4(a4, (int64_t)(r0 + ri) * lda, k, K);
      } else if (u < ua + uw) {
        const int c = (u - ua) / (K4 / 4), k = (u - ua - c * (K4 / 4)) * 4;
        v[q] = ld4(w2, (int64_t)c * ldw, k, K);
      }
    }
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int u = threadIdx.x + q * kBlock;
      if (u < ua) {
        const int ri = u / (K4 / 4), k = (u - ri * (K4 / 4)) * 4;
        *reinterpret_cast<float4*>(a + ri * S + k) = v[q];
      } else if (u < ua + uw) {
        const int c = (u - ua) / (K4 / 4), k = (u - ua - c * (K4 / 4)) * 4;
        *reinterpret_cast<float4*>(w + c * S + k) = v[q];
      }
    }
  }
  for (int i = threadIdx.x; i < 2 * kRows * kMaxC; i += kBlock) (&terms[0][0][0])[i] = 0.f;
  __syncthreads();
  // z, prob, loss terms, dz: thread t takes class c = t % 16 of rows t / 16 and t / 16 + 16
  {
    const int c = threadIdx.x % kMaxC, rg = threadIdx.x / kMaxC;
#pragma unroll
    for (int h = 0; h < kRows / (kBlock / kMaxC); ++h) {
      const int ri = rg + h * (kBlock / kMaxC);
      if (c < C && ri < nr) {
        const int64_t r = r0 + ri;
        const int set = row_set[r];
        const float t = labels[r * ldl + c];
        const float4* ar = reinterpret_cast<const float4*>(a + ri * S);
        const float4* wr = reinterpret_cast<const float4*>(w + c * S);
        float zz = 0.f;
        for (int k4 = 0; k4 < K4 / 4; ++k4) {
          const float4 x = ar[k4], y = wr[k4];
          zz = fmaf(x.x, y.x, zz);
          zz = fmaf(x.y, y.y, zz);
          zz = fmaf(x.z, y.z, zz);
          zz = fmaf(x.w, y.w, zz);
        }
        zz = zz + b2[c];
        const float pr = 1.f / (1.f + expf(-zz));
        if (prob) prob[r * ldp + c] = pr;
        float gz = 0.f;
        if (set != 0) {
          const float wc = cw[2 * c];        // (float)w_c
          const float w1 = cw[2 * c + 1];    // (float)(w_c + 1)
          const float cp = fminf(fmaxf(pr, 1e-9f), 10.f);
          const float q = 1.f - pr;
          const float cq = fminf(fmaxf(q, 1e-9f), 10.f);
          const float la = logf(cp), lb = logf(cq);
          terms[set - 1][ri][c] = ((t * la) * wc + (1.f - t) * lb) / w1 * 2.f;
          if (set == 1) {
            float gg = -inv_n_train;
            gg = gg * 2.f;
            gg = gg / w1;
            float ga = (gg * wc) * t;
            ga = ga / cp;
            if (!(pr >= 1e-9f && pr <= 10.f)) ga = 0.f;
            float gb = gg * (1.f - t);
            gb = gb / cq;
            if (!(q >= 1e-9f && q <= 10.f)) gb = 0.f;
            const float dp = ga + (-gb);
            gz = (dp * (1.f - pr)) * pr;
          }
        }
        g[ri][c] = gz;
        if (dz) dz[r * lddz + c] = gz;
        if (dz_bf16) dz_bf16[r * lddz + c] = __builtin_bit_cast(uint16_t, static_cast<__bf16>(gz));
      } else if (c >= C) {
        g[ri][c] = 0.f;
      }
    }
  }
  __syncthreads();
  // per-block class sums in row order, stored [set][c][block] (the final reduction reads
  // each pair's blocks contiguously)
  if ((int)threadIdx.x < 2 * C) {
    const int set = threadIdx.x / C, c = threadIdx.x % C;
    float s = 0.f;
    for (int ri = 0; ri < nr; ++ri) s += terms[set][ri][c];
    part[((int64_t)set * C + c) * nb + blockIdx.x] = s;
  }
  // dA4 = (dz W2) * leaky'(A4): thread t owns column j = t % 128 (its W2 column in
  // registers) and rows t / 128, t / 128 + 2, ...
  if (da4) {
    const int j = threadIdx.x % kMaxK, r2 = threadIdx.x / kMaxK;
    if (j < K) {
      float wj[kMaxC];
#pragma unroll
      for (int c = 0; c < kMaxC; ++c) wj[c] = c < C ? w[c * S + j] : 0.f;
      for (int ri = r2; ri < nr; ri += kBlock / kMaxK) {
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < kMaxC; ++c) s = fmaf(g[ri][c], wj[c], s);
        const float y = a[ri * S + j];
        st_elem(da4, (int64_t)(r0 + ri) * ldg + j, y > 0.f ? s : s * slope);
      }
    }
  }
}

// loss[s] = sum_c -(sum over blocks of part[s][c][b]) / n_s: one workgroup per set, one
// wave per class. Lane l sums blocks l, l + 64, ... in order (coalesced), the wave folds its
// lanes in a fixed butterfly, and thread 0 adds the classes in order: deterministic.
__global__ __launch_bounds__(64 * kMaxC) void head_final_kernel(const float* __restrict__ part, int nb,
                                                                int C, int64_t n_train, int64_t n_val,
                                                                float* __restrict__ loss) {
  __shared__ float cls[kMaxC];
  const int set = blockIdx.x, c = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t ns = set == 0 ? n_train : n_val;
  float s = 0.f;
  if (c < C) {
    // 8 blocks' loads in flight per lane, summed in the same order as one at a time
    const float* pp = part + ((int64_t)set * C + c) * nb;
    for (int b0 = lane; b0 < nb; b0 += 8 * 64) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = pp[min(b0 + e * 64, nb - 1)];
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (b0 + e * 64 < nb) s += v[e];
    }
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0 && c < C) cls[c] = ns > 0 ? -s / (float)ns : 0.f;
  __syncthreads();
  if (threadIdx.x == 0 && ns > 0) {
    float total = 0.f;
    for (int k = 0; k < C; ++k) total += cls[k];
    loss[set] = total;
  }
}

}  // namespace

extern "C" {

size_t pg_mlp_head_workspace(int64_t n, int32_t C) {
  const int64_t nb = std::max<int64_t>(1, (n + kRows - 1) / kRows);
  return (size_t)(nb * 2 * std::max(C, 1) * 4);
}

int pg_mlp_head(const void* a4, int64_t lda, int64_t n, int32_t K, int a_dtype, const float* w2,
                int64_t ldw, const float* b2, int32_t C, const float* labels, int64_t ldl,
                const float* class_w, const int8_t* row_set, int64_t n_train, int64_t n_val,
                float* prob, int64_t ldp, float* dz, int64_t lddz, void* dz_bf16, void* da4,
                int64_t ldg, float slope, float* loss2, void* ws, size_t ws_bytes,
                pg_stream_t stream) {
  if (n < 0 || n > INT32_MAX || K <= 0 || K > kMaxK || C <= 0 || C > kMaxC || lda < K || ldw < K ||
      ldl < C || (prob && ldp < C) || ((dz || dz_bf16) && lddz < C) || (da4 && ldg < K))
    return pg::set_error(PG_ERR_INVALID, "pg_mlp_head: bad shape (K <= %d, C <= %d)", kMaxK, kMaxC);
  if (a_dtype != PG_DTYPE_F32 && a_dtype != PG_DTYPE_BF16)
    return pg::set_error(PG_ERR_INVALID, "pg_mlp_head: bad a_dtype");
  if (n == 0) return pg::ok();
  if (!a4 || !w2 || !b2 || !labels || !class_w || !row_set || !loss2)
    return pg::set_error(PG_ERR_INVALID, "pg_mlp_head: NULL buffer");
  if (ws_bytes < pg_mlp_head_workspace(n, C))
    return pg::set_error(PG_ERR_WORKSPACE, "pg_mlp_head: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int nb = (int)((n + kRows - 1) / kRows);
  float* part = (float*)ws;
  const float inv_n = n_train > 0 ? 1.0f / (float)n_train : 0.f;
  if (a_dtype == PG_DTYPE_F32)
    hipLaunchKernelGGL(head_kernel<float>, dim3(nb), dim3(kBlock), 0, st, (const float*)a4, lda, (int)n,
                       (int)K, w2, ldw, b2, (int)C, labels, ldl, class_w, row_set, inv_n, prob, ldp, dz,
                       lddz, (uint16_t*)dz_bf16, (float*)da4, ldg, slope, part, nb);
  else
    hipLaunchKernelGGL(head_kernel<uint16_t>, dim3(nb), dim3(kBlock), 0, st, (const uint16_t*)a4, lda,
                       (int)n, (int)K, w2, ldw, b2, (int)C, labels, ldl, class_w, row_set, inv_n, prob,
                       ldp, dz, lddz, (uint16_t*)dz_bf16, (uint16_t*)da4, ldg, slope, part, nb);
  hipLaunchKernelGGL(head_final_kernel, dim3(2), dim3(64 * kMaxC), 0, st, (const float*)part, nb, (int)C,
                     n_train, n_val, loss2);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pg::set_error((int)e, "pg_mlp_head: launch failed: %s", hipGetErrorString(e));
  return pg::ok();
}

}  // extern "C"
