// Pieces shared by the fp32 (gemm.hip) and bf16 (gemm_bf16.hip) GEMMs: the fused
// epilogue modes and the deterministic split-K combine.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace pg_gemm {

// Epilogue modes: activation of the result, or multiplication by the derivative of an
// activation given its OUTPUT y (the fused backward of relu / leaky_relu), or split-K.
enum Epi { EPI_NONE = 0, EPI_RELU = 1, EPI_LEAKY = 2, EPI_DRELU = 3, EPI_DLEAKY = 4, EPI_SPLIT = 5 };

template <int EPI>
__device__ __forceinline__ float epi_apply(float x, float y, float slope) {
  if constexpr (EPI == EPI_RELU) return x > 0.f ? x : 0.f;
  else if constexpr (EPI == EPI_LEAKY) return x > 0.f ? x : x * slope;
  else if constexpr (EPI == EPI_DRELU) return y > 0.f ? x : 0.f;
  else if constexpr (EPI == EPI_DLEAKY) return y > 0.f ? x : x * slope;
  else return x;
}

// Split-K combine: C = alpha * sum_z ws[z] (+ beta * C); the row sums likewise (their
// slices follow the partial slabs in the workspace). G threads per output: thread group g
// sums slices [S g / G, S (g+1) / G) in order, then one thread adds the G group sums in
// order (a fixed order: deterministic). Consecutive threads take consecutive outputs, so
// every slab read is coalesced; a thread's slice loads are issued 8 at a time (summed in
// slice order afterwards), so they are not one dependent round trip each.
template <int G>
__device__ __forceinline__ float splitk_sum(const float* __restrict__ p, int64_t stride, int z0, int z1) {
  float s = 0.f;
  for (int z = z0; z < z1; z += 8) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = z + e < z1 ? p[(int64_t)(z + e) * stride] : 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (z + e < z1) s += v[e];
  }
  return s;
}

template <int G>
__device__ __forceinline__ void splitk_reduce_body(const float* __restrict__ ws, int splits, int M, int N,
                                                   float alpha, float beta, float* __restrict__ C,
                                                   int64_t ldc, const float* __restrict__ ws_rowsum,
                                                   float* __restrict__ rowsum, int blk, int nblk) {
  constexpr int OPB = 256 / G;  // outputs per block
  __shared__ float part[256];
  const int64_t n = (int64_t)M * N;
  const int64_t total = n + (rowsum ? M : 0);
  const int ol = threadIdx.x % OPB, g = threadIdx.x / OPB;
  const int z0 = (int)((int64_t)splits * g / G), z1 = (int)((int64_t)splits * (g + 1) / G);
  for (int64_t base = (int64_t)blk * OPB; base < total; base += (int64_t)nblk * OPB) {
    const int64_t i = base + ol;
    float s = 0.f;
    if (i < total) s = i < n ? splitk_sum<G>(ws + i, n, z0, z1) : splitk_sum<G>(ws_rowsum + (i - n), M, z0, z1);
    if constexpr (G > 1) {
      part[threadIdx.x] = s;
      __syncthreads();
      if (g == 0) {
#pragma unroll
        for (int q = 1; q < G; ++q) s += part[q * OPB + ol];
      }
      __syncthreads();
    }
    if (g == 0 && i < total) {
      if (i >= n) {
        rowsum[i - n] = s;
      } else {
        const int64_t r = i / N;
        const int c = (int)(i - r * N);
        float v = alpha * s;
        if (beta != 0.f) v = v + beta * C[r * ldc + c];
        C[r * ldc + c] = v;
      }
    }
  }
}

template <int G>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws,
                                                            int splits, int M, int N, float alpha,
                                                            float beta, float* __restrict__ C,
                                                            int64_t ldc, const float* __restrict__ ws_rowsum,
                                                            float* __restrict__ rowsum) {
  splitk_reduce_body<G>(ws, splits, M, N, alpha, beta, C, ldc, ws_rowsum, rowsum, blockIdx.x, gridDim.x);
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Threads per output of the split-K combine: enough slice groups that each thread sums
// <= ~8 slices.
inline int splitk_groups(int split_k) { return split_k <= 8 ? 1 : split_k <= 32 ? 4 : 16; }

}  // namespace pg_gemm
