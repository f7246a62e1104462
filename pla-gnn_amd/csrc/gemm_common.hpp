// Pieces shared by the fp32 (gemm.hip) and bf16 (gemm_bf16.hip) GEMMs: the fused
// epilogue modes and the deterministic split-K combine.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace pg_gemm {

// Epilogue modes: activation of the result, or multiplication by the derivative of an
// activation given its OUTPUT y (the fused backward of relu / leaky_relu), or split-K.
enum Epi { EPI_NONE = 0, EPI_RELU = 1, EPI_LEAKY = 2, EPI_DRELU = 3, EPI_DLEAKY = 4, EPI_SPLIT = 5 };

__host__ __device__ inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

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

__device__ __forceinline__ float4 splitk_sum4(const float* __restrict__ p, int64_t stride, int z0, int z1) {
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int z = z0; z < z1; z += 8) {
    float4 v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e)
      v[e] = z + e < z1 ? *reinterpret_cast<const float4*>(p + (int64_t)(z + e) * stride) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (z + e < z1) {
        s.x += v[e].x; s.y += v[e].y; s.z += v[e].z; s.w += v[e].w;
      }
  }
  return s;
}

// vec4 (N % 4 == 0, 16-B aligned slabs): a work unit is 4 consecutive outputs of one row
// (float4 slab loads, each component summed in the same slice order: bitwise the same as
// the scalar form), the row sums stay scalar units after them.
template <int G>
__device__ __forceinline__ void splitk_reduce_body(const float* __restrict__ ws, int splits, int M, int N,
                                                   float alpha, float beta, float* __restrict__ C,
                                                   int64_t ldc, const float* __restrict__ ws_rowsum,
                                                   float* __restrict__ rowsum, int blk, int nblk) {
  constexpr int OPB = 256 / G;  // units per block
  __shared__ float4 part[256];
  const int64_t n = (int64_t)M * N;
  const bool vec = (N % 4) == 0 && al16(ws);
  const int64_t nu = vec ? n / 4 : n;  // units of the product
  const int64_t total = nu + (rowsum ? M : 0);
  const int ol = threadIdx.x % OPB, g = threadIdx.x / OPB;
  const int z0 = (int)((int64_t)splits * g / G), z1 = (int)((int64_t)splits * (g + 1) / G);
  for (int64_t base = (int64_t)blk * OPB; base < total; base += (int64_t)nblk * OPB) {
    const int64_t u = base + ol;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (u < total) {
      if (u >= nu) s.x = splitk_sum<G>(ws_rowsum + (u - nu), M, z0, z1);
      else if (vec) s = splitk_sum4(ws + 4 * u, n, z0, z1);
      else s.x = splitk_sum<G>(ws + u, n, z0, z1);
    }
    if constexpr (G > 1) {
      part[threadIdx.x] = s;
      __syncthreads();
      if (g == 0) {
#pragma unroll
        for (int q = 1; q < G; ++q) {
          const float4 t = part[q * OPB + ol];
          s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
        }
      }
      __syncthreads();
    }
    if (g == 0 && u < total) {
      if (u >= nu) {
        rowsum[u - nu] = s.x;
      } else {
        const int64_t i = vec ? 4 * u : u;
        const int64_t r = i / N;
        const int c = (int)(i - r * N);
        float* cp = C + r * ldc + c;
        const float sv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (e > 0 && !vec) break;
          float v = alpha * sv[e];
          if (beta != 0.f) v = v + beta * cp[e];
          cp[e] = v;
        }
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

// The three-piece bf16 GEMM (gemm_x3.hip): arguments and launcher (C = alpha op(A) op(B) +
// beta C with the fused epilogue, or split-K partial slabs when epi == EPI_SPLIT).
struct X3Args {
  bool ta, tb;
  int bm, bn, epi;
  int M, N, K, kps, tiles_n, tiles, n_split;
  float alpha;
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  float beta;
  float* C;
  int64_t ldc;
  const float* bias;
  float slope;
  const float* dact;
  int64_t lddact;
  float* rowsum;
  float* ws;
  float* ws_rowsum;
};
int gemm_x3_launch(const X3Args& a, hipStream_t st);
// The same with both operands concatenated along K: op(A) = [A | A2], op(B) = [B ; B2]
// (k < kcat from the first; kcat a multiple of 4; no split-K; ta = false; EPI_NONE or
// EPI_LEAKY).
int gemm_x3_cat_launch(const X3Args& a, const float* A2, int64_t lda2, const float* B2, int64_t ldb2, int kcat,
                       hipStream_t st);

// Grouped split-K partials (pg_gemm_f32_group): one tile shape and one (ta, tb) for the
// group. 128 x 256 (two workgroups per CU, each wave 64 x 128: a third less staging per
// MFMA than 128 x 128): cfg2 GEMM 0.796 -> 0.790 ms per step, cfg3 1.867 -> 1.857
// (scripts/ab_lib.sh, round 5); 128 x 64 was slower in round 4.
#ifndef PG_X3_GROUP_TILE
#define PG_X3_GROUP_TILE 128256  // variant builds: BM * 1000 + BN
#endif
constexpr int kX3GroupBM = PG_X3_GROUP_TILE / 1000, kX3GroupBN = PG_X3_GROUP_TILE % 1000;
struct X3Part {
  int M, N, K, kps, tiles_n, tiles, first_item;
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  float* ws;         // [n_split][M][N] slabs
  float* ws_rowsum;  // [n_split][M] row-sum slices
  float* rowsum;     // non-null: row sums wanted (the slices are written; the combine writes here)
};
constexpr int kX3MaxParts = 16;
struct X3Group {
  X3Part p[kX3MaxParts];
  int n, items;
};
int gemm_x3_group_launch(const X3Group& g, bool ta, bool tb, hipStream_t st);

// Threads per output of the split-K combine: enough slice groups that each thread sums
// <= ~8 slices.
inline int splitk_groups(int split_k) { return split_k <= 8 ? 1 : split_k <= 32 ? 4 : 16; }

}  // namespace pg_gemm
