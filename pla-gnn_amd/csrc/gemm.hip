// fp32 GEMM on the gfx950 matrix cores (v_mfma_f32_32x32x2_f32: exact f32 products,
// f32 accumulate; gfx950 has no xf32 shortcut) with a fused epilogue
// (alpha/beta, + bias row vector, relu / leaky_relu). Serves every nn.Linear of the
// PLA-GNN step: SAGEConv's fc_pool / fc_self / fc_neigh (code/model.py:13-15) and
// liner1 / liner2 (code/model.py:16-17), forward and backward.
//
// Tile: 128 x 64 per 256-thread workgroup, K step 16; each wave owns a 32 x 64 strip
// (two 32x32 accumulators, 32 AGPR/VGPR). Global -> register prefetch of the next K
// tile overlaps the MFMAs of the current one; LDS holds A as [k][m] and B as [k][n]
// so every MFMA operand is one conflict-free ds_read_b32 per lane.
// MFMA 32x32x2 f32 operand map (cdna_hip_programming.md §3): lane l holds
// A[i = l & 31][k = l >> 5] and B[k = l >> 5][j = l & 31]; the accumulator holds
// C[row = (r & 3) + 8 (r >> 2) + 4 (l >> 5)][col = l & 31] in register r.
// Long-K products (weight gradients, K = number of nodes) use split-K with partial
// slabs summed in a fixed order (deterministic).
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace {

constexpr int BM = 128, BN = 64, BK = 16;
constexpr int kThreads = 256;
constexpr int LDA_S = BM + 4;  // [k][m] rows padded: 2-way worst case on the transposing store
constexpr int LDB_S = BN + 4;

using f32x16 = __attribute__((ext_vector_type(16))) float;

template <bool VEC>
__device__ __forceinline__ void ld4(const float* __restrict__ p, bool ok0, bool ok1, bool ok2,
                                    bool ok3, float (&r)[4]) {
  if constexpr (VEC) {
    if (ok0) {
      const float4 t = *reinterpret_cast<const float4*>(p);
      r[0] = t.x; r[1] = t.y; r[2] = t.z; r[3] = t.w;
    } else {
      r[0] = r[1] = r[2] = r[3] = 0.f;
    }
  } else {
    r[0] = ok0 ? p[0] : 0.f;
    r[1] = ok1 ? p[1] : 0.f;
    r[2] = ok2 ? p[2] : 0.f;
    r[3] = ok3 ? p[3] : 0.f;
  }
}

template <int ACT>
__device__ __forceinline__ float epi_act(float x, float slope) {
  if constexpr (ACT == PG_ACT_RELU) return x > 0.f ? x : 0.f;
  else if constexpr (ACT == PG_ACT_LEAKY) return x > 0.f ? x : x * slope;
  else return x;
}

// TA: A stored K x M (use A^T). TB: B stored N x K (use B^T).
// VA/VB: 16-byte vector loads legal for A/B (alignment + leading dim multiple of 4).
template <bool TA, bool TB, bool VA, bool VB, int ACT, bool SPLIT>
__global__ __launch_bounds__(kThreads) void gemm_f32_kernel(
    int M, int N, int K, int k_per_split, float alpha, const float* __restrict__ A, int64_t lda,
    const float* __restrict__ B, int64_t ldb, float beta, float* __restrict__ C, int64_t ldc,
    const float* __restrict__ bias, float slope, float* __restrict__ ws) {
  __shared__ float As[BK][LDA_S];
  __shared__ float Bs[BK][LDB_S];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int m0 = blockIdx.y * BM;
  const int n0 = blockIdx.x * BN;
  const int kz0 = blockIdx.z * k_per_split;
  const int kz1 = min(K, kz0 + k_per_split);

  f32x16 acc0 = {0}, acc1 = {0};

  // per-thread global load coordinates ------------------------------------------------
  // A tile: 128 (m) x 16 (k) = 512 float4 -> 2 per thread
  // B tile: 64 (n) x 16 (k) = 256 float4 -> 1 per thread
  float ra[2][4], rb[4];

  auto load_a = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + i * kThreads;
      if constexpr (!TA) {  // A[m][k], float4 along k
        const int m = m0 + (q >> 2), k = k0 + ((q & 3) << 2);
        const bool okm = m < M;
        const float* p = A + (int64_t)m * lda + k;
        ld4<VA>(p, okm && k < kz1, okm && k + 1 < kz1, okm && k + 2 < kz1, okm && k + 3 < kz1, ra[i]);
      } else {  // A[k][m], float4 along m
        const int k = k0 + (q >> 5), m = m0 + ((q & 31) << 2);
        const bool okk = k < kz1;
        const float* p = A + (int64_t)k * lda + m;
        ld4<VA>(p, okk && m < M, okk && m + 1 < M, okk && m + 2 < M, okk && m + 3 < M, ra[i]);
      }
    }
  };
  auto load_b = [&](int k0) {
    if constexpr (TB) {  // B[n][k], float4 along k
      const int n = n0 + (tid >> 2), k = k0 + ((tid & 3) << 2);
      const bool okn = n < N;
      const float* p = B + (int64_t)n * ldb + k;
      ld4<VB>(p, okn && k < kz1, okn && k + 1 < kz1, okn && k + 2 < kz1, okn && k + 3 < kz1, rb);
    } else {  // B[k][n], float4 along n
      const int k = k0 + (tid >> 4), n = n0 + ((tid & 15) << 2);
      const bool okk = k < kz1;
      const float* p = B + (int64_t)k * ldb + n;
      ld4<VB>(p, okk && n < N, okk && n + 1 < N, okk && n + 2 < N, okk && n + 3 < N, rb);
    }
  };
  auto store_ab = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + i * kThreads;
      if constexpr (!TA) {
        const int m = q >> 2, k = (q & 3) << 2;
#pragma unroll
        for (int j = 0; j < 4; ++j) As[k + j][m] = ra[i][j];
      } else {
        const int k = q >> 5, m = (q & 31) << 2;
        *reinterpret_cast<float4*>(&As[k][m]) = make_float4(ra[i][0], ra[i][1], ra[i][2], ra[i][3]);
      }
    }
    if constexpr (TB) {
      const int n = tid >> 2, k = (tid & 3) << 2;
#pragma unroll
      for (int j = 0; j < 4; ++j) Bs[k + j][n] = rb[j];
    } else {
      const int k = tid >> 4, n = (tid & 15) << 2;
      *reinterpret_cast<float4*>(&Bs[k][n]) = make_float4(rb[0], rb[1], rb[2], rb[3]);
    }
  };

  const int am = wave * 32 + (lane & 31);
  const int kh = lane >> 5;
  const int bn = lane & 31;

  if (kz0 < kz1) {
    load_a(kz0);
    load_b(kz0);
    store_ab();
    __syncthreads();
    for (int k0 = kz0; k0 < kz1; k0 += BK) {
      const bool more = k0 + BK < kz1;
      if (more) {
        load_a(k0 + BK);
        load_b(k0 + BK);
      }
#pragma unroll
      for (int kk = 0; kk < BK; kk += 2) {
        const float a = As[kk + kh][am];
        const float b0 = Bs[kk + kh][bn];
        const float b1 = Bs[kk + kh][32 + bn];
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b1, acc1, 0, 0, 0);
      }
      __syncthreads();
      if (more) {
        store_ab();
        __syncthreads();
      }
    }
  }

  // epilogue ----------------------------------------------------------------------------
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const f32x16& acc = t == 0 ? acc0 : acc1;
    const int col = n0 + t * 32 + (lane & 31);
    if (col >= N) continue;
    const float bv = (!SPLIT && bias) ? bias[col] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row >= M) continue;
      if constexpr (SPLIT) {
        ws[((int64_t)blockIdx.z * M + row) * N + col] = acc[r];
      } else {
        float v = alpha * acc[r];
        if (beta != 0.f) v = v + beta * C[(int64_t)row * ldc + col];
        if (bias) v = v + bv;
        C[(int64_t)row * ldc + col] = epi_act<ACT>(v, slope);
      }
    }
  }
}

// Split-K combine: C = alpha * sum_z ws[z] (+ beta * C), slices summed in order.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws,
                                                            int splits, int M, int N, float alpha,
                                                            float beta, float* __restrict__ C,
                                                            int64_t ldc) {
  const int64_t n = (int64_t)M * N;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float s = 0.f;
    for (int z = 0; z < splits; ++z) s += ws[(int64_t)z * n + i];
    const int64_t r = i / N;
    const int c = (int)(i - r * N);
    float v = alpha * s;
    if (beta != 0.f) v = v + beta * C[r * ldc + c];
    C[r * ldc + c] = v;
  }
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <bool TA, bool TB, bool SPLIT>
int launch_typed(bool va, bool vb, int act, dim3 grid, hipStream_t st, int M, int N, int K,
                 int kps, float alpha, const float* A, int64_t lda, const float* B, int64_t ldb,
                 float beta, float* C, int64_t ldc, const float* bias, float slope, float* ws) {
#define PG_GEMM_LAUNCH(VA_, VB_, ACT_)                                                        \
  hipLaunchKernelGGL((gemm_f32_kernel<TA, TB, VA_, VB_, ACT_, SPLIT>), grid, dim3(kThreads), 0, \
                     st, M, N, K, kps, alpha, A, lda, B, ldb, beta, C, ldc, bias, slope, ws)
#define PG_GEMM_ACT(VA_, VB_)                                              \
  switch (act) {                                                          \
    case PG_ACT_NONE: PG_GEMM_LAUNCH(VA_, VB_, PG_ACT_NONE); break;         \
    case PG_ACT_RELU: PG_GEMM_LAUNCH(VA_, VB_, PG_ACT_RELU); break;         \
    case PG_ACT_LEAKY: PG_GEMM_LAUNCH(VA_, VB_, PG_ACT_LEAKY); break;       \
    default: return PG_ERR_INVALID;                                       \
  }
  if (va && vb) { PG_GEMM_ACT(true, true) }
  else if (va) { PG_GEMM_ACT(true, false) }
  else if (vb) { PG_GEMM_ACT(false, true) }
  else { PG_GEMM_ACT(false, false) }
#undef PG_GEMM_ACT
#undef PG_GEMM_LAUNCH
  return PG_OK;
}

}  // namespace

extern "C" {

size_t pg_gemm_f32_workspace(int64_t M, int64_t N, int64_t K, int split_k) {
  (void)K;
  if (split_k <= 1 || M <= 0 || N <= 0) return 0;
  return (size_t)split_k * (size_t)M * (size_t)N * 4;
}

int pg_gemm_f32(int transa, int transb, int64_t M, int64_t N, int64_t K, float alpha,
                const float* A, int64_t lda, const float* B, int64_t ldb, float beta, float* C,
                int64_t ldc, const float* bias, int act, float slope, int split_k, void* ws,
                size_t ws_bytes, pg_stream_t stream) {
  if (M < 0 || N < 0 || K < 0 || M > INT32_MAX || N > INT32_MAX || K > INT32_MAX)
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_f32: bad sizes");
  if (ldc < N || (!transa && lda < K) || (transa && lda < M) || (!transb && ldb < N) ||
      (transb && ldb < K))
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_f32: leading dimension too small");
  if (act != PG_ACT_NONE && act != PG_ACT_RELU && act != PG_ACT_LEAKY)
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_f32: bad act %d", act);
  if (split_k < 1) split_k = 1;
  if (split_k > 1 && (bias || act != PG_ACT_NONE || (beta != 0.f && beta != 1.f)))
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_f32: split_k > 1 takes no bias/act, beta 0|1");
  if (M == 0 || N == 0) return pg::ok();
  if (split_k > 1 && ws_bytes < pg_gemm_f32_workspace(M, N, K, split_k))
    return pg::set_error(PG_ERR_WORKSPACE, "pg_gemm_f32: workspace too small");
  // float4 loads run along k for A (not transposed) / B^T, along m / n otherwise: the
  // run's extent must be a multiple of 4 so no vector straddles the matrix edge
  const bool va = al16(A) && (lda % 4) == 0 && ((transa ? M : K) % 4) == 0;
  const bool vb = al16(B) && (ldb % 4) == 0 && ((transb ? K : N) % 4) == 0;
  int kps = (int)K;
  if (split_k > 1) {
    kps = (int)((K + split_k - 1) / split_k);
    kps = (kps + BK - 1) / BK * BK;
    split_k = (int)((K + kps - 1) / kps);
    if (split_k < 1) split_k = 1;
  }
  dim3 grid((unsigned)((N + BN - 1) / BN), (unsigned)((M + BM - 1) / BM), (unsigned)split_k);
  hipStream_t st = (hipStream_t)stream;
  const bool split = split_k > 1;
  int rc;
#define PG_DISPATCH(TA_, TB_)                                                                  \
  rc = split ? launch_typed<TA_, TB_, true>(va, vb, act, grid, st, (int)M, (int)N, (int)K, kps,   \
                                            alpha, A, lda, B, ldb, beta, C, ldc, bias, slope,     \
                                            (float*)ws)                                           \
             : launch_typed<TA_, TB_, false>(va, vb, act, grid, st, (int)M, (int)N, (int)K, kps,  \
                                             alpha, A, lda, B, ldb, beta, C, ldc, bias, slope,    \
                                             nullptr);
  if (!transa && !transb) { PG_DISPATCH(false, false) }
  else if (!transa && transb) { PG_DISPATCH(false, true) }
  else if (transa && !transb) { PG_DISPATCH(true, false) }
  else { PG_DISPATCH(true, true) }
#undef PG_DISPATCH
  if (rc != PG_OK) return pg::set_error(rc, "pg_gemm_f32: dispatch failed");
  if (split) {
    const int64_t n = M * N;
    const int blocks = (int)std::min<int64_t>(4096, (n + 255) / 256);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, (const float*)ws,
                       split_k, (int)M, (int)N, alpha, beta, C, ldc);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return pg::set_error((int)e, "pg_gemm_f32: launch failed: %s", hipGetErrorString(e));
  return pg::ok();
}

}  // extern "C"
