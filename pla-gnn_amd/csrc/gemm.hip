// fp32 GEMM on the gfx950 matrix cores (v_mfma_f32_32x32x2_f32: exact f32 products,
// f32 accumulate; gfx950 has no xf32 shortcut) with a fused epilogue. Serves every
// nn.Linear of the PLA-GNN step: SAGEConv's fc_pool / fc_self / fc_neigh
// (code/model.py:13-15) and liner1 / liner2 (code/model.py:16-17), forward and backward.
//
// Epilogue (pg_gemm_epilogue_t): + bias row vector, relu / leaky_relu, or the fused
// activation backward (multiply by act'(y) of a given activation output y), and the row
// sums of op(A) (for a weight-gradient GEMM dY^T X these are the bias gradients
// sum_nodes dY, computed from the A tiles already staged in LDS).
//
// Tiling: BM x BN per 256-thread workgroup (BM, BN in {64, 128}), K step 32; the four
// waves form a 2 x 2 grid, each owning (BM/2) x (BN/2) = TM x TN MFMA tiles of 32 x 32.
// Global -> register prefetch of the next K tile overlaps the MFMAs of the current one
// (a K step of 64 proved slower: the doubled staging registers halve occupancy). Workgroups are ordered so the
// column tiles of one row tile are consecutive on one XCD (`blockIdx % 8` group, the
// bijective remap of cdna_hip_programming.md §5): the A rows they share stay in that
// XCD's L2.
// LDS layout follows the global layout so every staging store is a ds_write_b128:
//   A not transposed (A[m][k]) -> As[m][k] (k contiguous, row stride BK+4 floats: the
//   16-lane groups of ds_read_b128 hit 16 distinct 4-bank slots since 9 is odd);
//   A transposed (A[k][m])     -> As[k][m] (m contiguous, read by ds_read_b32);
//   the same for B with n in place of m.
// K is consumed in a permuted order: at MFMA step s a lane of half h supplies
// k = 16 h + s (not 2 s + h) for A and B alike, so one lane's k-values are contiguous in
// a [row][k] image (ds_read_b128). Each MFMA still pairs A and B at equal k, so the
// product is exact f32 with a fixed (permuted) summation order.
// MFMA 32x32x2 f32 operand map (cdna_hip_programming.md §3): lane l holds
// A[i = l & 31][kk = l >> 5] and B[kk = l >> 5][j = l & 31]; the accumulator holds
// C[row = (r & 3) + 8 (r >> 2) + 4 (l >> 5)][col = l & 31] in register r.
// Long-K products (weight gradients, K = number of nodes) use split-K with partial
// slabs summed in a fixed order (deterministic).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "common.hpp"
#include "gemm_common.hpp"

namespace {

using namespace pg_gemm;

constexpr int BK = 32;
constexpr int HK = BK / 2;  // k-values per lane half per K step
constexpr int kThreads = 256;
constexpr int KPAD = BK + 4;  // [row][k] image row stride (floats)
// Compile-time tuning knobs (variant builds only: make variant VFLAGS=-D...; the shipped
// library reads nothing from the environment):
//   PG_GEMM_TILE_FORCE = BM * 1000 + BN forces one tile (64|128 each), 0 = the heuristic;
//   PG_SPLIT_TARGET    = workgroups a split-K product aims at (measured best: 1024).
#ifndef PG_GEMM_TILE_FORCE
#define PG_GEMM_TILE_FORCE 0
#endif
#ifndef PG_SPLIT_TARGET
#define PG_SPLIT_TARGET 1024
#endif
#ifndef PG_SPLIT_TILE
#define PG_SPLIT_TILE 64064  // BM * 1000 + BN of split-K products (weight gradients)
#endif
constexpr int kSplitBM = PG_SPLIT_TILE / 1000, kSplitBN = PG_SPLIT_TILE % 1000;
//   PG_GEMM_ALGO       = 1: products whose operands allow 16-B loads run on the bf16 matrix
//                        cores as three-piece splits (gemm_x3.hip), 0: f32 MFMA only;
//   PG_X3_TILE_FORCE   = BM * 1000 + BN forces one tile of the three-piece kernel;
//   PG_X3_SPLIT_TARGET = workgroups a split-K product of the three-piece kernel aims at.
#ifndef PG_GEMM_ALGO
#define PG_GEMM_ALGO 1
#endif
#ifndef PG_X3_TILE_FORCE
#define PG_X3_TILE_FORCE 0
#endif
#ifndef PG_X3_GROUP_TARGET
// workgroups of a grouped split-K launch: three 128 x 128 per CU, two 128 x 256 per CU
#define PG_X3_GROUP_TARGET (kX3GroupBN > 128 ? 512 : 768)
#endif
#ifndef PG_X3_MIN_SLICE
#define PG_X3_MIN_SLICE 128  // shortest K slice of a split product of the three-piece kernel
#endif
#ifndef PG_X3_SPLIT_TARGET
#define PG_X3_SPLIT_TARGET 512
#endif
#ifndef PG_GEMM_STAMP
#define PG_GEMM_STAMP 0  // probe builds only: per-workgroup clock stamps (scripts/probes)
#endif
#if PG_GEMM_STAMP
__device__ unsigned long long pg_gemm_stamp[65536][4];
__device__ unsigned long long pg_gemm_kstamp[64][64];  // shader clock at each K-step barrier
__device__ unsigned long long pg_gemm_kphase[64][4];   // start, prologue done, loop done, end
#endif

using f32x16 = __attribute__((ext_vector_type(16))) float;

// Load a ROWS x BK tile of a matrix stored [row][k] (k contiguous) or [k][row] (KMAJ),
// rows [r0, r0+ROWS) x k [k0, k0+BK), zero outside [0,R) x [0,kz1). 4 floats per unit.
template <int ROWS, bool KMAJ, bool VEC>
struct TileLoader {
  static constexpr int UNITS = ROWS * BK / 4;   // float4 units per tile
  static constexpr int PER = UNITS / kThreads;  // per thread
  static constexpr int UPR = BK / 4;            // units per [row][k] row
  float r[PER][4];

  __device__ __forceinline__ void load(const float* __restrict__ P, int64_t ld, int r0, int R,
                                       int k0, int kz1, int tid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = tid + i * kThreads;
      int row, k;
      if constexpr (!KMAJ) {
        row = q / UPR;
        k = (q % UPR) << 2;
      } else {
        k = q / (ROWS / 4);
        row = (q % (ROWS / 4)) << 2;
      }
      const int gr = r0 + row, gk = k0 + k;
      if constexpr (!KMAJ) {
        const float* p = P + (int64_t)gr * ld + gk;
        const bool okr = gr < R;
        if constexpr (VEC) {
          if (okr && gk < kz1) {
            const float4 t = *reinterpret_cast<const float4*>(p);
            r[i][0] = t.x; r[i][1] = t.y; r[i][2] = t.z; r[i][3] = t.w;
          } else {
            r[i][0] = r[i][1] = r[i][2] = r[i][3] = 0.f;
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) r[i][j] = (okr && gk + j < kz1) ? p[j] : 0.f;
        }
      } else {
        const float* p = P + (int64_t)gk * ld + gr;
        const bool okk = gk < kz1;
        if constexpr (VEC) {
          if (okk && gr < R) {
            const float4 t = *reinterpret_cast<const float4*>(p);
            r[i][0] = t.x; r[i][1] = t.y; r[i][2] = t.z; r[i][3] = t.w;
          } else {
            r[i][0] = r[i][1] = r[i][2] = r[i][3] = 0.f;
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) r[i][j] = (okk && gr + j < R) ? p[j] : 0.f;
        }
      }
    }
  }

  // store into the LDS image: [row][KPAD] (!KMAJ) or [k][ROWS + 4] (KMAJ)
  __device__ __forceinline__ void store(float* __restrict__ S, int tid) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = tid + i * kThreads;
      float* d;
      if constexpr (!KMAJ) {
        d = S + (q / UPR) * KPAD + ((q % UPR) << 2);
      } else {
        d = S + (q / (ROWS / 4)) * (ROWS + 4) + ((q % (ROWS / 4)) << 2);
      }
      *reinterpret_cast<float4*>(d) = make_float4(r[i][0], r[i][1], r[i][2], r[i][3]);
    }
  }
};

template <int ROWS, bool KMAJ>
constexpr int image_floats() {
  return KMAJ ? BK * (ROWS + 4) : ROWS * KPAD;
}

// 16 k-values (chunk c of lane half h) for MFMA row/col `rc` from an LDS image.
template <int ROWS, bool KMAJ>
__device__ __forceinline__ void read_frag(const float* __restrict__ S, int rc, int h, int c,
                                          float (&f)[16]) {
  const int kb = h * HK + c * 16;
  if constexpr (!KMAJ) {
    const float4* p = reinterpret_cast<const float4*>(S + rc * KPAD + kb);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 t = p[q];
      f[4 * q + 0] = t.x; f[4 * q + 1] = t.y; f[4 * q + 2] = t.z; f[4 * q + 3] = t.w;
    }
  } else {
#pragma unroll
    for (int s = 0; s < 16; ++s) f[s] = S[(kb + s) * (ROWS + 4) + rc];
  }
}

// Row sums of the A tile in LDS over its BK k-values: thread t owns row t % BM and the
// k-values k = t / BM, t / BM + G, ... (G = 256 / BM groups). The row sums are bias
// gradients, sums over all nodes whose terms largely cancel: they accumulate in float64
// (a float32 running sum over a K-slice of ~1000 nodes measured up to 1e-4 of the result
// off), rounded to float32 once per slice.
template <int BM, bool AK>
__device__ __forceinline__ double tile_rowsum(const float* __restrict__ As, int tid) {
  constexpr int G = kThreads / BM;
  const int m = tid % BM, g = tid / BM;
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < BK / G; ++i) {
    const int k = g + i * G;
    s += AK ? As[k * (BM + 4) + m] : As[m * KPAD + k];
  }
  return s;
}

// Row sums of op(A) (combined over the k-groups in order) and the epilogue of one tile.
template <int BM, int BN, int EPI>
__device__ __forceinline__ void finish_tile(
    const f32x16 (&acc)[BM / 64][BN / 64], double rs, bool do_rs, double* __restrict__ rsred, int tid,
    int m0, int n0, int M, int N, float alpha, float beta, float* __restrict__ C, int64_t ldc,
    const float* __restrict__ bias, float slope, const float* __restrict__ dact, int64_t lddact,
    float* __restrict__ rowsum, float* __restrict__ ws, float* __restrict__ ws_rowsum, int kz) {
  constexpr bool SPLIT = EPI == EPI_SPLIT;
  constexpr int TM = BM / 64, TN = BN / 64;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, h = lane >> 5, l32 = lane & 31;
  if (do_rs) {
    __syncthreads();
    rsred[tid] = rs;
    __syncthreads();
    if (tid < BM && m0 + tid < M) {
      double t = 0.0;
      for (int g = 0; g < kThreads / BM; ++g) t += rsred[g * BM + tid];
      if constexpr (SPLIT) ws_rowsum[(int64_t)kz * M + m0 + tid] = (float)t;
      else rowsum[m0 + tid] = (float)t;
    }
  }

  // epilogue ----------------------------------------------------------------------------
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * (BN / 2) + j * 32 + l32;
    if (col >= N) continue;
    const float bv = (!SPLIT && bias) ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * (BM / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row >= M) continue;
        if constexpr (SPLIT) {
          ws[((int64_t)kz * M + row) * N + col] = acc[i][j][r];
        } else {
          float v = alpha * acc[i][j][r];
          if (beta != 0.f) v = v + beta * C[(int64_t)row * ldc + col];
          if (bias) v = v + bv;
          float y = 0.f;
          if constexpr (EPI == EPI_DRELU || EPI == EPI_DLEAKY) y = dact[(int64_t)row * lddact + col];
          C[(int64_t)row * ldc + col] = epi_apply<EPI>(v, y, slope);
        }
      }
    }
  }
}

// The same through LDS: the accumulator tile is transposed into a [BM][BN] LDS image
// (the staging images are free by now) and written out row-major with 16-B loads/stores,
// instead of one 4-B store per lane and accumulator register. Needs N % 4 == 0 and 16-B
// aligned C / ldc (and dact / bias when present).
template <int BM, int BN, int EPI>
__device__ __forceinline__ void finish_tile_lds(
    const f32x16 (&acc)[BM / 64][BN / 64], double rs, bool do_rs, float* __restrict__ lds, int tid,
    int m0, int n0, int M, int N, float alpha, float beta, float* __restrict__ C, int64_t ldc,
    const float* __restrict__ bias, float slope, const float* __restrict__ dact, int64_t lddact,
    float* __restrict__ rowsum, float* __restrict__ ws, float* __restrict__ ws_rowsum, int kz) {
  constexpr bool SPLIT = EPI == EPI_SPLIT;
  constexpr int TM = BM / 64, TN = BN / 64;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, h = lane >> 5, l32 = lane & 31;
  if (do_rs) {
    double* rsred = reinterpret_cast<double*>(lds);
    rsred[tid] = rs;
    __syncthreads();
    if (tid < BM && m0 + tid < M) {
      double t = 0.0;
      for (int g = 0; g < kThreads / BM; ++g) t += rsred[g * BM + tid];
      if constexpr (SPLIT) ws_rowsum[(int64_t)kz * M + m0 + tid] = (float)t;
      else rowsum[m0 + tid] = (float)t;
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * (BM / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        lds[row * BN + wn * (BN / 2) + j * 32 + l32] = acc[i][j][r];
      }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < BM * BN / 4 / kThreads; ++it) {
    const int u = it * kThreads + tid;
    const int row = u / (BN / 4), c = (u % (BN / 4)) * 4;
    const int gr = m0 + row, gc = n0 + c;
    if (gr >= M || gc >= N) continue;
    float4 v = *reinterpret_cast<const float4*>(lds + row * BN + c);
    if constexpr (SPLIT) {
      *reinterpret_cast<float4*>(ws + ((int64_t)kz * M + gr) * N + gc) = v;
    } else {
      float* cp = C + (int64_t)gr * ldc + gc;
      float o[4] = {alpha * v.x, alpha * v.y, alpha * v.z, alpha * v.w};
      if (beta != 0.f) {
        const float4 c4 = *reinterpret_cast<const float4*>(cp);
        o[0] = o[0] + beta * c4.x; o[1] = o[1] + beta * c4.y;
        o[2] = o[2] + beta * c4.z; o[3] = o[3] + beta * c4.w;
      }
      if (bias) {
        const float4 b4 = *reinterpret_cast<const float4*>(bias + gc);
        o[0] = o[0] + b4.x; o[1] = o[1] + b4.y; o[2] = o[2] + b4.z; o[3] = o[3] + b4.w;
      }
      float y[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI == EPI_DRELU || EPI == EPI_DLEAKY) {
        const float4 d4 = *reinterpret_cast<const float4*>(dact + (int64_t)gr * lddact + gc);
        y[0] = d4.x; y[1] = d4.y; y[2] = d4.z; y[3] = d4.w;
      }
      *reinterpret_cast<float4*>(cp) = make_float4(epi_apply<EPI>(o[0], y[0], slope), epi_apply<EPI>(o[1], y[1], slope),
                                                   epi_apply<EPI>(o[2], y[2], slope), epi_apply<EPI>(o[3], y[3], slope));
    }
  }
}

#if PG_GEMM_STAMP
__device__ __forceinline__ void stamp(unsigned long long st_rt, unsigned long long st_ck, int tid) {
  if (tid == 0 && blockIdx.x < 65536) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    pg_gemm_stamp[blockIdx.x][0] = st_rt;
    pg_gemm_stamp[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
    pg_gemm_stamp[blockIdx.x][2] = __builtin_amdgcn_s_memtime() - st_ck;
    if (blockIdx.x < 64) pg_gemm_kphase[blockIdx.x][3] = st_ck + pg_gemm_stamp[blockIdx.x][2];
    pg_gemm_stamp[blockIdx.x][3] = ((unsigned long long)xcc << 32) | hw;
  }
}
#endif

// Fallback kernel for operands the LDS-DMA kernel cannot take (a row stride or extent that
// is not a multiple of 4 floats, or a base address that is not 16-B aligned: the drop-in
// path's 503-wide inputs): K tiles go global -> registers -> LDS, one image per operand.
// TA: A stored K x M (use A^T). TB: B stored N x K (use B^T).
template <int BM, int BN, bool TA, bool TB, bool VA, bool VB, int EPI>
__global__ __launch_bounds__(kThreads) void gemm_f32_kernel(
    int M, int N, int K, int k_per_split, int tiles_n, int tiles, float alpha,
    const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb, float beta,
    float* __restrict__ C, int64_t ldc, const float* __restrict__ bias, float slope,
    const float* __restrict__ dact, int64_t lddact, float* __restrict__ rowsum,
    float* __restrict__ ws, float* __restrict__ ws_rowsum) {
  constexpr bool AK = TA;    // A image k-major ([k][m]) when A is stored transposed
  constexpr bool BKM = !TB;  // B image k-major ([k][n]) when B is stored K x N
  constexpr int TM = BM / 64, TN = BN / 64;  // 32x32 tiles per wave (2x2 waves)
  __shared__ __attribute__((aligned(16))) float As_[image_floats<BM, AK>()];
  __shared__ __attribute__((aligned(16))) float Bs_[image_floats<BN, BKM>()];
  __shared__ double rsred[kThreads];

  // XCD-aware tile order: blocks b, b+8, ... share an XCD; give each such group a
  // contiguous run of tile ids (row-major over [tile_m][tile_n]).
  const int b = blockIdx.x;
  const int q8 = tiles / 8, r8 = tiles % 8, x8 = b % 8;
  const int tile = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + b / 8;
  const int tm = tile / tiles_n, tn = tile % tiles_n;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = tm * BM;
  const int n0 = tn * BN;
  const int kz0 = blockIdx.z * k_per_split;
  const int kz1 = min(K, kz0 + k_per_split);
  const int h = lane >> 5;
  const int l32 = lane & 31;
  const bool do_rs = rowsum != nullptr && tn == 0;
  double rs = 0.0;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  TileLoader<BM, AK, VA> la;
  TileLoader<BN, BKM, VB> lb;
  if (kz0 < kz1) {
    la.load(A, lda, m0, M, kz0, kz1, tid);
    lb.load(B, ldb, n0, N, kz0, kz1, tid);
    la.store(As_, tid);
    lb.store(Bs_, tid);
    __syncthreads();
    for (int k0 = kz0; k0 < kz1; k0 += BK) {
      const bool more = k0 + BK < kz1;
      if (more) {  // the next tile's global loads overlap this tile's MFMAs
        la.load(A, lda, m0, M, k0 + BK, kz1, tid);
        lb.load(B, ldb, n0, N, k0 + BK, kz1, tid);
      }
      if (do_rs) rs += tile_rowsum<BM, AK>(As_, tid);
#pragma unroll
      for (int c = 0; c < HK / 16; ++c) {
        float fa[TM][16], fb[TN][16];
#pragma unroll
        for (int i = 0; i < TM; ++i) read_frag<BM, AK>(As_, wm * (BM / 2) + i * 32 + l32, h, c, fa[i]);
#pragma unroll
        for (int j = 0; j < TN; ++j) read_frag<BN, BKM>(Bs_, wn * (BN / 2) + j * 32 + l32, h, c, fb[j]);
#pragma unroll
        for (int s = 0; s < 16; ++s)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
      }
      __syncthreads();
      if (more) {
        la.store(As_, tid);
        lb.store(Bs_, tid);
        __syncthreads();
      }
    }
  }
  finish_tile<BM, BN, EPI>(acc, rs, do_rs, rsred, tid, m0, n0, M, N, alpha, beta, C, ldc, bias,
                           slope, dact, lddact, rowsum, ws, ws_rowsum, blockIdx.z);
}

// ---------------------------------------------------------------------------------------
// Main kernel (16-B aligned operands with extents that are multiples of 4): LDS-DMA staging.
//
// K tiles go global -> LDS by global_load_lds_dwordx4 (no register round trip, no ds_write)
// into two LDS images per operand; the tile for step t+1 is issued at the top of step t and
// waited for by the single barrier of step t. Fragments are read in chunks of 4 k-values
// (one ds_read_b128, or 4 ds_read_b32 for a k-major image) one chunk ahead of the MFMAs
// that consume them, across K steps too: the barrier sits after chunk 2's MFMAs and the
// next tile's chunk 0 is read under chunk 3's, so the LDS traffic of a wave overlaps its
// own MFMAs instead of waiting for other waves to fill the matrix pipe.
//
// LDS images (no padding; one DMA wave-instruction fills 1 KiB contiguously):
//   [row][k] (operand stored k-contiguous): row r = 128 B = 8 chunks of 4 k-values; chunk c
//     is stored at chunk c ^ ((r >> 1) & 7): the 16-lane groups of ds_read_b128 (16
//     consecutive rows, same chunk) hit 16 distinct 16-B bank slots. The XOR is applied
//     to the DMA's per-lane SOURCE address (the destination is lane-linear).
//   [k][row] (operand stored row-contiguous): plain; ds_read_b32 over 32 consecutive rows.
// Rows past the matrix edge are loaded from a clamped (valid) row: they only feed output
// rows / columns that are never stored. In a partial last K tile the units past K are
// zero-filled by ds_write instead of loaded.
template <int ROWS, bool KMAJ>
__device__ __forceinline__ int img_off(int row, int k) {  // float offset of (row, k)
  if constexpr (KMAJ) return k * ROWS + row;
  else return row * BK + ((((k >> 2) ^ ((row >> 1) & 7))) << 2) + (k & 3);
}

template <int ROWS, bool KMAJ, bool FULL>
__device__ __forceinline__ void dma_tile(const float* __restrict__ P, int64_t ld, int r0, int R,
                                         int k0, int kvalid, float* S, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < ROWS / 32; ++j) {
    const int piece = j * 4 + wave;  // 1-KiB piece of the image
    const int u = piece * 64 + lane;  // 16-B unit
    const float* src;
    bool valid;
    if constexpr (!KMAJ) {
      const int row = u >> 3, c = (u & 7) ^ ((row >> 1) & 7);
      valid = 4 * c < kvalid;
      src = P + (int64_t)min(r0 + row, R - 1) * ld + k0 + 4 * c;
    } else {
      const int k = u / (ROWS / 4), c4 = u % (ROWS / 4);
      valid = k < kvalid;
      src = P + (int64_t)(k0 + k) * ld + min(r0 + 4 * c4, R - 4);
    }
    // units past K (partial last tile) are zero-filled by the lane that owns them instead
    // (a DMA lane masked off by EXEC writes nothing)
    if (FULL || valid) __builtin_amdgcn_global_load_lds(src, S + piece * 256, 16, 0, 0);
    else *reinterpret_cast<float4*>(S + u * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int ROWS, bool KMAJ>
__device__ __forceinline__ void frag_chunk(const float* __restrict__ S, int rc, int h, int q,
                                           float (&f)[4]) {
  const int kb = h * HK + 4 * q;
  if constexpr (!KMAJ) {
    const float4 t = *reinterpret_cast<const float4*>(S + img_off<ROWS, false>(rc, kb));
    f[0] = t.x; f[1] = t.y; f[2] = t.z; f[3] = t.w;
  } else {
#pragma unroll
    for (int s = 0; s < 4; ++s) f[s] = S[(kb + s) * ROWS + rc];
  }
}

template <int BM, bool AK>
__device__ __forceinline__ double img_rowsum(const float* __restrict__ As, int tid) {
  constexpr int G = kThreads / BM;
  const int m = tid % BM, g = tid / BM;
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < BK / G; ++i) s += As[img_off<BM, AK>(m, g + i * G)];
  return s;
}

template <int BM, int BN, bool TA, bool TB, int EPI>
__global__ __launch_bounds__(kThreads) void gemm_dma_kernel(
    int M, int N, int K, int k_per_split, int tiles_n, int tiles, float alpha,
    const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb, float beta,
    float* __restrict__ C, int64_t ldc, const float* __restrict__ bias, float slope,
    const float* __restrict__ dact, int64_t lddact, float* __restrict__ rowsum,
    float* __restrict__ ws, float* __restrict__ ws_rowsum, int vec_out, int n_split) {
  constexpr bool AK = TA, BKM = !TB;
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int IA = BM * BK, IB = BN * BK;  // image sizes (floats)
  // one LDS array: [A0 | A1 | B0 | B1] (a second __shared__ object can make hipcc drain
  // the DMA at every LDS read)
  __shared__ __attribute__((aligned(16))) float lds[2 * (IA + IB)];

  // XCD-aware order over the (slice, tile) items of a 1-D grid: blocks b, b + 8, ... share
  // an XCD and take a contiguous run of slice-major item ids, so an XCD holds whole
  // K-slices (every tile of a slice reads the same K rows of A and B: they meet in one L2)
  // and, without split, the column tiles of a row tile (their shared A rows)
  const int b = blockIdx.x;
  const int items = tiles * n_split;
  const int q8 = items / 8, r8 = items % 8, x8 = b % 8;
  const int item = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + b / 8;
  const int kz = item / tiles, tile = item % tiles;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, h = lane >> 5, l32 = lane & 31;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kz0 = kz * k_per_split;
  const int kz1 = min(K, kz0 + k_per_split);
  const bool do_rs = rowsum != nullptr && tn == 0;
#if PG_GEMM_STAMP
  unsigned long long st_rt = __builtin_amdgcn_s_memrealtime(), st_ck = __builtin_amdgcn_s_memtime();
#endif
  double rs = 0.0;
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = kz1 > kz0 ? (kz1 - kz0 + BK - 1) / BK : 0;
  // issue the DMA of K tile t into LDS image `buf`
  auto issue = [&](int t, int buf) {
    const int k0 = kz0 + t * BK;
    if (kz1 - k0 >= BK) {
      dma_tile<BM, AK, true>(A, lda, m0, M, k0, BK, lds + buf * IA, wave, lane);
      dma_tile<BN, BKM, true>(B, ldb, n0, N, k0, BK, lds + 2 * IA + buf * IB, wave, lane);
    } else {
      dma_tile<BM, AK, false>(A, lda, m0, M, k0, kz1 - k0, lds + buf * IA, wave, lane);
      dma_tile<BN, BKM, false>(B, ldb, n0, N, k0, kz1 - k0, lds + 2 * IA + buf * IB, wave, lane);
    }
  };

  if (nk > 0) {
    issue(0, 0);
    __syncthreads();
#if PG_GEMM_STAMP
    if (tid == 0 && blockIdx.x < 64) pg_gemm_kphase[blockIdx.x][1] = __builtin_amdgcn_s_memtime();
#endif
    float fa[2][TM][4], fb[2][TN][4];
    const int ra = wm * (BM / 2) + l32, rb = wn * (BN / 2) + l32;
#pragma unroll
    for (int i = 0; i < TM; ++i) frag_chunk<BM, AK>(lds, ra + i * 32, h, 0, fa[0][i]);
#pragma unroll
    for (int j = 0; j < TN; ++j) frag_chunk<BN, BKM>(lds + 2 * IA, rb + j * 32, h, 0, fb[0][j]);
    for (int t = 0; t < nk; ++t) {
      const int cur = t & 1;
      const bool more = t + 1 < nk;
      if (more) issue(t + 1, cur ^ 1);
      const float* As = lds + cur * IA;
      const float* Bs = lds + 2 * IA + cur * IB;
      if (do_rs) rs += img_rowsum<BM, AK>(As, tid);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int u = q & 1;
        if (q < 3) {
#pragma unroll
          for (int i = 0; i < TM; ++i) frag_chunk<BM, AK>(As, ra + i * 32, h, q + 1, fa[u ^ 1][i]);
#pragma unroll
          for (int j = 0; j < TN; ++j) frag_chunk<BN, BKM>(Bs, rb + j * 32, h, q + 1, fb[u ^ 1][j]);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[u][i][s], fb[u][j][s], acc[i][j], 0, 0, 0);
        if (q == 2) {
          __syncthreads();  // tile t+1 landed (vmcnt) and every wave is past its reads of tile t-1
#if PG_GEMM_STAMP
          if (tid == 0 && blockIdx.x < 64 && t < 64) pg_gemm_kstamp[blockIdx.x][t] = __builtin_amdgcn_s_memtime();
#endif
          if (more) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
              frag_chunk<BM, AK>(lds + (cur ^ 1) * IA, ra + i * 32, h, 0, fa[0][i]);
#pragma unroll
            for (int j = 0; j < TN; ++j)
              frag_chunk<BN, BKM>(lds + 2 * IA + (cur ^ 1) * IB, rb + j * 32, h, 0, fb[0][j]);
          }
        }
      }
    }
    __syncthreads();  // the row-sum scratch below reuses the staging array
  }
#if PG_GEMM_STAMP
  if (tid == 0 && blockIdx.x < 64) {
    pg_gemm_kphase[blockIdx.x][0] = st_ck;
    pg_gemm_kphase[blockIdx.x][2] = __builtin_amdgcn_s_memtime();
  }
#endif
  if (vec_out)
    finish_tile_lds<BM, BN, EPI>(acc, rs, do_rs, lds, tid, m0, n0, M, N, alpha, beta, C, ldc, bias,
                                 slope, dact, lddact, rowsum, ws, ws_rowsum, kz);
  else
    finish_tile<BM, BN, EPI>(acc, rs, do_rs, reinterpret_cast<double*>(lds), tid, m0, n0, M, N, alpha, beta, C,
                             ldc, bias, slope, dact, lddact, rowsum, ws, ws_rowsum, kz);
#if PG_GEMM_STAMP
  stamp(st_rt, st_ck, tid);
#endif
}


struct Args {
  int M, N, K, kps, tiles_n, tiles;
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
  int vec_out;
};

template <int BM, int BN, bool TA, bool TB, bool VA, bool VB>
int launch_epi(int epi, dim3 grid, hipStream_t st, const Args& a) {
#define PG_L(EPI_)                                                                          \
  hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, TA, TB, VA, VB, EPI_>), grid, dim3(kThreads), 0, \
                     st, a.M, a.N, a.K, a.kps, a.tiles_n, a.tiles, a.alpha, a.A, a.lda, a.B,  \
                     a.ldb, a.beta, a.C, a.ldc, a.bias, a.slope, a.dact, a.lddact, a.rowsum,  \
                     a.ws, a.ws_rowsum)
  switch (epi) {
    case EPI_NONE: PG_L(EPI_NONE); break;
    case EPI_RELU: PG_L(EPI_RELU); break;
    case EPI_LEAKY: PG_L(EPI_LEAKY); break;
    case EPI_DRELU: PG_L(EPI_DRELU); break;
    case EPI_DLEAKY: PG_L(EPI_DLEAKY); break;
    case EPI_SPLIT: PG_L(EPI_SPLIT); break;
    default: return PG_ERR_INVALID;
  }
#undef PG_L
  return PG_OK;
}

template <int BM, int BN, bool TA, bool TB>
int launch_dma(int epi, dim3 grid, hipStream_t st, const Args& a) {
#define PG_L(EPI_)                                                                          \
  hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, TA, TB, EPI_>), dim3(grid.x * grid.z), dim3(kThreads), \
                     0, st, a.M, a.N, a.K, a.kps, a.tiles_n, a.tiles, a.alpha, a.A, a.lda, a.B,  \
                     a.ldb, a.beta, a.C, a.ldc, a.bias, a.slope, a.dact, a.lddact, a.rowsum,     \
                     a.ws, a.ws_rowsum, a.vec_out, (int)grid.z)
  switch (epi) {
    case EPI_NONE: PG_L(EPI_NONE); break;
    case EPI_RELU: PG_L(EPI_RELU); break;
    case EPI_LEAKY: PG_L(EPI_LEAKY); break;
    case EPI_DRELU: PG_L(EPI_DRELU); break;
    case EPI_DLEAKY: PG_L(EPI_DLEAKY); break;
    case EPI_SPLIT: PG_L(EPI_SPLIT); break;
    default: return PG_ERR_INVALID;
  }
#undef PG_L
  return PG_OK;
}

template <int BM, int BN, bool TA, bool TB>
int launch_vec(bool va, bool vb, int epi, dim3 grid, hipStream_t st, const Args& a) {
  if (va && vb) return launch_dma<BM, BN, TA, TB>(epi, grid, st, a);
  if (va) return launch_epi<BM, BN, TA, TB, true, false>(epi, grid, st, a);
  if (vb) return launch_epi<BM, BN, TA, TB, false, true>(epi, grid, st, a);
  return launch_epi<BM, BN, TA, TB, false, false>(epi, grid, st, a);
}

template <int BM, int BN>
int launch_trans(bool ta, bool tb, bool va, bool vb, int epi, dim3 grid, hipStream_t st,
                 const Args& a) {
  if (!ta && !tb) return launch_vec<BM, BN, false, false>(va, vb, epi, grid, st, a);
  if (!ta && tb) return launch_vec<BM, BN, false, true>(va, vb, epi, grid, st, a);
  if (ta && !tb) return launch_vec<BM, BN, true, false>(va, vb, epi, grid, st, a);
  return launch_vec<BM, BN, true, true>(va, vb, epi, grid, st, a);
}

// Tile choice (measured on the PLA-GNN step shapes, scripts/gemm_bench.py): split-K
// products (weight gradients) 64 x 64; outputs wider than 512 columns 128 x 128 when that
// still gives >= 3 workgroups per CU, else 64 x 128; 129..512 columns with short K
// (K <= 1024) 128 x 64 (if >= 720 tiles: ~3 workgroups per CU); everything else 64 x 64 (5 workgroups per CU: long-K
// and small products balance best on the finest tile).
inline void pick_tile(int64_t M, int64_t N, int64_t K, int split, int& bm, int& bn) {
  if constexpr (PG_GEMM_TILE_FORCE != 0) {  // variant builds only
    bm = PG_GEMM_TILE_FORCE / 1000;
    bn = PG_GEMM_TILE_FORCE % 1000;
    return;
  }
  auto tiles = [&](int tm, int tn) { return ((M + tm - 1) / tm) * ((N + tn - 1) / tn); };
  bm = bn = 64;
  if (split > 1) {
    bm = kSplitBM;
    bn = kSplitBN;
    return;
  }
  if (N > 512) {
    bn = 128;
    bm = tiles(128, 128) >= 3 * 256 ? 128 : 64;
  } else if (N > 128 && K <= 1024 && tiles(128, 64) >= 3 * 256 - 48) {
    bm = 128;
  }
}

// Tile of the three-piece kernel (measured per cfg2 shape with each tile forced, within 1-3 %
// of the best everywhere): 128 x 128 (4 waves of 64 x 64: 0.5 fragment reads per MFMA)
// wherever that gives >= 2 workgroups per CU; else 128 x 64, else 64 x 64. (Round 6: a
// long-K product with 256-511 128 x 128 tiles, cfg2's fwd.cat.l1, runs 87.2 instead of 91.0
// us on 128 x 64 tiles: 752 tiles share out over 256 CUs, 376 leave 136 CUs one tile idle.) Split products: 128 x 128, ~2 workgroups per CU (512: 1.636 ms/step, 768: 1.667,
// 1024: 1.721).
inline void pick_tile_x3(int64_t M, int64_t N, int64_t K, int split, int& bm, int& bn) {
  if constexpr (PG_X3_TILE_FORCE != 0) {  // variant builds only
    bm = PG_X3_TILE_FORCE / 1000;
    bn = PG_X3_TILE_FORCE % 1000;
    return;
  }
  auto tiles = [&](int tm, int tn) { return ((M + tm - 1) / tm) * ((N + tn - 1) / tn); };
  if (split > 1) {
    bm = M > 64 ? 128 : 64;
    bn = N > 64 ? 128 : 64;
    return;
  }
  bm = bn = 64;
#ifndef PG_X3_LONGK_128
#define PG_X3_LONGK_128 0  // 1: long-K products with 256-511 128 x 128 tiles keep 128 x 128
#endif
  if (tiles(128, 128) >= 512 || (PG_X3_LONGK_128 && tiles(128, 128) >= 256 && K >= 1000)) bm = bn = 128;
  else if (tiles(128, 64) >= 512) bm = 128;
}

// the three-piece kernel takes the product: 16-B loads along every contiguous extent, and
// 16-B epilogue stores
inline bool x3_ok(int transa, int transb, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                  const float* B, int64_t ldb, const float* C, int64_t ldc, const pg_gemm_epilogue_t* ep,
                  bool split, const void* ws) {
  if constexpr (PG_GEMM_ALGO == 0) return false;
  // the three-piece kernel addresses each operand by 32-bit byte offsets
  const int64_t a_ext = transa ? (K - 1) * lda + M : (M - 1) * lda + K;
  const int64_t b_ext = transb ? (N - 1) * ldb + K : (K - 1) * ldb + N;
  if (a_ext * 4 >= ((int64_t)1 << 32) - 64 || b_ext * 4 >= ((int64_t)1 << 32) - 64) return false;
  return al16(A) && lda % 4 == 0 && (transa ? M : K) % 4 == 0 && al16(B) && ldb % 4 == 0 &&
         (transb ? K : N) % 4 == 0 && N % 4 == 0 &&
         (split ? al16(ws) : (al16(C) && ldc % 4 == 0)) && (!ep->bias || al16(ep->bias)) &&
         (!ep->dact || (al16(ep->dact) && ep->lddact % 4 == 0));
}

}  // namespace

extern "C" {

int pg_gemm_f32_split_k(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K < 1024) return 1;
  if constexpr (PG_GEMM_ALGO != 0) {
    // three-piece kernel (the engine's operands are aligned): ~2 128 x 128 workgroups per
    // CU, each slice >= 8 K steps
    int bm, bn;
    pick_tile_x3(M, N, K, 1, bm, bn);
    if (((M + bm - 1) / bm) * ((N + bn - 1) / bn) >= 512) return 1;
    pick_tile_x3(M, N, K, 2, bm, bn);
    const int64_t tiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
    const int64_t target = (PG_X3_SPLIT_TARGET + tiles - 1) / tiles;
    return (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(target, K / PG_X3_MIN_SLICE), 256));
  }
  int bm, bn;
  pick_tile(M, N, K, 1, bm, bn);
  if (((M + bm - 1) / bm) * ((N + bn - 1) / bn) >= 768) return 1;
  // split products run 64 x 64 tiles: ~4 workgroups per CU (256 CUs), each slice >= 3 K
  // steps, at most 256 slices. Measured on the cfg2 step (whole step, batched combine):
  // 1024 workgroups 1.984 ms, 768 1.992, 1280 2.022, 640 / 896 2.06 / 2.03 (not a multiple
  // of the 256 CUs), 512 1.99, 384 2.15.
  const int64_t tiles = ((M + kSplitBM - 1) / kSplitBM) * ((N + kSplitBN - 1) / kSplitBN);
  const int64_t target = (PG_SPLIT_TARGET + tiles - 1) / tiles;
  const int64_t by_k = K / (3 * BK);
  return (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(target, by_k), 256));
}

size_t pg_gemm_f32_workspace(int64_t M, int64_t N, int64_t K, int split_k) {
  (void)K;
  if (split_k <= 1 || M <= 0 || N <= 0) return 0;
  return (size_t)split_k * (size_t)M * (size_t)(N + 1) * 4;
}

}  // extern "C"

namespace {

// defer: split-K partial slabs (and row-sum slices) are left in ws for a later
// pg_gemm_splitk_reduce_batch; *split_used = the slice count actually run.
int gemm_f32_impl(int transa, int transb, int64_t M, int64_t N, int64_t K, float alpha,
                  const float* A, int64_t lda, const float* B, int64_t ldb, float beta, float* C,
                  int64_t ldc, const pg_gemm_epilogue_t* ep, int split_k, void* ws,
                  size_t ws_bytes, pg_stream_t stream, bool defer, int* split_used) {
  const pg_gemm_epilogue_t none{nullptr, PG_ACT_NONE, 0.f, nullptr, 0, nullptr};
  if (!ep) ep = &none;
  const int act = ep->act;
  if (M < 0 || N < 0 || K < 0 || M > INT32_MAX || N > INT32_MAX || K > INT32_MAX)
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_f32: bad sizes");
  if (ldc < N || (!transa && lda < K) || (transa && lda < M) || (!transb && ldb < N) ||
      (transb && ldb < K))
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_f32: leading dimension too small");
  if (act != PG_ACT_NONE && act != PG_ACT_RELU && act != PG_ACT_LEAKY)
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_f32: bad act %d", act);
  if (split_k < 1) split_k = 1;
  if (split_k > 1 && (ep->bias || act != PG_ACT_NONE || ep->dact || (beta != 0.f && beta != 1.f)))
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_f32: split_k > 1 takes no bias/act, beta 0|1");
  if (ep->dact && (act == PG_ACT_NONE || ep->lddact < N))
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_f32: dact needs act relu|leaky and lddact >= N");
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
  const bool split = split_k > 1;
  if (split_used) *split_used = split_k;
  if (defer && !split) return pg::set_error(PG_ERR_INVALID, "pg_gemm_f32_partials: needs split_k > 1");
  hipStream_t st = (hipStream_t)stream;
  float* wsf = split ? (float*)ws : nullptr;
  float* ws_rs = split ? wsf + (int64_t)split_k * M * N : nullptr;  // row-sum slices after the slabs
  const int epi = split ? EPI_SPLIT
                        : ep->dact ? (act == PG_ACT_RELU ? EPI_DRELU : EPI_DLEAKY)
                                   : (act == PG_ACT_RELU ? EPI_RELU : act == PG_ACT_LEAKY ? EPI_LEAKY : EPI_NONE);
  int bm, bn;
  int rc;
  if (x3_ok(transa, transb, M, N, K, A, lda, B, ldb, C, ldc, ep, split, ws)) {
    pick_tile_x3(M, N, K, split_k, bm, bn);
    const int tiles_n = (int)((N + bn - 1) / bn);
    const int tiles = tiles_n * (int)((M + bm - 1) / bm);
    const X3Args xa{transa != 0, transb != 0, bm, bn, epi, (int)M, (int)N, (int)K, kps, tiles_n, tiles,
                    split_k, alpha, A, lda, B, ldb, beta, C, ldc, ep->bias, ep->slope, ep->dact,
                    ep->lddact, ep->rowsum, wsf, ws_rs};
    rc = gemm_x3_launch(xa, st);
  } else {
    pick_tile(M, N, K, split_k, bm, bn);
    const int tiles_n = (int)((N + bn - 1) / bn);
    const int tiles = tiles_n * (int)((M + bm - 1) / bm);
    dim3 grid((unsigned)tiles, 1, (unsigned)split_k);
    // 16-B epilogue stores (finish_tile_lds) when every output-side operand allows them
    const bool vec_out = (N % 4) == 0 && (split ? al16(wsf) : (al16(C) && (ldc % 4) == 0)) &&
                         (!ep->bias || al16(ep->bias)) &&
                         (!ep->dact || (al16(ep->dact) && (ep->lddact % 4) == 0));
    const Args a{(int)M, (int)N, (int)K, kps, tiles_n, tiles, alpha, A, lda, B, ldb, beta, C, ldc,
                 ep->bias, ep->slope, ep->dact, ep->lddact, ep->rowsum, wsf, ws_rs, vec_out ? 1 : 0};
    const bool ta = transa != 0, tb = transb != 0;
    if (bm == 128 && bn == 128)
      rc = launch_trans<128, 128>(ta, tb, va, vb, epi, grid, st, a);
    else if (bm == 64 && bn == 128)
      rc = launch_trans<64, 128>(ta, tb, va, vb, epi, grid, st, a);
    else if (bm == 128)
      rc = launch_trans<128, 64>(ta, tb, va, vb, epi, grid, st, a);
    else
      rc = launch_trans<64, 64>(ta, tb, va, vb, epi, grid, st, a);
  }
  if (rc != PG_OK) return pg::set_error(rc, "pg_gemm_f32: dispatch failed");
  if (split && !defer) {
    const int64_t n = (N % 4 == 0 ? M * N / 4 : M * N) + (ep->rowsum ? M : 0);  // work units
    // threads per output: enough slice groups that each thread sums <= ~8 slices
    const int G = splitk_groups(split_k);
    const int opb = 256 / G;
    const int blocks = (int)std::min<int64_t>(8192, (n + opb - 1) / opb);
#define PG_R(G_)                                                                              \
  hipLaunchKernelGGL(splitk_reduce_kernel<G_>, dim3(blocks), dim3(256), 0, st, (const float*)wsf, \
                     split_k, (int)M, (int)N, alpha, beta, C, ldc, (const float*)ws_rs,          \
                     ep->rowsum)
    if (G == 1) PG_R(1);
    else if (G == 4) PG_R(4);
    else PG_R(16);
#undef PG_R
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return pg::set_error((int)e, "pg_gemm_f32: launch failed: %s", hipGetErrorString(e));
  return pg::ok();
}

// Several split-K combines in one launch: block ranges per job, each job reduced exactly as
// splitk_reduce_kernel<G> does (same G, same order: bitwise the same result).
constexpr int kMaxBatch = 16;
struct BatchArgs {
  pg_splitk_job_t job[kMaxBatch];
  int G[kMaxBatch];
  int first_block[kMaxBatch + 1];
  int n;
};

__global__ __launch_bounds__(256) void splitk_reduce_batch_kernel(BatchArgs a) {
  int k = 0;
  while (k + 1 < a.n && (int)blockIdx.x >= a.first_block[k + 1]) ++k;
  const int blk = blockIdx.x - a.first_block[k];
  const int nblk = a.first_block[k + 1] - a.first_block[k];
  const pg_splitk_job_t& j = a.job[k];
  const float* wr = j.ws + (int64_t)j.split_k * j.M * j.N;
  switch (a.G[k]) {
    case 1: splitk_reduce_body<1>(j.ws, j.split_k, (int)j.M, (int)j.N, j.alpha, j.beta, j.C, j.ldc, wr, j.rowsum, blk, nblk); break;
    case 4: splitk_reduce_body<4>(j.ws, j.split_k, (int)j.M, (int)j.N, j.alpha, j.beta, j.C, j.ldc, wr, j.rowsum, blk, nblk); break;
    default: splitk_reduce_body<16>(j.ws, j.split_k, (int)j.M, (int)j.N, j.alpha, j.beta, j.C, j.ldc, wr, j.rowsum, blk, nblk); break;
  }
}

}  // namespace

extern "C" {

int pg_gemm_f32_cat(int transb, int64_t M, int64_t N, int64_t K1, int64_t K2, float alpha, const float* A1,
                    int64_t lda1, const float* A2, int64_t lda2, const float* B1, int64_t ldb1, const float* B2,
                    int64_t ldb2, float beta, float* C, int64_t ldc, const pg_gemm_epilogue_t* ep,
                    pg_stream_t stream) {
  const pg_gemm_epilogue_t none{nullptr, PG_ACT_NONE, 0.f, nullptr, 0, nullptr};
  if (!ep) ep = &none;
  const int64_t K = K1 + K2;
  if (M < 0 || N < 0 || K1 < 0 || K2 < 0 || M > INT32_MAX || N > INT32_MAX || K > INT32_MAX)
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_f32_cat: bad sizes");
  if (ldc < N || lda1 < K1 || lda2 < K2 || (transb ? (ldb1 < K1 || ldb2 < K2) : (ldb1 < N || ldb2 < N)))
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_f32_cat: leading dimension too small");
  if (ep->act != PG_ACT_NONE && ep->act != PG_ACT_LEAKY)
    return pg::set_error(PG_ERR_UNSUPPORTED, "pg_gemm_f32_cat: act none or leaky");
  if (ep->dact || ep->rowsum)
    return pg::set_error(PG_ERR_UNSUPPORTED, "pg_gemm_f32_cat: no dact / rowsum epilogue");
  if (M == 0 || N == 0) return pg::ok();
  if (K1 % 4 != 0 || K2 <= 0 || K1 <= 0 ||
      !x3_ok(0, transb, M, N, K1, A1, lda1, B1, ldb1, C, ldc, ep, false, nullptr) ||
      !x3_ok(0, transb, M, N, K2, A2, lda2, B2, ldb2, C, ldc, ep, false, nullptr))
    return pg::set_error(PG_ERR_UNSUPPORTED,
                         "pg_gemm_f32_cat: needs K1 %% 4 == 0 and operands the three-piece kernel takes");
  int bm, bn;
  pick_tile_x3(M, N, K, 1, bm, bn);
  const int tiles_n = (int)((N + bn - 1) / bn);
  const int tiles = tiles_n * (int)((M + bm - 1) / bm);
  const int epi = ep->act == PG_ACT_LEAKY ? EPI_LEAKY : EPI_NONE;
  const X3Args xa{false, transb != 0, bm, bn, epi, (int)M, (int)N, (int)K, (int)K, tiles_n, tiles, 1, alpha, A1,
                  lda1, B1, ldb1, beta, C, ldc, ep->bias, ep->slope, nullptr, 0, nullptr, nullptr, nullptr};
  const int rc = gemm_x3_cat_launch(xa, A2, lda2, B2, ldb2, (int)K1, (hipStream_t)stream);
  const hipError_t e = hipGetLastError();
  if (rc != PG_OK || e != hipSuccess)
    return pg::set_error(rc != PG_OK ? rc : (int)e, "pg_gemm_f32_cat: launch failed");
  return pg::ok();
}

int pg_gemm_f32(int transa, int transb, int64_t M, int64_t N, int64_t K, float alpha,
                const float* A, int64_t lda, const float* B, int64_t ldb, float beta, float* C,
                int64_t ldc, const pg_gemm_epilogue_t* ep, int split_k, void* ws,
                size_t ws_bytes, pg_stream_t stream) {
  return gemm_f32_impl(transa, transb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, ep, split_k, ws,
                       ws_bytes, stream, false, nullptr);
}

int pg_gemm_f32_partials(int transa, int transb, int64_t M, int64_t N, int64_t K, const float* A,
                         int64_t lda, const float* B, int64_t ldb, const pg_gemm_epilogue_t* ep,
                         int split_k, void* ws, size_t ws_bytes, int* split_used, pg_stream_t stream) {
  if (ep && (ep->bias || ep->act != PG_ACT_NONE || ep->dact))
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_f32_partials: the epilogue may only carry rowsum");
  return gemm_f32_impl(transa, transb, M, N, K, 1.f, A, lda, B, ldb, 0.f, nullptr, N, ep, split_k, ws,
                       ws_bytes, stream, true, split_used);
}

int pg_gemm_splitk_reduce_batch(const pg_splitk_job_t* jobs, int n_jobs, pg_stream_t stream) {
  if (n_jobs < 0 || n_jobs > kMaxBatch || (n_jobs > 0 && !jobs))
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_splitk_reduce_batch: 0..%d jobs", kMaxBatch);
  if (n_jobs == 0) return pg::ok();
  BatchArgs a{};
  a.n = n_jobs;
  int blocks = 0;
  for (int k = 0; k < n_jobs; ++k) {
    const pg_splitk_job_t& j = jobs[k];
    if (j.split_k < 1 || j.M <= 0 || j.N <= 0 || !j.ws || !j.C || j.ldc < j.N ||
        (j.beta != 0.f && j.beta != 1.f))
      return pg::set_error(PG_ERR_INVALID, "pg_gemm_splitk_reduce_batch: bad job %d", k);
    a.job[k] = j;
    a.G[k] = splitk_groups(j.split_k);
    a.first_block[k] = blocks;
    const int64_t n = (j.N % 4 == 0 ? j.M * j.N / 4 : j.M * j.N) + (j.rowsum ? j.M : 0);  // work units
    const int opb = 256 / a.G[k];
    blocks += (int)std::min<int64_t>(8192, (n + opb - 1) / opb);
  }
  a.first_block[n_jobs] = blocks;
  hipLaunchKernelGGL(splitk_reduce_batch_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return pg::set_error((int)e, "pg_gemm_splitk_reduce_batch: launch failed: %s", hipGetErrorString(e));
  return pg::ok();
}

}  // extern "C"

namespace {

// The group's plan: one K-slice count for every part, chosen so that the union of the
// parts' 128 x 128 tiles times the slices fills PG_X3_GROUP_TARGET workgroups (three per
// CU), each slice >= PG_X3_MIN_SLICE entries of K; each part's slabs (+ row-sum slices) at
// a 256-B aligned offset of ws.
struct GroupPlan {
  int split[kX3MaxParts];
  int kps[kX3MaxParts];
  size_t off[kX3MaxParts + 1];
};

inline void group_plan(const pg_gemm_part_t* parts, int n, GroupPlan& g) {
  int64_t tiles = 0;
  for (int p = 0; p < n; ++p)
    tiles += ((parts[p].M + kX3GroupBM - 1) / kX3GroupBM) * ((parts[p].N + kX3GroupBN - 1) / kX3GroupBN);
  const int64_t s = std::max<int64_t>(1, PG_X3_GROUP_TARGET / std::max<int64_t>(1, tiles));
  size_t off = 0;
  for (int p = 0; p < n; ++p) {
    const pg_gemm_part_t& q = parts[p];
    int64_t sp = std::max<int64_t>(1, std::min<int64_t>(s, q.K / PG_X3_MIN_SLICE));
    int64_t kps = (q.K + sp - 1) / sp;
    kps = std::max<int64_t>(BK, (kps + BK - 1) / BK * BK);
    sp = std::max<int64_t>(1, (q.K + kps - 1) / kps);
    g.split[p] = (int)sp;
    g.kps[p] = (int)kps;
    g.off[p] = off;
    off += ((size_t)sp * (size_t)std::max<int64_t>(q.M, 0) * (size_t)(std::max<int64_t>(q.N, 0) + 1) * 4 + 255) /
           256 * 256;
  }
  g.off[n] = off;
}

inline bool part_ok(const pg_gemm_part_t& q) {
  const bool bufs = (q.M == 0 || q.N == 0 || q.C) && (q.M == 0 || q.N == 0 || q.K == 0 || (q.A && q.B));
  return bufs && q.M >= 0 && q.N >= 0 && q.K >= 0 && q.M <= INT32_MAX && q.N <= INT32_MAX && q.K <= INT32_MAX &&
         q.ldc >= q.N && (q.transa ? q.lda >= q.M : q.lda >= q.K) && (q.transb ? q.ldb >= q.K : q.ldb >= q.N) &&
         (q.beta == 0.f || q.beta == 1.f);
}

}  // namespace

extern "C" {

size_t pg_gemm_f32_group_workspace(const pg_gemm_part_t* parts, int n) {
  if (n <= 0 || n > kX3MaxParts || !parts) return 0;
  GroupPlan g;
  group_plan(parts, n, g);
  size_t need = g.off[n];
  for (int p = 0; p < n; ++p) {  // the per-part path (operands the grouped kernel does not take)
    const pg_gemm_part_t& q = parts[p];
    need = std::max(need, pg_gemm_f32_workspace(q.M, q.N, q.K, pg_gemm_f32_split_k(q.M, q.N, q.K)));
  }
  return std::max<size_t>(need, 256);
}

int pg_gemm_f32_group(const pg_gemm_part_t* parts, int n, void* ws, size_t ws_bytes, pg_stream_t stream) {
  if (n < 0 || n > kX3MaxParts || (n > 0 && !parts))
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_f32_group: 0..%d parts", kX3MaxParts);
  if (n == 0) return pg::ok();
  for (int p = 0; p < n; ++p)
    if (!part_ok(parts[p])) return pg::set_error(PG_ERR_INVALID, "pg_gemm_f32_group: bad part %d", p);
  if (ws_bytes < pg_gemm_f32_group_workspace(parts, n) || !ws)
    return pg::set_error(PG_ERR_WORKSPACE, "pg_gemm_f32_group: workspace too small");
  GroupPlan g;
  group_plan(parts, n, g);
  const pg_gemm_epilogue_t none{nullptr, PG_ACT_NONE, 0.f, nullptr, 0, nullptr};
  bool grouped = PG_GEMM_ALGO != 0;
  for (int p = 0; p < n && grouped; ++p) {
    const pg_gemm_part_t& q = parts[p];
    grouped = q.transa == parts[0].transa && q.transb == parts[0].transb &&
              x3_ok(q.transa, q.transb, q.M, q.N, q.K, (const float*)q.A, q.lda, (const float*)q.B, q.ldb, nullptr, 0, &none, true,
                    (char*)ws + g.off[p]);
  }
  if (!grouped) {  // each part on its own (split-K product + combine)
    for (int p = 0; p < n; ++p) {
      const pg_gemm_part_t& q = parts[p];
      const pg_gemm_epilogue_t ep{nullptr, PG_ACT_NONE, 0.f, nullptr, 0, q.rowsum};
      const int rc = gemm_f32_impl(q.transa, q.transb, q.M, q.N, q.K, 1.f, (const float*)q.A, q.lda, (const float*)q.B, q.ldb, q.beta, q.C,
                                   q.ldc, &ep, pg_gemm_f32_split_k(q.M, q.N, q.K), ws, ws_bytes, stream, false,
                                   nullptr);
      if (rc != PG_OK) return rc;
    }
    return pg::ok();
  }
  X3Group xg{};
  pg_splitk_job_t jobs[kX3MaxParts];
  int items = 0, nj = 0;
  for (int p = 0; p < n; ++p) {
    const pg_gemm_part_t& q = parts[p];
    if (q.M == 0 || q.N == 0) continue;
    float* w = (float*)((char*)ws + g.off[p]);
    X3Part& x = xg.p[nj];
    x.M = (int)q.M; x.N = (int)q.N; x.K = (int)q.K; x.kps = g.kps[p];
    x.tiles_n = (int)((q.N + kX3GroupBN - 1) / kX3GroupBN);
    x.tiles = x.tiles_n * (int)((q.M + kX3GroupBM - 1) / kX3GroupBM);
    x.first_item = items;
    x.A = (const float*)q.A; x.lda = q.lda; x.B = (const float*)q.B; x.ldb = q.ldb;
    x.ws = w;
    x.ws_rowsum = w + (int64_t)g.split[p] * q.M * q.N;
    x.rowsum = q.rowsum;
    items += x.tiles * g.split[p];
    pg_splitk_job_t& j = jobs[nj];
    j.ws = w; j.split_k = g.split[p]; j.M = q.M; j.N = q.N;
    j.alpha = 1.f; j.beta = q.beta; j.C = q.C; j.ldc = q.ldc; j.rowsum = q.rowsum;
    ++nj;
  }
  if (nj == 0) return pg::ok();
  xg.n = nj;
  xg.items = items;
  const int rc = gemm_x3_group_launch(xg, parts[0].transa != 0, parts[0].transb != 0, (hipStream_t)stream);
  const hipError_t e = hipGetLastError();
  if (rc != PG_OK || e != hipSuccess)
    return pg::set_error(rc != PG_OK ? rc : (int)e, "pg_gemm_f32_group: launch failed");
  return pg_gemm_splitk_reduce_batch(jobs, nj, stream);
}

}  // extern "C"
