// bf16-storage GEMM on the gfx950 matrix cores (v_mfma_f32_32x32x16_bf16: bf16 operands,
// f32 accumulate) with the same fused epilogues as the fp32 GEMM (gemm.hip). Serves the
// nn.Linear layers of the PLA-GNN step (code/model.py:13-17) in the bf16-storage mode of
// the engine (BASELINE configs[4]: "hidden=512 bf16"): activations and their gradients
// are stored as bf16, weights are bf16 copies of the f32 master parameters, every
// product accumulates in f32, weight gradients leave in f32.
//
// Tiling: BM x BN per 256-thread workgroup (BM, BN in {64, 128}); 2 x 2 waves, each
// owning (BM/2) x (BN/2) = TM x TN MFMA tiles of 32 x 32; K step 64 (four MFMA k-steps of
// 16). K tiles go global -> LDS by LDS-DMA (global_load_lds_dwordx4, no register round
// trip) into two images per operand; the tile for step t+1 is issued at the top of step
// t and waited for by the step's single barrier. Fragments for k-step s+1 are read while
// the MFMAs of k-step s run (across K steps too), as in the fp32 kernel.
//
// Operand images (one DMA wave-instruction fills 1 KiB of LDS lane-linearly, so every
// swizzle is applied to the DMA's per-lane SOURCE address):
//   row image, operand stored k-contiguous (A[m][k], or B stored [n][k]): [row][64 k],
//     128-B rows of 8 chunks of 8 k; chunk c of row r sits at c ^ ((r >> 1) & 7): the
//     16-lane groups of the ds_read_b128 fragment reads (16 consecutive rows, one chunk)
//     hit 16 distinct bank quads.
//   k image, operand stored row-contiguous (A stored [k][m] for dY^T X weight gradients,
//     B stored [k][n]): [64 k][ROWS], chunk c (8 rows) of k-row k at c ^ f(k), f(k) =
//     ((k >> 1) & 1) * 4 for 128-B k-rows, (k & 3) * 4 for 256-B k-rows. Fragments come
//     from ds_read_b64_tr_b16 (cdna_hip_programming.md T10): each 16-lane group reads a
//     4 k x 16 row block and every lane receives its row's 4 k-values; two reads give the
//     8 k-values of a 32x32x16 fragment. With f(k) each 32-lane half covers all 64 banks
//     once (conflict-free).
// MFMA 32x32x16 bf16 operand map (cdna_hip_programming.md §3): lane l (r = l & 31,
// h = l >> 5) holds A[row r][k = 8h + j] and B[k = 8h + j][col r], j = 0..7; C/D as the
// f32 form: row = (reg & 3) + 8 (reg >> 2) + 4h, col = r.
// Requirements (checked): 16-B aligned operands, leading dimensions and contiguous
// extents (K of a row image, M / N of a k image) multiples of 8. Rows past M / N are
// read from a clamped valid row (they only feed outputs that are never stored); a
// partial last K tile is zero-filled by ds_write.
// Output: f32 or bf16 (round to nearest even); C for beta != 0 is read in the output's
// storage type; dact (the activation output of the fused activation backward) is bf16.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "common.hpp"
#include "gemm_common.hpp"

namespace {

using namespace pg_gemm;

constexpr int BK = 64;  // bf16 k-values per K step (two-stage kernels; deep ones use 32)
#ifndef PG_BF16_WM  // wave grid of the 256 x 256 tile: 2 x 4 = eight waves, two per SIMD (measured
                    // +9 ... +25 % over 2 x 2 on the cfg5 shapes: the second wave of a SIMD issues
                    // its LDS reads and DMA while the first one runs MFMAs)
#define PG_BF16_WM 2
#endif
#ifndef PG_BF16_WN
#define PG_BF16_WN 4
#endif
#ifndef PG_BF16_DEEP
#define PG_BF16_DEEP 0
#endif
#ifndef PG_BF16_T2  // variant builds: 256 x 128 tiles, KB = 32, two workgroups per CU
#define PG_BF16_T2 0
#endif
#ifndef PG_BF16_T2_NS
#define PG_BF16_T2_NS 2
#endif

using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using bf16x4 = __attribute__((ext_vector_type(4))) __bf16;
using f32x16 = __attribute__((ext_vector_type(16))) float;
using lds_bf16x4 = __attribute__((address_space(3))) bf16x4;

// element offset (u16 units) of (row, k) in an image of KB k-values per row. Row images:
// 128-B rows (KB = 64) swizzle chunk c to c ^ ((row >> 1) & 7), 64-B rows (KB = 32) to
// c ^ ((row >> 2) & 3): either way 16 consecutive rows at one chunk hit 16 distinct bank
// quads for ds_read_b128.
template <int ROWS, bool KMAJ, int KB = BK>
__device__ __forceinline__ int img_off(int row, int k) {
  if constexpr (!KMAJ) {
    if constexpr (KB == 64) return row * KB + ((((k >> 3) ^ ((row >> 1) & 7))) << 3) + (k & 7);
    else return row * KB + ((((k >> 3) ^ ((row >> 2) & 3))) << 3) + (k & 7);
  } else {
    const int f = ROWS == 64 ? ((k >> 1) & 1) * 4 : (k & 3) * 4;
    return k * ROWS + ((((row >> 3) ^ f)) << 3) + (row & 7);
  }
}

// DMA of one ROWS x BK tile (rows [r0, r0 + ROWS) x k [k0, k0 + BK)) into an image;
// units past K (kvalid) are zero-filled by the lane that owns them.
template <int ROWS, bool KMAJ, bool FULL, int NW, int KB = BK>
__device__ __forceinline__ void dma_tile(const uint16_t* __restrict__ P, int64_t ld, int r0, int R,
                                         int k0, int kvalid, uint16_t* S, int wave, int lane) {
  constexpr int PIECES = ROWS * KB * 2 / 1024;  // 1-KiB pieces of the image
  static_assert(PIECES % NW == 0, "image pieces per wave");
#pragma unroll
  for (int j = 0; j < PIECES / NW; ++j) {
    const int piece = j * NW + wave;
    const int u = piece * 64 + lane;  // 16-B unit
    const uint16_t* src;
    bool valid;
    if constexpr (!KMAJ) {
      constexpr int UPR = KB / 8;  // units per row
      const int row = u / UPR;
      const int c = KB == 64 ? ((u & 7) ^ ((row >> 1) & 7)) : ((u & 3) ^ ((row >> 2) & 3));
      valid = 8 * c < kvalid;
      src = P + (int64_t)min(r0 + row, R - 1) * ld + k0 + 8 * c;
    } else {
      constexpr int CPR = ROWS / 8;  // chunks per k-row
      const int k = u / CPR, pos = u % CPR;
      const int f = ROWS == 64 ? ((k >> 1) & 1) * 4 : (k & 3) * 4;
      const int c = pos ^ f;
      valid = k < kvalid;
      src = P + (int64_t)(k0 + k) * ld + min(r0 + 8 * c, R - 8);
    }
    if (FULL || valid) __builtin_amdgcn_global_load_lds(src, S + piece * 512, 16, 0, 0);
    else *reinterpret_cast<uint4*>(S + u * 8) = make_uint4(0u, 0u, 0u, 0u);
  }
}

// the 8 k-values of k-step s for MFMA row/col `rc` (tile-local) of lane half h
template <int ROWS, bool KMAJ, int KB = BK>
__device__ __forceinline__ bf16x8 frag(const uint16_t* __restrict__ S, int rc, int s, int lane) {
  if constexpr (!KMAJ) {
    const int h = lane >> 5;
    return *reinterpret_cast<const bf16x8*>(S + img_off<ROWS, false, KB>(rc, 16 * s + 8 * h));
  } else {
    // ds_read_b64_tr_b16: lane 4q + p of a 16-lane group supplies the address of block row
    // q (k), columns 4p .. 4p + 3 (rows of the operand); the group's block is k-rows
    // kb .. kb + 3 x operand rows m0 .. m0 + 15, and lane i of the group receives row m0 + i.
    // rc = tile base row + (lane & 31); the group's m0 = rc - (lane & 15).
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int m = rc - (lane & 15) + 4 * p;
    const int kb = 16 * s + 8 * (g >> 1);
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (lds_bf16x4*)(S + img_off<ROWS, true, KB>(m, kb + q)));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (lds_bf16x4*)(S + img_off<ROWS, true, KB>(m, kb + 4 + q)));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

__device__ __attribute__((aligned(16))) float g_zero4f[4] = {0.f, 0.f, 0.f, 0.f};  // never written; read as a float4

__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }
__device__ __forceinline__ uint16_t f2bf(float x) {
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(x));
}

// row sums of the A tile in LDS over its BK k-values (thread t: row t % BM, k-group t / BM)
template <int BM, bool AK, int NT, int KB = BK>
__device__ __forceinline__ float img_rowsum(const uint16_t* __restrict__ As, int tid) {
  constexpr int G = NT / BM;
  const int m = tid % BM, g = tid / BM;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < KB / G; ++i) s += bf2f(As[img_off<BM, AK, KB>(m, g + i * G)]);
  return s;
}

// row sums of a k-image A tile ([KB k][BM rows], 8-row chunks swizzled per k-row): thread t
// adds chunk t % (BM / 8)'s 8 rows over the k-rows t / (BM / 8) + G i with one
// ds_read_b128 each (8x fewer LDS reads than one u16 per row and k)
template <int BM, int NT, int KB = BK>
__device__ __forceinline__ void img_rowsum8(const uint16_t* __restrict__ As, int tid, float (&rs)[8]) {
  constexpr int CPR = BM / 8, G = NT / CPR;
  static_assert(NT % CPR == 0 && KB % G == 0, "k-groups");
  const int c = tid % CPR, g = tid / CPR;
#pragma unroll
  for (int i = 0; i < KB / G; ++i) {
    const int k = g + i * G;
    const int f = BM == 64 ? ((k >> 1) & 1) * 4 : (k & 3) * 4;
    const uint4 v = *reinterpret_cast<const uint4*>(As + k * BM + ((c ^ f) << 3));
    rs[0] += bf2f(v.x & 0xFFFF); rs[1] += bf2f(v.x >> 16); rs[2] += bf2f(v.y & 0xFFFF); rs[3] += bf2f(v.y >> 16);
    rs[4] += bf2f(v.z & 0xFFFF); rs[5] += bf2f(v.z >> 16); rs[6] += bf2f(v.w & 0xFFFF); rs[7] += bf2f(v.w >> 16);
  }
}

// s_waitcnt vmcnt(N) alone (expcnt, lgkmcnt left at their no-wait maxima), gfx9 encoding
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// one output quad (row gr, columns gc .. gc + 3) with the fused epilogue, or its split-K
// partial (slab kz)
// (d2: the activation operand's quad at (gr, gc), b4: the bias quad at gc, both loaded by
// the caller ahead of the store loop)
template <int EPI, bool OBF>
__device__ __forceinline__ void store4(const float4 v, int gr, int gc, int M, int N, float alpha, float beta,
                                       void* __restrict__ Cv, int64_t ldc, const float* __restrict__ bias,
                                       const float4 b4, float slope, const uint2 d2, float* __restrict__ ws,
                                       int kz) {
  if constexpr (EPI == EPI_SPLIT) {
    *reinterpret_cast<float4*>(ws + ((int64_t)kz * M + gr) * N + gc) = v;
    return;
  } else {
    float o[4] = {alpha * v.x, alpha * v.y, alpha * v.z, alpha * v.w};
    float y[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI == EPI_DRELU || EPI == EPI_DLEAKY) {
      y[0] = bf2f(d2.x & 0xFFFF); y[1] = bf2f(d2.x >> 16); y[2] = bf2f(d2.y & 0xFFFF); y[3] = bf2f(d2.y >> 16);
    }
    if constexpr (OBF) {
      uint16_t* cp = (uint16_t*)Cv + (int64_t)gr * ldc + gc;
      if (beta != 0.f) {
        const uint2 c2 = *reinterpret_cast<const uint2*>(cp);
        o[0] = o[0] + beta * bf2f(c2.x & 0xFFFF); o[1] = o[1] + beta * bf2f(c2.x >> 16);
        o[2] = o[2] + beta * bf2f(c2.y & 0xFFFF); o[3] = o[3] + beta * bf2f(c2.y >> 16);
      }
      if (bias) {
        o[0] = o[0] + b4.x; o[1] = o[1] + b4.y; o[2] = o[2] + b4.z; o[3] = o[3] + b4.w;
      }
      uint2 w;
      w.x = (uint32_t)f2bf(epi_apply<EPI>(o[0], y[0], slope)) |
            ((uint32_t)f2bf(epi_apply<EPI>(o[1], y[1], slope)) << 16);
      w.y = (uint32_t)f2bf(epi_apply<EPI>(o[2], y[2], slope)) |
            ((uint32_t)f2bf(epi_apply<EPI>(o[3], y[3], slope)) << 16);
      *reinterpret_cast<uint2*>(cp) = w;
    } else {
      float* cp = (float*)Cv + (int64_t)gr * ldc + gc;
      if (beta != 0.f) {
        const float4 c4 = *reinterpret_cast<const float4*>(cp);
        o[0] = o[0] + beta * c4.x; o[1] = o[1] + beta * c4.y;
        o[2] = o[2] + beta * c4.z; o[3] = o[3] + beta * c4.w;
      }
      if (bias) {
        o[0] = o[0] + b4.x; o[1] = o[1] + b4.y; o[2] = o[2] + b4.z; o[3] = o[3] + b4.w;
      }
      *reinterpret_cast<float4*>(cp) =
          make_float4(epi_apply<EPI>(o[0], y[0], slope), epi_apply<EPI>(o[1], y[1], slope),
                      epi_apply<EPI>(o[2], y[2], slope), epi_apply<EPI>(o[3], y[3], slope));
    }
  }
}

// epilogue through LDS: the accumulator tile is transposed into a row-major f32 image and
// written out 4 consecutive outputs per thread (16-B f32 / 8-B bf16 stores). A tile whose
// f32 image does not fit the staging array (256 x 256) goes in PASSES row bands: in pass
// p the waves of wave row p stage their rows.
template <int BM, int BN, int WM, int WN, int EPI, bool OBF, int PASSES>
__device__ __forceinline__ void finish_tile(const f32x16 (&acc)[BM / WM / 32][BN / WN / 32], float rs,
                                            bool do_rs, float* __restrict__ lds, int tid, int m0, int n0,
                                            int M, int N, float alpha, float beta, void* __restrict__ Cv,
                                            int64_t ldc, const float* __restrict__ bias, float slope,
                                            const uint16_t* __restrict__ dact, int64_t lddact,
                                            float* __restrict__ rowsum, float* __restrict__ ws,
                                            float* __restrict__ ws_rowsum, int kz) {
  constexpr bool SPLIT = EPI == EPI_SPLIT;
  constexpr int NT = 64 * WM * WN;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int BAND = BM / PASSES;  // rows staged per pass
  static_assert(PASSES == 1 || PASSES == WM, "one pass per wave row");
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN, h = lane >> 5, l32 = lane & 31;
  if (do_rs) {
    lds[tid] = rs;
    __syncthreads();
    if (tid < BM && m0 + tid < M) {
      float t = 0.f;
      for (int g = 0; g < NT / BM; ++g) t += lds[g * BM + tid];
      if constexpr (SPLIT) ws_rowsum[(int64_t)kz * M + m0 + tid] = t;
      else rowsum[m0 + tid] = t;
    }
    __syncthreads();
  }
  // this thread's column quad is the same in every iteration: its bias is loaded once, and
  // the activation operand's quads CH at a time ahead of their use (clamped addresses, no
  // branch: inside the store loop's bounds test each load would wait out its own latency)
  constexpr int IT = BAND * BN / 4 / NT;  // output quads per thread and pass
  constexpr int CH = IT < 8 ? IT : 8;
  constexpr bool DACT = EPI == EPI_DRELU || EPI == EPI_DLEAKY;
  static_assert(NT % (BN / 4) == 0 && IT % CH == 0, "one column quad per thread");
  const int cq = (tid % (BN / 4)) * 4;
  const int gcl = min(n0 + cq, N - 4);
  float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (!SPLIT) b4 = *reinterpret_cast<const float4*>(bias ? bias + gcl : g_zero4f);
  uint2 d2[CH];
  auto prefetch = [&](int pass, int c0) {
    if constexpr (DACT) {
#pragma unroll
      for (int q = 0; q < CH; ++q) {
        const int row = ((c0 + q) * NT + tid) / (BN / 4);
        const int gr = min(m0 + pass * BAND + row, M - 1);
        d2[q] = *reinterpret_cast<const uint2*>(dact + (int64_t)gr * lddact + gcl);
      }
    } else {
#pragma unroll
      for (int q = 0; q < CH; ++q) d2[q] = make_uint2(0u, 0u);
    }
  };
#pragma unroll
  for (int pass = 0; pass < PASSES; ++pass) {
    prefetch(pass, 0);
    if (PASSES == 1 || wm == pass) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h - pass * BAND;
            lds[row * BN + wn * (BN / WN) + j * 32 + l32] = acc[i][j][r];
          }
    }
    __syncthreads();
#pragma unroll
    for (int c0 = 0; c0 < IT; c0 += CH) {
      if (c0 > 0) prefetch(pass, c0);
#pragma unroll
      for (int q = 0; q < CH; ++q) {
        const int u = (c0 + q) * NT + tid;
        const int row = u / (BN / 4), c = cq;
        const int gr = m0 + pass * BAND + row, gc = n0 + c;
        if (gr >= M || gc >= N) continue;
        const float4 v = *reinterpret_cast<const float4*>(lds + row * BN + c);
        store4<EPI, OBF>(v, gr, gc, M, N, alpha, beta, Cv, ldc, bias, b4, slope, d2[q], ws, kz);
      }
    }
    if (PASSES > 1) __syncthreads();
  }
}

// KB k-values per stage, NS LDS stages. NS = 2: the tile for step t+1 is issued at the top
// of step t and waited for by __syncthreads. NS > 2 (the 256 x 256 tiles, one workgroup per
// CU, where nothing else hides the DMA latency): NS - 1 tiles in flight; each step waits for
// the next tile only with a counted s_waitcnt vmcnt (the later tiles stay in flight) and a
// raw s_barrier (cdna_hip_programming.md "Pipelining across barriers"); a partial last K
// tile (fewer DMAs) switches the count to 0.
template <int BM, int BN, int WM, int WN, int KB, int NS>
constexpr int bf16_lds_u16() {
  constexpr int STAGE = NS * (BM * KB + BN * KB);
  constexpr int PASSES = 2 * BM * BN > STAGE ? WM : 1;
  constexpr int EPI_U16 = 2 * BM * BN / PASSES;
  return STAGE > EPI_U16 ? STAGE : EPI_U16;
}

// One output tile (tm, tn) over the K slice kz of the product: the whole workgroup's work.
template <int BM, int BN, int WM, int WN, int KB, int NS, bool TA, bool TB, int EPI, bool OBF>
__device__ __forceinline__ void bf16_tile(
    uint16_t* __restrict__ lds, int M, int N, int K, int k_per_split, int kz, int tm, int tn, float alpha,
    const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb,
    float beta, void* __restrict__ C, int64_t ldc, const float* __restrict__ bias, float slope,
    const uint16_t* __restrict__ dact, int64_t lddact, float* __restrict__ rowsum,
    float* __restrict__ ws, float* __restrict__ ws_rowsum) {
  constexpr bool AK = TA, BKM = !TB;  // k images for A stored [k][m] / B stored [k][n]
  constexpr int NW = WM * WN, NT = 64 * NW;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;  // 32 x 32 MFMA tiles per wave
  constexpr int IA = BM * KB, IB = BN * KB;  // image sizes (u16)
  constexpr int SS = KB / 16;                // MFMA k-steps per stage
  constexpr int D = (BM + BN) * KB * 2 / 1024 / NW;  // DMA instructions per tile and wave
  static_assert(SS >= 2 && SS % 2 == 0, "an even number (>= 2) of MFMA k-steps per stage");
  // one LDS array [A0 .. A(NS-1) | B0 .. B(NS-1)]; the epilogue reuses it as a row-major f32
  // image of the tile (in WM row bands when the whole tile does not fit)
  constexpr int STAGE = NS * (IA + IB);
  constexpr int PASSES = 2 * BM * BN > STAGE ? WM : 1;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN, l32 = lane & 31;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kz0 = kz * k_per_split;
  const int kz1 = min(K, kz0 + k_per_split);
  const bool do_rs = rowsum != nullptr && tn == 0;
  float rs = 0.f;
  float rs8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // k-image A: 8 rows per thread
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = kz1 > kz0 ? (kz1 - kz0 + KB - 1) / KB : 0;
  const bool tail = ((kz1 - kz0) % KB) != 0;  // the last tile is partial (fewer DMAs)
  auto issue = [&](int t, int buf) {
    const int k0 = kz0 + t * KB;
    if (kz1 - k0 >= KB) {
      dma_tile<BM, AK, true, NW, KB>(A, lda, m0, M, k0, KB, lds + buf * IA, wave, lane);
      dma_tile<BN, BKM, true, NW, KB>(B, ldb, n0, N, k0, KB, lds + NS * IA + buf * IB, wave, lane);
    } else {
      dma_tile<BM, AK, false, NW, KB>(A, lda, m0, M, k0, kz1 - k0, lds + buf * IA, wave, lane);
      dma_tile<BN, BKM, false, NW, KB>(B, ldb, n0, N, k0, kz1 - k0, lds + NS * IA + buf * IB, wave, lane);
    }
  };
  // wait until tile `need` has landed (all waves), given tiles up to `last` issued
  auto sync_tile = [&](int need, int last) {
    if constexpr (NS == 2) {
      __syncthreads();
    } else {
      const int after = last - need;  // tiles issued after `need`, still allowed in flight
      if (after <= 0 || (tail && last == nk - 1)) wait_vmcnt<0>();
      else if (after == 1) wait_vmcnt<D>();
      else wait_vmcnt<2 * D>();
      static_assert(NS <= 4, "vmcnt cases");
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS stores (zero fill)
      __builtin_amdgcn_s_barrier();
    }
  };

  if (nk > 0) {
    int issued = -1;
    for (int p = 0; p < NS - 1 && p < nk; ++p) issue(p, p), issued = p;
    sync_tile(0, issued);
    const int ra = wm * (BM / WM) + l32, rb = wn * (BN / WN) + l32;
    bf16x8 fa[2][TM], fb[2][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[0][i] = frag<BM, AK, KB>(lds, ra + i * 32, 0, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[0][j] = frag<BN, BKM, KB>(lds + NS * IA, rb + j * 32, 0, lane);
    for (int t = 0; t < nk; ++t) {
      const int cur = t % NS;
      // the next tile into the buffer every wave finished reading before the last barrier
      if (t + NS - 1 < nk) {
        issue(t + NS - 1, (t + NS - 1) % NS);
        issued = t + NS - 1;
      }
      const uint16_t* As = lds + cur * IA;
      const uint16_t* Bs = lds + NS * IA + cur * IB;
      if (do_rs) {
        if constexpr (AK) img_rowsum8<BM, NT, KB>(As, tid, rs8);
        else rs += img_rowsum<BM, AK, NT, KB>(As, tid);
      }
#pragma unroll
      for (int s = 0; s < SS; ++s) {
        const int u = s & 1;
        if (s < SS - 1) {
#pragma unroll
          for (int i = 0; i < TM; ++i) fa[u ^ 1][i] = frag<BM, AK, KB>(As, ra + i * 32, s + 1, lane);
#pragma unroll
          for (int j = 0; j < TN; ++j) fb[u ^ 1][j] = frag<BN, BKM, KB>(Bs, rb + j * 32, s + 1, lane);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[u][i], fb[u][j], acc[i][j], 0, 0, 0);
        if (s == SS - 2) {
          // tile t+1 landed and every wave is past its reads of tile t-1
          if (t + 1 < nk) sync_tile(t + 1, issued);
          else if constexpr (NS == 2) __syncthreads();
          if (t + 1 < nk) {
            const int nx = (t + 1) % NS;
#pragma unroll
            for (int i = 0; i < TM; ++i) fa[0][i] = frag<BM, AK, KB>(lds + nx * IA, ra + i * 32, 0, lane);
#pragma unroll
            for (int j = 0; j < TN; ++j)
              fb[0][j] = frag<BN, BKM, KB>(lds + NS * IA + nx * IB, rb + j * 32, 0, lane);
          }
        }
      }
    }
    if constexpr (NS > 2) wait_vmcnt<0>();
    __syncthreads();  // the epilogue reuses the staging array
  }
  if constexpr (AK) {
    // the k-groups' partial row sums combined in a fixed order
    if (do_rs) {
      constexpr int CPR = BM / 8, G = NT / CPR;
      float* red = reinterpret_cast<float*>(lds);
#pragma unroll
      for (int e = 0; e < 8; ++e) red[(tid / CPR) * BM + 8 * (tid % CPR) + e] = rs8[e];
      __syncthreads();
      if (tid < BM && m0 + tid < M) {
        float t = 0.f;
        for (int g = 0; g < G; ++g) t += red[g * BM + tid];
        if constexpr (EPI == EPI_SPLIT) ws_rowsum[(int64_t)kz * M + m0 + tid] = t;
        else rowsum[m0 + tid] = t;
      }
      __syncthreads();
    }
  }
  finish_tile<BM, BN, WM, WN, EPI, OBF, PASSES>(acc, rs, do_rs && !AK, reinterpret_cast<float*>(lds), tid, m0, n0,
                                                M, N, alpha, beta, C, ldc, bias, slope, dact, lddact, rowsum, ws,
                                                ws_rowsum, kz);
}

template <int BM, int BN, int WM, int WN, int KB, int NS, bool TA, bool TB, int EPI, bool OBF>
__global__ __launch_bounds__(64 * WM * WN) void gemm_bf16_kernel(
    int M, int N, int K, int k_per_split, int tiles_n, int tiles, float alpha,
    const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb,
    float beta, void* __restrict__ C, int64_t ldc, const float* __restrict__ bias, float slope,
    const uint16_t* __restrict__ dact, int64_t lddact, float* __restrict__ rowsum,
    float* __restrict__ ws, float* __restrict__ ws_rowsum) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[bf16_lds_u16<BM, BN, WM, WN, KB, NS>()];
  // XCD-aware tile order (as gemm.hip): blocks b, b + 8, ... share an XCD and get a
  // contiguous run of row-major tile ids, so the tiles sharing A rows meet in one L2
  const int b = blockIdx.x;
  const int q8 = tiles / 8, r8 = tiles % 8, x8 = b % 8;
  const int tile = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + b / 8;
  bf16_tile<BM, BN, WM, WN, KB, NS, TA, TB, EPI, OBF>(lds, M, N, K, k_per_split, blockIdx.z, tile / tiles_n,
                                                      tile % tiles_n, alpha, A, lda, B, ldb, beta, C, ldc, bias,
                                                      slope, dact, lddact, rowsum, ws, ws_rowsum);
}

// Grouped split-K partials (pg_gemm_bf16_group): every part's items (tiles x K slices,
// slice-major) end to end in one launch, XCD-aware over the items as gemm_x3's group.
struct BPart {
  int M, N, K, kps, tiles_n, tiles, first_item;
  const uint16_t* A;
  int64_t lda;
  const uint16_t* B;
  int64_t ldb;
  float* ws;
  float* ws_rowsum;
  float* rowsum;
};
constexpr int kBMaxParts = 16;
struct BGroup {
  BPart p[kBMaxParts];
  int n, items;
};

template <int BM, int BN, int WM, int WN, bool TA, bool TB>
__global__ __launch_bounds__(64 * WM * WN) void gemm_bf16_group_kernel(BGroup g) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[bf16_lds_u16<BM, BN, WM, WN, BK, 2>()];
  const int b = blockIdx.x;
  const int q8 = g.items / 8, r8 = g.items % 8, x8 = b % 8;
  const int item = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + b / 8;
  int k = 0;
  while (k + 1 < g.n && item >= g.p[k + 1].first_item) ++k;
  const BPart& p = g.p[k];
  const int local = item - p.first_item;
  const int kz = local / p.tiles, tile = local % p.tiles;
  bf16_tile<BM, BN, WM, WN, BK, 2, TA, TB, EPI_SPLIT, false>(lds, p.M, p.N, p.K, p.kps, kz, tile / p.tiles_n,
                                                             tile % p.tiles_n, 1.f, p.A, p.lda, p.B, p.ldb, 0.f,
                                                             nullptr, 0, nullptr, 0.f, nullptr, 0, p.rowsum, p.ws,
                                                             p.ws_rowsum);
}

// ---- 256 x 256 ping-pong kernel for A[m][k] x B[n][k]^T (both operands row images) -----
// Eight waves (2 x 4, two per SIMD), each owning 128 x 64 outputs as 8 x 4 tiles of
// v_mfma_f32_16x16x32_bf16. A K tile (64 k) is four phases; phase q covers one 64 x 32
// quadrant of every wave's block (snake order (0,0) (0,1) (1,1) (1,0), so one operand's
// fragments carry over) in two sections: R (the quadrant's fragment reads, ds_read_b128,
// plus a share of the next K tile's LDS-DMA) and M (16 MFMAs between s_setprio 1/0).
// Wave row 1 runs one barrier behind wave row 0, so on every SIMD one wave's R section
// sits beside the other's M section (cdna_hip_programming.md §5, the 256² template).
// LDS: two K-tile buffers [A 256 x 64 | B 256 x 64] (128 KiB), filled by LDS-DMA with the
// row-image swizzle. Each quarter of a buffer (the A rows or B columns of one quadrant row /
// column) is restaged two phases after its last read — the MFMAs that consumed those reads
// have finished in both wave rows by then — so a tile's pieces go out up to six phases
// before they are read; one counted vmcnt per K tile (phase 4) retires tile t + 1 while
// tile t + 2's first pieces stay in flight. (With B stored [k][n] — a k image every phase
// reads whole — this schedule measured slower than the two-phase kernel: DESIGN.md §7.)
// Raw s_barrier throughout (a __syncthreads would wait vmcnt(0) at every barrier).
using f32x4 = __attribute__((ext_vector_type(4))) float;

// end of a section. RETIRE: lgkmcnt(0) first (this wave's fragment reads and zero fills
// done), so a buffer read in this section may be restaged right after the barrier; else the
// reads stay in flight across it (the MFMAs' own waits retire them)
template <bool RETIRE>
__device__ __forceinline__ void pp_bar() {
  if constexpr (RETIRE) __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
}

template <int EPI, bool OBF>
__global__ __launch_bounds__(512) void gemm_bf16_pp_kernel(
    int M, int N, int K, int tiles_n, int tiles, float alpha, const uint16_t* __restrict__ A, int64_t lda,
    const uint16_t* __restrict__ B, int64_t ldb, float beta, void* __restrict__ C, int64_t ldc,
    const float* __restrict__ bias, float slope, const uint16_t* __restrict__ dact, int64_t lddact) {
  constexpr int IMG = 256 * 64;  // one operand's K-tile image (u16)
  constexpr int BUF = 2 * IMG;   // [A | B]
  constexpr int EPS = 260;       // f32 epilogue image row stride (floats; 16-B aligned rows)
  static_assert(64 * EPS * 4 <= 2 * BUF * 2, "epilogue band fits");
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * BUF];

  const int b = blockIdx.x;
  const int q8 = tiles / 8, r8 = tiles % 8, x8 = b % 8;
  const int tile = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + b / 8;
  const int m0 = (tile / tiles_n) * 256, n0 = (tile % tiles_n) * 256;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int l16 = lane & 15, kq = 8 * (lane >> 4);
  const int nk = (K + 63) / 64;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // LDS-DMA of one 1-KiB piece (8 rows x 64 k) of a row image; lanes past K zero-fill
  auto piece_row = [&](const uint16_t* P, int64_t ld, int r0, int R, int k0, uint16_t* img, int piece) {
    const int u = piece * 64 + lane;
    const int row = u >> 3;
    const int c = (u & 7) ^ ((row >> 1) & 7);
    const uint16_t* src = P + (int64_t)min(r0 + row, R - 1) * ld + k0 + 8 * c;
    if (K - k0 >= 64 || 8 * c < K - k0) __builtin_amdgcn_global_load_lds(src, img + piece * 512, 16, 0, 0);
    else *reinterpret_cast<uint4*>(img + u * 8) = make_uint4(0u, 0u, 0u, 0u);
  };
  // A rows of quadrant row s of both wave rows: pieces 8 s .. 8 s + 7 and 16 + the same
  auto stage_a = [&](int t, int buf, int sub) {
    uint16_t* img = lds + buf * BUF;
    piece_row(A, lda, m0, M, t * 64, img, sub * 8 + wave);
    piece_row(A, lda, m0, M, t * 64, img, 16 + sub * 8 + wave);
  };
  // B (row image) columns of quadrant column s of every wave column: rows wc 64 + 32 s ..
  auto stage_b = [&](int t, int buf, int sub) {
    uint16_t* img = lds + buf * BUF + IMG;
    const int pc = (wave >> 1) * 8 + sub * 4 + (wave & 1) * 2;
    piece_row(B, ldb, n0, N, t * 64, img, pc);
    piece_row(B, ldb, n0, N, t * 64, img, pc + 1);
  };
  bf16x8 fa[4][2], fb[2][2];
  auto read_a = [&](const uint16_t* S, int asub) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        fa[i][ks] = *reinterpret_cast<const bf16x8*>(
            S + img_off<256, false, 64>(wr * 128 + asub * 64 + i * 16 + l16, 32 * ks + kq));
  };
  auto read_b = [&](const uint16_t* S, int bsub) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        fb[j][ks] = *reinterpret_cast<const bf16x8*>(
            S + IMG + img_off<256, false, 64>(wc * 64 + bsub * 32 + j * 16 + l16, 32 * ks + kq));
  };
  auto mfma = [&](int asub, int bsub) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc[asub * 4 + i][bsub * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][ks], fb[j][ks], acc[asub * 4 + i][bsub * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  if (nk > 0) {
    // prologue: tile 0, and tile 1's pieces that steady state stages one tile early
    stage_a(0, 0, 0);
    stage_a(0, 0, 1);
    stage_b(0, 0, 0);
    stage_b(0, 0, 1);
    if (nk > 1) {
      stage_a(1, 1, 0);
      stage_b(1, 1, 1);
      wait_vmcnt<4>();
    } else {
      wait_vmcnt<0>();
    }
    pp_bar<true>();
    if (wr == 1) pp_bar<false>();  // wave row 1 runs one barrier behind
    for (int t = 0; t < nk; ++t) {
      const int c = t & 1;
      const uint16_t* S = lds + c * BUF;
      // phase 1: quadrant (0, 0); A rows of quadrant row 1 of tile t + 1 (their last reads,
      // phase 3 of tile t - 1, were consumed by MFMAs both wave rows finished before this)
      read_a(S, 0);
      read_b(S, 0);
      if (t + 1 < nk) stage_a(t + 1, c ^ 1, 1);
      pp_bar<false>();
      mfma(0, 0);
      pp_bar<false>();
      // phase 2: (0, 1); B columns of quadrant column 0 of tile t + 1 (last read in phase 4)
      read_b(S, 1);
      if (t + 1 < nk) stage_b(t + 1, c ^ 1, 0);
      pp_bar<false>();
      mfma(0, 1);
      pp_bar<false>();
      // phase 3: (1, 1); A rows of quadrant row 0 of tile t + 2 (last read in phase 1)
      read_a(S, 1);
      if (t + 2 < nk) stage_a(t + 2, c, 0);
      pp_bar<false>();
      mfma(1, 1);
      pp_bar<false>();
      // phase 4: (1, 0); B quadrant column 1 of tile t + 2 (last read in phase 2); then
      // every piece of tile t + 1 retired (only tile t + 2's pieces stay in flight) and the
      // zero fills done, before the section's barrier
      read_b(S, 0);
      if (t + 2 < nk) {
        stage_b(t + 2, c, 1);
        wait_vmcnt<4>();
      } else {
        wait_vmcnt<0>();
      }
      pp_bar<true>();
      mfma(1, 0);
      pp_bar<false>();
    }
    if (wr == 0) pp_bar<false>();
  }
  __syncthreads();  // every wave past its last fragment read: the epilogue reuses the LDS

  // epilogue in four 64-row bands (band p = wave row p / 2, A half p % 2); this thread's
  // column quad is the same in every iteration (bias loaded once, the activation operand's
  // 8 quads of a band loaded before the band is staged)
  float* img = reinterpret_cast<float*>(lds);
  constexpr bool DACT = EPI == EPI_DRELU || EPI == EPI_DLEAKY;
  const int gcl = min(n0 + (tid & 63) * 4, N - 4);
  const float4 b4 = *reinterpret_cast<const float4*>(bias ? bias + gcl : g_zero4f);
  uint2 d2[64 * 64 / 512];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
#pragma unroll
    for (int it = 0; it < 64 * 64 / 512; ++it) {
      d2[it] = make_uint2(0u, 0u);
      if constexpr (DACT) {
        const int gr = min(m0 + p * 64 + ((it * 512 + tid) >> 6), M - 1);
        d2[it] = *reinterpret_cast<const uint2*>(dact + (int64_t)gr * lddact + gcl);
      }
    }
    if (wr == (p >> 1)) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            img[(i * 16 + 4 * (lane >> 4) + e) * EPS + wc * 64 + j * 16 + l16] = acc[(p & 1) * 4 + i][j][e];
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 64 * 64 / 512; ++it) {
      const int u = it * 512 + tid;
      const int row = u >> 6, c = (u & 63) * 4;
      const int gr = m0 + p * 64 + row, gc = n0 + c;
      if (gr < M && gc < N)
        store4<EPI, OBF>(*reinterpret_cast<const float4*>(img + row * EPS + c), gr, gc, M, N, alpha, beta, C,
                         ldc, bias, b4, slope, d2[it], nullptr, 0);
    }
    __syncthreads();
  }
}

struct Args {
  int M, N, K, kps, tiles_n, tiles;
  float alpha;
  const uint16_t* A;
  int64_t lda;
  const uint16_t* B;
  int64_t ldb;
  float beta;
  void* C;
  int64_t ldc;
  const float* bias;
  float slope;
  const uint16_t* dact;
  int64_t lddact;
  float* rowsum;
  float* ws;
  float* ws_rowsum;
};

template <int BM, int BN, int WM, int WN, bool TA, bool TB, bool OBF>
int launch_epi(int epi, dim3 grid, hipStream_t st, const Args& a) {
  // KB = 64 x 2 stages. PG_BF16_DEEP=1 (build-time experiment): 256 x 256 tiles with KB = 32
  // x 4 stages and counted vmcnt instead; measured slower (fwd.cat 670 us either way, 8192^3
  // 1580 vs 1180 us): the DMA latency is not what holds this structure back.
  constexpr bool deep = PG_BF16_DEEP && BM == 256 && BN == 256;
  constexpr bool t2 = PG_BF16_T2 && BM == 256 && BN == 128;
  constexpr int KB = deep || t2 ? 32 : 64;
  constexpr int NS = deep ? 4 : t2 ? PG_BF16_T2_NS : 2;
#define PG_L(EPI_)                                                                                    \
  hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, KB, NS, TA, TB, EPI_, OBF>), grid, dim3(64 * WM * WN), 0, st, \
                     a.M, a.N, a.K, a.kps, a.tiles_n, a.tiles, a.alpha, a.A, a.lda, a.B, a.ldb,   \
                     a.beta, a.C, a.ldc, a.bias, a.slope, a.dact, a.lddact, a.rowsum, a.ws,      \
                     a.ws_rowsum)
  switch (epi) {
    case EPI_NONE: PG_L(EPI_NONE); break;
    case EPI_RELU: PG_L(EPI_RELU); break;
    case EPI_LEAKY: PG_L(EPI_LEAKY); break;
    case EPI_DRELU: PG_L(EPI_DRELU); break;
    case EPI_DLEAKY: PG_L(EPI_DLEAKY); break;
    case EPI_SPLIT:
      if constexpr (!OBF) {
        PG_L(EPI_SPLIT);
        break;
      }
      return PG_ERR_INVALID;
    default: return PG_ERR_INVALID;
  }
#undef PG_L
  return PG_OK;
}

template <int BM, int BN, int WM, int WN>
int launch_tile(bool ta, bool tb, bool obf, int epi, dim3 grid, hipStream_t st, const Args& a) {
#define PG_T(TA_, TB_)                                                      \
  return obf ? launch_epi<BM, BN, WM, WN, TA_, TB_, true>(epi, grid, st, a) \
             : launch_epi<BM, BN, WM, WN, TA_, TB_, false>(epi, grid, st, a)
  if (!ta && !tb) PG_T(false, false);
  if (!ta && tb) PG_T(false, true);
  if (ta && !tb) PG_T(true, false);
  PG_T(true, true);
#undef PG_T
}

#ifndef PG_BF16_PP
#define PG_BF16_PP 1  // 0 (variant builds): the two-phase 256 x 256 kernel for A B^T as well
#endif
int launch_pp(bool obf, int epi, hipStream_t st, const Args& a) {
#define PG_P(EPI_, OBF_)                                                                                    \
  hipLaunchKernelGGL((gemm_bf16_pp_kernel<EPI_, OBF_>), dim3((unsigned)a.tiles), dim3(512), 0, st, a.M, a.N, a.K, \
                     a.tiles_n, a.tiles, a.alpha, a.A, a.lda, a.B, a.ldb, a.beta, a.C, a.ldc, a.bias, a.slope,  \
                     a.dact, a.lddact)
#define PG_PO(EPI_) \
  if (obf) PG_P(EPI_, true); else PG_P(EPI_, false)
  switch (epi) {
    case EPI_NONE: PG_PO(EPI_NONE); break;
    case EPI_RELU: PG_PO(EPI_RELU); break;
    case EPI_LEAKY: PG_PO(EPI_LEAKY); break;
    case EPI_DRELU: PG_PO(EPI_DRELU); break;
    case EPI_DLEAKY: PG_PO(EPI_DLEAKY); break;
    default: return PG_ERR_INVALID;
  }
#undef PG_PO
#undef PG_P
  return PG_OK;
}

// Tile choice. The bf16 MFMA rate (4096 flop/clk/CU) needs ~64 flop per byte staged
// from L2 (BM BN / (BM + BN) per workgroup): 256 x 256 tiles (4 waves of 128 x 128, the
// 256 accumulators in AGPRs at one wave per SIMD; one 128-KiB workgroup per CU) wherever they still give >= 1 workgroup per CU, 128 x 128
// (two per CU) next, 128 x 64 / 64 x 64 for narrow or small products. Split products
// (weight gradients) use 256 x 256 when both sides allow it, else 64 x 64.
#ifndef PG_BF16_TILE_FORCE
#define PG_BF16_TILE_FORCE 0  // variant builds: BM * 1000 + BN forces one tile
#endif
inline void pick_tile(int64_t M, int64_t N, int64_t K, int split, int& bm, int& bn) {
  if constexpr (PG_BF16_TILE_FORCE != 0) {
    bm = PG_BF16_TILE_FORCE / 1000;
    bn = PG_BF16_TILE_FORCE % 1000;
    return;
  }
  auto tiles = [&](int tm, int tn) { return ((M + tm - 1) / tm) * ((N + tn - 1) / tn); };
  bm = bn = 64;
  if (split > 1) {
    if (M >= 256 && N >= 256) bm = bn = 256;
    return;
  }
#ifndef PG_BF16_SMALLK_TILE
#define PG_BF16_SMALLK_TILE 0  // variant builds: BM * 1000 + BN for products with K <= 128
#endif
  if constexpr (PG_BF16_SMALLK_TILE != 0) {
    if (K <= 128) {
      bm = PG_BF16_SMALLK_TILE / 1000;
      bn = PG_BF16_SMALLK_TILE % 1000;
      return;
    }
  }
  // (a short K leaves a 256 x 256 workgroup, alone on its CU, mostly in its epilogue)
  if (PG_BF16_T2 && N >= 128 && K >= 384 && tiles(256, 128) >= 512) {
    bm = 256;
    bn = 128;
  } else if (N >= 256 && K >= 384 && tiles(256, 256) >= 256) {
    bm = bn = 256;
  } else if (N > 64 && tiles(128, 128) >= 512) {
    bm = bn = 128;
  } else if (tiles(128, 64) >= 512) {
    bm = 128;
  }
}

}  // namespace

extern "C" {

int pg_gemm_bf16_split_k(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K < 2048) return 1;
  int bm, bn;
  pick_tile(M, N, K, 1, bm, bn);
  if (((M + bm - 1) / bm) * ((N + bn - 1) / bn) >= 256 * (bm == 256 ? 1 : 3)) return 1;
  pick_tile(M, N, K, 2, bm, bn);
  const int64_t tiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  // workgroups aimed at: one 256 x 256 per CU (LDS-bound), else ~5 64 x 64 per CU
  const int64_t want = bm == 256 ? 256 : 1280;
  const int64_t target = (want + tiles - 1) / tiles;
  const int64_t by_k = K / (3 * BK);
  return (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(target, by_k), 256));
}

size_t pg_gemm_bf16_workspace(int64_t M, int64_t N, int64_t K, int split_k) {
  (void)K;
  if (split_k <= 1 || M <= 0 || N <= 0) return 0;
  return (size_t)split_k * (size_t)M * (size_t)(N + 1) * 4;
}

int pg_gemm_bf16(int transa, int transb, int64_t M, int64_t N, int64_t K, float alpha,
                 const void* A, int64_t lda, const void* B, int64_t ldb, float beta, void* C,
                 int64_t ldc, int c_dtype, const pg_gemm_epilogue_t* ep, int split_k, void* ws,
                 size_t ws_bytes, pg_stream_t stream) {
  const pg_gemm_epilogue_t none{nullptr, PG_ACT_NONE, 0.f, nullptr, 0, nullptr};
  if (!ep) ep = &none;
  const int act = ep->act;
  if (M < 0 || N < 0 || K < 0 || M > INT32_MAX || N > INT32_MAX || K > INT32_MAX)
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_bf16: bad sizes");
  if (c_dtype != PG_DTYPE_F32 && c_dtype != PG_DTYPE_BF16)
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_bf16: c_dtype must be PG_DTYPE_F32 or PG_DTYPE_BF16");
  if (ldc < N || (!transa && lda < K) || (transa && lda < M) || (!transb && ldb < N) ||
      (transb && ldb < K))
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_bf16: leading dimension too small");
  if (act != PG_ACT_NONE && act != PG_ACT_RELU && act != PG_ACT_LEAKY)
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_bf16: bad act %d", act);
  if (split_k < 1) split_k = 1;
  const bool obf = c_dtype == PG_DTYPE_BF16;
  if (split_k > 1 && (obf || ep->bias || act != PG_ACT_NONE || ep->dact || (beta != 0.f && beta != 1.f)))
    return pg::set_error(PG_ERR_INVALID,
                         "pg_gemm_bf16: split_k > 1 needs an f32 C, no bias/act, beta 0|1");
  if (ep->dact && (act == PG_ACT_NONE || ep->lddact < N))
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_bf16: dact needs act relu|leaky and lddact >= N");
  if (M == 0 || N == 0) return pg::ok();
  // operand layout requirements of the DMA staging (16-B units of 8 bf16)
  const int64_t ext_a = transa ? M : K, ext_b = transb ? K : N;
  if (!al16(A) || !al16(B) || !al16(C) || lda % 8 || ldb % 8 || ext_a % 8 || ext_b % 8 || N % 4 ||
      ldc % (obf ? 4 : 4) || (ep->bias && !al16(ep->bias)) ||
      (ep->dact && (((uintptr_t)ep->dact & 7) || ep->lddact % 4)))
    return pg::set_error(PG_ERR_UNSUPPORTED,
                         "pg_gemm_bf16: operands must be 16-B aligned with leading dimensions and "
                         "contiguous extents multiples of 8, N and ldc multiples of 4");
  if (split_k > 1 && ws_bytes < pg_gemm_bf16_workspace(M, N, K, split_k))
    return pg::set_error(PG_ERR_WORKSPACE, "pg_gemm_bf16: workspace too small");
  if (split_k > 1 && !al16(ws)) return pg::set_error(PG_ERR_INVALID, "pg_gemm_bf16: workspace alignment");
  int kps = (int)K;
  if (split_k > 1) {
    kps = (int)((K + split_k - 1) / split_k);
    kps = (kps + BK - 1) / BK * BK;
    split_k = (int)((K + kps - 1) / kps);
    if (split_k < 1) split_k = 1;
  }
  const bool split = split_k > 1;
  int bm, bn;
  pick_tile(M, N, K, split_k, bm, bn);
  // a k image needs >= 8 valid rows for its clamped 16-B chunks
  if ((transa && M < 8) || (!transb && N < 8))
    return pg::set_error(PG_ERR_UNSUPPORTED, "pg_gemm_bf16: row-contiguous operand narrower than 8");
  const int tiles_n = (int)((N + bn - 1) / bn);
  const int tiles = tiles_n * (int)((M + bm - 1) / bm);
  dim3 grid((unsigned)tiles, 1, (unsigned)split_k);
  hipStream_t st = (hipStream_t)stream;
  float* wsf = split ? (float*)ws : nullptr;
  const Args a{(int)M, (int)N, (int)K, kps, tiles_n, tiles, alpha, (const uint16_t*)A, lda,
               (const uint16_t*)B, ldb, beta, C, ldc, ep->bias, ep->slope,
               (const uint16_t*)ep->dact, ep->lddact, ep->rowsum, wsf,
               split ? wsf + (int64_t)split_k * M * N : nullptr};
  const bool ta = transa != 0, tb = transb != 0;
  const int epi = split ? EPI_SPLIT
                        : ep->dact ? (act == PG_ACT_RELU ? EPI_DRELU : EPI_DLEAKY)
                                   : (act == PG_ACT_RELU ? EPI_RELU : act == PG_ACT_LEAKY ? EPI_LEAKY : EPI_NONE);
  int rc;
  if (PG_BF16_PP && bm == 256 && bn == 256 && !ta && tb && !split && !ep->rowsum) rc = launch_pp(obf, epi, st, a);
  else if (bm == 256 && bn == 256) rc = launch_tile<256, 256, PG_BF16_WM, PG_BF16_WN>(ta, tb, obf, epi, grid, st, a);
  else if (bm == 256) rc = launch_tile<256, 128, 2, 2>(ta, tb, obf, epi, grid, st, a);
  else if (bm == 128 && bn == 128) rc = launch_tile<128, 128, 2, 2>(ta, tb, obf, epi, grid, st, a);
  else if (bm == 128) rc = launch_tile<128, 64, 2, 2>(ta, tb, obf, epi, grid, st, a);
  else if (bn == 128) rc = launch_tile<64, 128, 2, 2>(ta, tb, obf, epi, grid, st, a);
  else rc = launch_tile<64, 64, 2, 2>(ta, tb, obf, epi, grid, st, a);
  if (rc != PG_OK) return pg::set_error(rc, "pg_gemm_bf16: dispatch failed");
  if (split) {
    const int64_t n = (N % 4 == 0 ? M * N / 4 : M * N) + (ep->rowsum ? M : 0);  // work units
    const int G = splitk_groups(split_k);
    const int opb = 256 / G;
    const int blocks = (int)std::min<int64_t>(8192, (n + opb - 1) / opb);
#define PG_R(G_)                                                                              \
  hipLaunchKernelGGL(splitk_reduce_kernel<G_>, dim3(blocks), dim3(256), 0, st, (const float*)wsf, \
                     split_k, (int)M, (int)N, alpha, beta, (float*)C, ldc, (const float*)a.ws_rowsum, \
                     ep->rowsum)
    if (G == 1) PG_R(1);
    else if (G == 4) PG_R(4);
    else PG_R(16);
#undef PG_R
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return pg::set_error((int)e, "pg_gemm_bf16: launch failed: %s", hipGetErrorString(e));
  return pg::ok();
}

}  // extern "C"

namespace {

// The bf16 group (pg_gemm_bf16_group): 256 x 256 tiles, one workgroup per CU. A part joins
// when its tiles waste at most 4x its area; one K-slice count for the members, the one
// (<= 64, slices >= 3 BK) whose items fill whole rounds of 256 workgroups best (the
// smallest such count within 1 %).
struct BPlan {
  bool in[kBMaxParts];
  int split[kBMaxParts];
  int kps[kBMaxParts];
  size_t off[kBMaxParts + 1];
};

inline bool bgroup_member(const pg_gemm_part_t& q) {
  const int64_t pm = (q.M + 255) / 256 * 256, pn = (q.N + 255) / 256 * 256;
  return q.M > 0 && q.N > 0 && pm * pn <= 4 * q.M * q.N;
}

inline void bgroup_plan(const pg_gemm_part_t* parts, int n, BPlan& g) {
  int64_t T = 0, kmin = INT64_MAX;
  for (int p = 0; p < n; ++p) {
    g.in[p] = bgroup_member(parts[p]);
    if (!g.in[p]) continue;
    T += ((parts[p].M + 255) / 256) * ((parts[p].N + 255) / 256);
    kmin = std::min<int64_t>(kmin, parts[p].K);
  }
  int best = 1;
  if (T > 0) {
    double bf = -1.0;
    const int smax = (int)std::max<int64_t>(1, std::min<int64_t>(64, kmin / (3 * BK)));
    for (int sc = 1; sc <= smax; ++sc) {
      const int64_t items = T * sc, rounds = (items + 255) / 256;
      const double fill = (double)items / (double)(rounds * 256);
      if (fill > bf + 0.01) bf = fill, best = sc;
    }
  }
  size_t off = 0;
  for (int p = 0; p < n; ++p) {
    const pg_gemm_part_t& q = parts[p];
    g.split[p] = 1;
    g.kps[p] = BK;
    g.off[p] = off;
    if (!g.in[p]) continue;
    int64_t sp = std::max<int64_t>(1, std::min<int64_t>(best, q.K / (3 * BK)));
    int64_t kps = (q.K + sp - 1) / sp;
    kps = std::max<int64_t>(BK, (kps + BK - 1) / BK * BK);
    sp = std::max<int64_t>(1, (q.K + kps - 1) / kps);
    g.split[p] = (int)sp;
    g.kps[p] = (int)kps;
    off += ((size_t)sp * (size_t)q.M * (size_t)(q.N + 1) * 4 + 255) / 256 * 256;
  }
  g.off[n] = off;
}

inline bool bpart_layout_ok(const pg_gemm_part_t& q) {
  const int64_t ext_a = q.transa ? q.M : q.K, ext_b = q.transb ? q.K : q.N;
  return al16(q.A) && al16(q.B) && q.lda % 8 == 0 && q.ldb % 8 == 0 && ext_a % 8 == 0 && ext_b % 8 == 0 &&
         q.N % 4 == 0 && !(q.transa && q.M < 8) && !(!q.transb && q.N < 8);
}

int bpart_alone(const pg_gemm_part_t& q, void* ws, size_t ws_bytes, pg_stream_t stream) {
  const pg_gemm_epilogue_t ep{nullptr, PG_ACT_NONE, 0.f, nullptr, 0, q.rowsum};
  return pg_gemm_bf16(q.transa, q.transb, q.M, q.N, q.K, 1.f, q.A, q.lda, q.B, q.ldb, q.beta, q.C, q.ldc,
                      PG_DTYPE_F32, &ep, pg_gemm_bf16_split_k(q.M, q.N, q.K), ws, ws_bytes, stream);
}

}  // namespace

extern "C" {

size_t pg_gemm_bf16_group_workspace(const pg_gemm_part_t* parts, int n) {
  if (n <= 0 || n > kBMaxParts || !parts) return 0;
  BPlan g;
  bgroup_plan(parts, n, g);
  size_t need = g.off[n];
  for (int p = 0; p < n; ++p) {
    const pg_gemm_part_t& q = parts[p];
    need = std::max(need, pg_gemm_bf16_workspace(q.M, q.N, q.K, pg_gemm_bf16_split_k(q.M, q.N, q.K)));
  }
  return std::max<size_t>(need, 256);
}

int pg_gemm_bf16_group(const pg_gemm_part_t* parts, int n, void* ws, size_t ws_bytes, pg_stream_t stream) {
  if (n < 0 || n > kBMaxParts || (n > 0 && !parts))
    return pg::set_error(PG_ERR_INVALID, "pg_gemm_bf16_group: 0..%d parts", kBMaxParts);
  if (n == 0) return pg::ok();
  for (int p = 0; p < n; ++p) {
    const pg_gemm_part_t& q = parts[p];
    if (q.M < 0 || q.N < 0 || q.K < 0 || q.M > INT32_MAX || q.N > INT32_MAX || q.K > INT32_MAX || q.ldc < q.N ||
        (q.transa ? q.lda < q.M : q.lda < q.K) || (q.transb ? q.ldb < q.K : q.ldb < q.N) ||
        (q.beta != 0.f && q.beta != 1.f) || (q.M > 0 && q.N > 0 && !q.C) ||
        (q.M > 0 && q.N > 0 && q.K > 0 && (!q.A || !q.B)))
      return pg::set_error(PG_ERR_INVALID, "pg_gemm_bf16_group: bad part %d", p);
  }
  if (ws_bytes < pg_gemm_bf16_group_workspace(parts, n) || !ws || !al16(ws))
    return pg::set_error(PG_ERR_WORKSPACE, "pg_gemm_bf16_group: workspace too small or misaligned");
  BPlan g;
  bgroup_plan(parts, n, g);
  int first = -1;
  bool grouped = true;
  for (int p = 0; p < n; ++p) {
    if (!g.in[p]) continue;
    if (first < 0) first = p;
    grouped = grouped && bpart_layout_ok(parts[p]) && parts[p].transa == parts[first].transa &&
              parts[p].transb == parts[first].transb;
  }
  if (first < 0 || !grouped) {
    for (int p = 0; p < n; ++p) {
      const int rc = bpart_alone(parts[p], ws, ws_bytes, stream);
      if (rc != PG_OK) return rc;
    }
    return pg::ok();
  }
  BGroup bg{};
  pg_splitk_job_t jobs[kBMaxParts];
  int items = 0, nj = 0;
  for (int p = 0; p < n; ++p) {
    if (!g.in[p]) continue;
    const pg_gemm_part_t& q = parts[p];
    float* w = (float*)((char*)ws + g.off[p]);
    BPart& x = bg.p[nj];
    x.M = (int)q.M; x.N = (int)q.N; x.K = (int)q.K; x.kps = g.kps[p];
    x.tiles_n = (int)((q.N + 255) / 256);
    x.tiles = x.tiles_n * (int)((q.M + 255) / 256);
    x.first_item = items;
    x.A = (const uint16_t*)q.A; x.lda = q.lda; x.B = (const uint16_t*)q.B; x.ldb = q.ldb;
    x.ws = w;
    x.ws_rowsum = w + (int64_t)g.split[p] * q.M * q.N;
    x.rowsum = q.rowsum;
    items += x.tiles * g.split[p];
    pg_splitk_job_t& j = jobs[nj];
    j.ws = w; j.split_k = g.split[p]; j.M = q.M; j.N = q.N;
    j.alpha = 1.f; j.beta = q.beta; j.C = q.C; j.ldc = q.ldc; j.rowsum = q.rowsum;
    ++nj;
  }
  bg.n = nj;
  bg.items = items;
  const bool ta = parts[first].transa != 0, tb = parts[first].transb != 0;
  const dim3 grid((unsigned)items), block(64 * PG_BF16_WM * PG_BF16_WN);
  hipStream_t st = (hipStream_t)stream;
#define PG_G(TA_, TB_) \
  hipLaunchKernelGGL((gemm_bf16_group_kernel<256, 256, PG_BF16_WM, PG_BF16_WN, TA_, TB_>), grid, block, 0, st, bg)
  if (ta && !tb) PG_G(true, false);
  else if (!ta && !tb) PG_G(false, false);
  else if (!ta && tb) PG_G(false, true);
  else PG_G(true, true);
#undef PG_G
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return pg::set_error((int)e, "pg_gemm_bf16_group: launch failed: %s", hipGetErrorString(e));
  int rc = pg_gemm_splitk_reduce_batch(jobs, nj, stream);
  // the parts a 256 x 256 tile would waste, after the combine on the same stream (so they
  // may reuse the workspace)
  for (int p = 0; p < n && rc == PG_OK; ++p)
    if (!g.in[p]) rc = bpart_alone(parts[p], ws, ws_bytes, stream);
  return rc;
}

}  // extern "C"
