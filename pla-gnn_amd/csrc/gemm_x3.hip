// fp32 GEMM on the bf16 matrix cores: every f32 operand element is split into three bf16
// pieces, a = a_h + a_m + a_l (each the round-to-nearest bf16 of what the previous pieces
// leave), and C = sum over the six products A_h B_h + A_h B_m + A_m B_h + A_h B_l +
// A_l B_h + A_m B_m of v_mfma_f32_32x32x16_bf16 (bf16 x bf16 products are exact in f32,
// accumulation in f32). The three dropped products (A_m B_l, A_l B_m, A_l B_l) and the
// split's remainder are below 2^-24 of |a b| each: per product the result is as accurate
// as an f32 multiply; the sums run in f32 as in the exact kernel (gemm.hip), in another
// order. Six bf16 MFMAs (6 x 32 cycles per 32x32x16 block) replace eight f32 MFMAs
// (8 x 64 cycles): 2.67x the f32 MFMA peak is the ceiling (419 TF/s f32-equivalent).
// Serves the same nn.Linear GEMMs as gemm.hip (code/model.py:13-17, forward and backward)
// with the same epilogues and split-K partials; used where the operands allow 16-B loads.
//
// Tiling: BM x BN per 256-thread workgroup, 2 x 2 waves of (BM/2) x (BN/2) = TM x TN MFMA
// tiles of 32 x 32, one MFMA k-step (16 k) per K step. K tiles go global -> registers
// (float4 per thread and unit, issued one K step ahead; two for tiles of <= 128 x 64, the
// loads unconditional so the waits are counted), are split in registers and
// stored as three bf16 images per operand (ds_write_b64 per piece) into the other half of
// a double-buffered LDS array: one barrier per K step.
// Images (u16 units), per piece:
//   row image, operand stored k-contiguous (A[m][k], B stored [n][k]): [row][16 k], 32-B
//     rows of two 8-k chunks; chunk c of row r at c ^ ((r >> 3) & 1), so the 16-lane groups
//     of the ds_read_b128 fragment reads hit 16 distinct bank quads.
//   k image, operand stored row-contiguous (A stored [k][m], B stored [k][n]): [16 k][ROWS],
//     chunk c (8 rows) of k-row k at c ^ f(k) (gemm_bf16.hip's layout), read by
//     ds_read_b64_tr_b16.
// Requirements (the caller checks): 16-B aligned operands, leading dimensions and the
// contiguous extents (K of a row image, M / N of a k image) multiples of 4.
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "gemm_common.hpp"
#include "x3_split.hpp"

namespace {

using namespace pg_gemm;
using pg_x3::split4;

constexpr int KS = 16;  // k per K step
constexpr int NT = 256;

using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using bf16x4 = __attribute__((ext_vector_type(4))) __bf16;
using f32x16 = __attribute__((ext_vector_type(16))) float;
using lds_bf16x4 = __attribute__((address_space(3))) bf16x4;

template <int ROWS, bool KMAJ>
__device__ __forceinline__ int img_off(int row, int k) {
  if constexpr (!KMAJ) {
    return row * KS + ((((k >> 3) ^ ((row >> 3) & 1))) << 3) + (k & 7);
  } else {
    const int f = ROWS == 64 ? ((k >> 1) & 1) * 4 : (k & 3) * 4;
    return k * ROWS + ((((row >> 3) ^ f)) << 3) + (row & 7);
  }
}

// the 8 k-values of MFMA row/col `rc` (tile-local) for lane half h = lane >> 5
template <int ROWS, bool KMAJ>
__device__ __forceinline__ bf16x8 frag(const uint16_t* __restrict__ S, int rc, int lane) {
  if constexpr (!KMAJ) {
    return *reinterpret_cast<const bf16x8*>(S + img_off<ROWS, false>(rc, 8 * (lane >> 5)));
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int m = rc - (lane & 15) + 4 * p;
    const int kb = 8 * (g >> 1);
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(S + img_off<ROWS, true>(m, kb + q)));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(S + img_off<ROWS, true>(m, kb + 4 + q)));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// One operand's K tile: ROWS x KS, float4 units; row image unit = (row, 4 k), k image unit
// = (k, 4 rows).
__device__ __attribute__((aligned(16))) float g_zero4[4] = {0.f, 0.f, 0.f, 0.f};  // never written; read as a float4

#ifndef PG_X3_BUFLOAD
#define PG_X3_BUFLOAD 1  // K tiles by buffer loads with per-unit 32-bit offsets (0: 64-bit addresses)
#endif

// One operand's buffer descriptor (wave-uniform: built from readfirstlane'd inputs, so the
// compiler keeps it in SGPRs) covering `bytes` from P; every byte offset of the operand is
// below 2^32 (x3_ok checks the extent on the host).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t x3_rsrc(const float* P, uint32_t bytes) { return pg_x3::rsrc(P, bytes); }
constexpr uint32_t kX3Oob = 0xFFFFFFF0u;  // a byte offset past every descriptor's range: reads 0

template <int ROWS, bool KMAJ, int NTH = NT>
struct Stage {
  static constexpr int UNITS = ROWS * KS / 4;
  static constexpr int PER = UNITS / NTH;
  static_assert(PER >= 1 && UNITS % NTH == 0, "units per thread");
  float4 v[PER];

  __device__ __forceinline__ static void unit_pos(int q, int& row, int& k) {
    if constexpr (!KMAJ) {
      row = q >> 2;
      k = (q & 3) << 2;
    } else {
      k = q / (ROWS / 4);
      row = (q % (ROWS / 4)) << 2;
    }
  }
#if PG_X3_BUFLOAD
  template <typename Addr>
  __device__ __forceinline__ void load(const Addr& a, __amdgpu_buffer_rsrc_t rs, uint32_t step_bytes, int kt, int kz1) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const uint32_t o = kt + a.kq(i) < kz1 ? a.off(i) + step_bytes : kX3Oob;
      v[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o, 0, 0));
    }
  }
  // K-concatenated operand: k < kcat from the first, the rest from the second (kcat a
  // multiple of 4, so no unit straddles it; a K step may). Each unit loads through both
  // descriptors, the one it does not use at an out-of-range offset (zeros), and ORs the
  // bits: exact.
  template <typename Addr>
  __device__ __forceinline__ void load_cat(const Addr& a1, const Addr& a2, __amdgpu_buffer_rsrc_t rs1,
                                           __amdgpu_buffer_rsrc_t rs2, uint32_t step1, uint32_t step2,
                                           int kcat, int kt, int kz1) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int k = kt + a1.kq(i);
      const uint32_t o1 = k < kcat && k < kz1 ? a1.off(i) + step1 : kX3Oob;
      const uint32_t o2 = k >= kcat && k < kz1 ? a2.off(i) + step2 : kX3Oob;
      const uint4 x = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs1, (int)o1, 0, 0));
      const uint4 y = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs2, (int)o2, 0, 0));
      v[i] = __builtin_bit_cast(float4, make_uint4(x.x | y.x, x.y | y.y, x.z | y.z, x.w | y.w));
    }
  }
#else
  // rows past R read a clamped valid row (never stored); k past kz1 read as 0
  __device__ __forceinline__ void load(const float* __restrict__ P, int64_t ld, int r0, int R, int k0,
                                       int kz1, int tid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int row, k;
      unit_pos(tid + i * NTH, row, k);
      const int gk = k0 + k;
      // straight-line: a unit past kz1 reads a 16-B zero word in global memory instead of
      // being zeroed behind a branch, so every load is unconditional and the compiler
      // counts the waits
      const float* p = !KMAJ ? P + (int64_t)min(r0 + row, R - 1) * ld + gk
                             : P + (int64_t)gk * ld + min(r0 + row, R - 4);
      v[i] = *reinterpret_cast<const float4*>(gk < kz1 ? p : g_zero4);
    }
  }
#endif
  // split and store the three pieces (images of IMG u16 each, consecutive)
  template <int IMG>
  __device__ __forceinline__ void store(uint16_t* __restrict__ S, int tid) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int row, k;
      unit_pos(tid + i * NTH, row, k);
      uint2 pc[3];
      split4(v[i], pc);
      const int off = img_off<ROWS, KMAJ>(row, k);
#pragma unroll
      for (int piece = 0; piece < 3; ++piece) *reinterpret_cast<uint2*>(S + piece * IMG + off) = pc[piece];
    }
  }
  // running row sums (float64) of an A tile: row image -> one row per unit, k image -> the
  // same 4 rows for every unit of this thread
  static constexpr int RSN = KMAJ ? 4 : PER;
  __device__ __forceinline__ void rowsum(double (&rs)[RSN]) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if constexpr (!KMAJ) {
        rs[i] += ((double)v[i].x + (double)v[i].y) + ((double)v[i].z + (double)v[i].w);
      } else {
        rs[0] += v[i].x; rs[1] += v[i].y; rs[2] += v[i].z; rs[3] += v[i].w;
      }
    }
  }
};

#if PG_X3_BUFLOAD
// A K tile's addressing, set up once per tile (shared by the register slots of a deeper
// pipeline): the byte offset of each unit at the slice's first k (rows past R clamped to a
// valid row, never stored) and its k within a K step. A step then costs one add, one
// compare and one select per unit (a unit at or past kz1 reads through an out-of-range
// offset: zeros), no 64-bit address arithmetic.
template <int ROWS, bool KMAJ, int NTH = NT>
struct StageAddr {
  static constexpr int PER = Stage<ROWS, KMAJ, NTH>::PER;
  // k image: unit i of a thread sits KQS k-rows below unit 0 in the same 4 rows, so one
  // offset and a wave-uniform stride describe them all; row image: every unit its own row
  // (clamped), one k
  static constexpr int KQS = KMAJ ? NTH / (ROWS / 4) : 0;
  static constexpr int NOFF = KMAJ ? 1 : PER;
  uint32_t off_[NOFF];
  uint32_t ustride;  // KMAJ: bytes between consecutive units (wave-uniform)
  int kq0;
  __device__ __forceinline__ void setup(int64_t ld, int r0, int R, int k0, int tid) {
    int row, k;
    Stage<ROWS, KMAJ, NTH>::unit_pos(tid, row, k);
    kq0 = k;
    if constexpr (KMAJ) {
      off_[0] = ((uint32_t)(k0 + k) * (uint32_t)ld + (uint32_t)min(r0 + row, R - 4)) * 4u;
      ustride = (uint32_t)KQS * (uint32_t)ld * 4u;
    } else {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        Stage<ROWS, KMAJ, NTH>::unit_pos(tid + i * NTH, row, k);
        off_[i] = ((uint32_t)min(r0 + row, R - 1) * (uint32_t)ld + (uint32_t)(k0 + k)) * 4u;
      }
      ustride = 0;
    }
  }
  __device__ __forceinline__ uint32_t off(int i) const {
    if constexpr (KMAJ) return off_[0] + (uint32_t)i * ustride;
    else return off_[i];
  }
  __device__ __forceinline__ int kq(int i) const { return kq0 + i * KQS; }
};
#endif

// The accumulator tile leaves through LDS in PASSES row bands (16-B stores), with the
// epilogue (alpha, beta C, bias, act / act', or the split-K partial slab).
template <int BM, int BN, int EPI, int PASSES, int NTH = NT>
__device__ __forceinline__ void x3_store(const f32x16 (&acc)[BM / 64][BN / (32 * (NTH / 128))], float* __restrict__ img, int tid,
                                         int m0, int n0, int M, int N, int kz, float alpha, float beta,
                                         float* __restrict__ C, int64_t ldc, const float* __restrict__ bias,
                                         float slope, const float* __restrict__ dact, int64_t lddact,
                                         float* __restrict__ ws) {
  constexpr bool SPLIT = EPI == EPI_SPLIT;
  constexpr int WN = NTH / 128;  // waves along N (2 x WN waves)
  constexpr int TM = BM / 64, TN = BN / (32 * WN);
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN, h = lane >> 5, l32 = lane & 31;
  constexpr int BAND = BM / PASSES;
  constexpr int IT = BAND * BN / 4 / NTH;  // output quads per thread and pass
  constexpr int CH = IT < 8 ? IT : 8;     // quads whose operand loads are in flight together
  constexpr bool DACT = EPI == EPI_DRELU || EPI == EPI_DLEAKY;
  static_assert(NTH % (BN / 4) == 0 && IT % CH == 0, "one column quad per thread");
  // this thread's column quad is the same in every iteration: its bias is loaded once, and
  // the activation operand's quads are loaded CH at a time ahead of their use (clamped
  // addresses, no branch: behind the store loop's bounds test the loads would run one at a
  // time, each waiting out its latency)
  const int cq = (tid % (BN / 4)) * 4;
  const int gcl = min(n0 + cq, N - 4);
  float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (!SPLIT) b4 = *reinterpret_cast<const float4*>(bias ? bias + gcl : g_zero4);
  float4 y4[CH];
  auto prefetch = [&](int pass, int c0) {
    if constexpr (DACT) {
#pragma unroll
      for (int q = 0; q < CH; ++q) {
        const int row = ((c0 + q) * NTH + tid) / (BN / 4);
        const int gr = min(m0 + pass * BAND + row, M - 1);
        y4[q] = *reinterpret_cast<const float4*>(dact + (int64_t)gr * lddact + gcl);
      }
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
            const int row = wm * (BM / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h - pass * BAND;
            img[row * BN + wn * (BN / WN) + j * 32 + l32] = acc[i][j][r];
          }
    }
    __syncthreads();
#pragma unroll
    for (int c0 = 0; c0 < IT; c0 += CH) {
      if (c0 > 0) prefetch(pass, c0);
#pragma unroll
      for (int q = 0; q < CH; ++q) {
        const int u = (c0 + q) * NTH + tid;
        const int row = u / (BN / 4), c = cq;
        const int gr = m0 + pass * BAND + row, gc = n0 + c;
        if (gr >= M || gc >= N) continue;
        const float4 v = *reinterpret_cast<const float4*>(img + row * BN + c);
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
          if (bias) {  // (no add without a bias: -0 stays -0)
            o[0] = o[0] + b4.x; o[1] = o[1] + b4.y; o[2] = o[2] + b4.z; o[3] = o[3] + b4.w;
          }
          float y[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (DACT) {
            y[0] = y4[q].x; y[1] = y4[q].y; y[2] = y4[q].z; y[3] = y4[q].w;
          }
          *reinterpret_cast<float4*>(cp) =
              make_float4(epi_apply<EPI>(o[0], y[0], slope), epi_apply<EPI>(o[1], y[1], slope),
                          epi_apply<EPI>(o[2], y[2], slope), epi_apply<EPI>(o[3], y[3], slope));
        }
      }
    }
    if (PASSES > 1) __syncthreads();
  }
}


#ifndef PG_X3_STAMP
#define PG_X3_STAMP 0  // probe builds only: per-step shader-clock stamps of wave 0 of blocks 0..63
#endif
#if PG_X3_STAMP
__device__ unsigned long long pg_x3_stamp[64][66][4];
#define X3_STAMP(t, q)                                                                                \
  do {                                                                                                \
    if (tid == 0 && blockIdx.x < 64 && (t) < 66) pg_x3_stamp[blockIdx.x][(t)][(q)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define X3_STAMP(t, q) \
  do {                 \
  } while (0)
#endif

// Tiles of <= 128 x 64 keep two K tiles in flight in registers (DEPTH 2), capped at 128
// registers per lane so four workgroups still fit a CU (their LDS allows four).
template <int BM, int BN>
constexpr int x3_depth() { return BM * BN <= 128 * 64 ? 2 : 1; }

// Waves per SIMD the register allocation must allow. 128 x 128 tiles (48 KB of LDS, three
// per CU by LDS): left unbounded the compiler took 152 VGPRs + 64 AGPRs (216 allocated:
// two waves per SIMD, so two workgroups per CU); bounded to three it fits 145-153 VGPRs,
// no AGPRs, no spills.
#ifndef PG_X3_WAVES_BIG
#define PG_X3_WAVES_BIG 3
#endif
template <int BM, int BN>
constexpr int x3_waves() {
  return x3_depth<BM, BN>() == 2 ? 4 : BM * BN <= 128 * 128 ? PG_X3_WAVES_BIG : 2;
}

template <int BM, int BN>
constexpr int x3_lds_u16() {
  constexpr int STAGE_U16 = 2 * 3 * (BM * KS + BN * KS);  // two buffers of [A_h A_m A_l | B_h B_m B_l]
  constexpr int PASSES = 2 * BM * BN > STAGE_U16 ? 2 : 1;
  constexpr int EPI_U16 = 2 * BM * BN / PASSES;
  return STAGE_U16 > EPI_U16 ? STAGE_U16 : EPI_U16;
}

// One output tile (tm, tn) over the K slice kz of the product: the whole workgroup's work.
// KCAT: both operands are concatenations along K, [A | A2] and [B ; B2] (op(B)), split at
// k = cat.kcat (a multiple of 4; no split-K): the drop-in layer's [H | M] [Wself | Wneigh]^T
// and [dY | dP] [Wself ; Wpool] without building the concatenations.
struct X3Cat {
  const float* A2;
  int64_t lda2;
  const float* B2;
  int64_t ldb2;
  int kcat;
};
template <int BM, int BN, bool TA, bool TB, int EPI, bool KCAT = false, int NTH = NT>
__device__ __forceinline__ void x3_tile(
    uint16_t* __restrict__ lds, int M, int N, int K, int k_per_split, int kz, int tm, int tn, float alpha,
    const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb, float beta,
    float* __restrict__ C, int64_t ldc, const float* __restrict__ bias, float slope,
    const float* __restrict__ dact, int64_t lddact, float* __restrict__ rowsum,
    float* __restrict__ ws, float* __restrict__ ws_rowsum, X3Cat cat = {}) {
  constexpr bool AK = TA, BKM = !TB;
  constexpr bool SPLIT = EPI == EPI_SPLIT;
  constexpr int WN = NTH / 128;  // waves along N (2 x WN waves)
  constexpr int TM = BM / 64, TN = BN / (32 * WN);
  constexpr int IA = BM * KS, IB = BN * KS;  // one piece's image (u16)
  constexpr int BUF = 3 * (IA + IB);         // one buffer: [A_h A_m A_l | B_h B_m B_l]
  constexpr int STAGE_U16 = 2 * BUF;
  constexpr int PASSES = 2 * BM * BN > STAGE_U16 ? 2 : 1;  // f32 epilogue image in row bands
  static_assert(x3_lds_u16<BM, BN>() * 2 >= NTH * 4 * 8, "row-sum scratch");

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN, l32 = lane & 31;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kz0 = kz * k_per_split;
  const int kz1 = min(K, kz0 + k_per_split);
  const bool do_rs = rowsum != nullptr && tn == 0;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  Stage<BM, AK, NTH> sa;
  Stage<BN, BKM, NTH> sb;
  static_assert(!KCAT || PG_X3_BUFLOAD, "K-concatenated operands need the buffer-load addressing");
#if PG_X3_BUFLOAD
  // operand extents in bytes (row image: R rows of ld; k image: K rows of ld); with KCAT the
  // first operands end at k = kcat (the host checked that extent, not K's)
  const int K1 = KCAT ? cat.kcat : K;
  const uint32_t a_bytes = (uint32_t)(AK ? ((int64_t)(K1 - 1) * lda + M) * 4 : ((int64_t)(M - 1) * lda + K1) * 4);
  const uint32_t b_bytes = (uint32_t)(BKM ? ((int64_t)(K1 - 1) * ldb + N) * 4 : ((int64_t)(N - 1) * ldb + K1) * 4);
  const __amdgpu_buffer_rsrc_t rsa = x3_rsrc(A, a_bytes), rsb = x3_rsrc(B, b_bytes);
  const uint32_t a_kstride = AK ? (uint32_t)lda * 4u : 4u, b_kstride = BKM ? (uint32_t)ldb * 4u : 4u;
  StageAddr<BM, AK, NTH> aa;
  StageAddr<BN, BKM, NTH> ab;
  aa.setup(lda, m0, M, kz0, tid);
  ab.setup(ldb, n0, N, kz0, tid);
  // KCAT: the second operands' addressing (their own k starts at 0 where the first ends)
  StageAddr<BM, AK, NTH> aa2;
  StageAddr<BN, BKM, NTH> ab2;
  __amdgpu_buffer_rsrc_t rsa2 = rsa, rsb2 = rsb;
  uint32_t a2_kstride = 0, b2_kstride = 0;
  if constexpr (KCAT) {
    const int K2 = K - cat.kcat;
    const uint32_t a2_bytes =
        (uint32_t)(AK ? ((int64_t)(K2 - 1) * cat.lda2 + M) * 4 : ((int64_t)(M - 1) * cat.lda2 + K2) * 4);
    const uint32_t b2_bytes =
        (uint32_t)(BKM ? ((int64_t)(K2 - 1) * cat.ldb2 + N) * 4 : ((int64_t)(N - 1) * cat.ldb2 + K2) * 4);
    rsa2 = x3_rsrc(cat.A2, a2_bytes);
    rsb2 = x3_rsrc(cat.B2, b2_bytes);
    a2_kstride = AK ? (uint32_t)cat.lda2 * 4u : 4u;
    b2_kstride = BKM ? (uint32_t)cat.ldb2 * 4u : 4u;
    aa2.setup(cat.lda2, m0, M, 0, tid);
    ab2.setup(cat.ldb2, n0, N, 0, tid);
  }
  auto load_a = [&](Stage<BM, AK, NTH>& st, int kt) {
    if constexpr (KCAT) {
      st.load_cat(aa, aa2, rsa, rsa2, (uint32_t)(kt - kz0) * a_kstride, (uint32_t)(kt - cat.kcat) * a2_kstride,
                  cat.kcat, kt, kz1);
    } else {
      st.load(aa, rsa, (uint32_t)(kt - kz0) * a_kstride, kt, kz1);
    }
  };
  auto load_b = [&](Stage<BN, BKM, NTH>& st, int kt) {
    if constexpr (KCAT) {
      st.load_cat(ab, ab2, rsb, rsb2, (uint32_t)(kt - kz0) * b_kstride, (uint32_t)(kt - cat.kcat) * b2_kstride,
                  cat.kcat, kt, kz1);
    } else {
      st.load(ab, rsb, (uint32_t)(kt - kz0) * b_kstride, kt, kz1);
    }
  };
#else
  auto load_a = [&](Stage<BM, AK, NTH>& st, int kt) { st.load(A, lda, m0, M, kt, kz1, tid); };
  auto load_b = [&](Stage<BN, BKM, NTH>& st, int kt) { st.load(B, ldb, n0, N, kt, kz1, tid); };
#endif
  double rs[Stage<BM, AK, NTH>::RSN];
#pragma unroll
  for (int i = 0; i < Stage<BM, AK, NTH>::RSN; ++i) rs[i] = 0.0;

  const int nk = kz1 > kz0 ? (kz1 - kz0 + KS - 1) / KS : 0;
  const int ra = wm * (BM / 2) + l32, rb = wn * (BN / WN) + l32;
  auto mfmas = [&](const uint16_t* As, const uint16_t* Bs) {
    bf16x8 fa[3][TM], fb[3][TN];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[p][i] = frag<BM, AK>(As + p * IA, ra + i * 32, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[p][j] = frag<BN, BKM>(Bs + p * IB, rb + j * 32, lane);
    }
    // small terms first: (h,l) (l,h) (m,m) (h,m) (m,h) (h,h)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[2][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2][i], fb[0][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fb[1][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[1][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fb[0][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[0][j], acc[i][j], 0, 0, 0);
      }
  };
  if (x3_depth<BM, BN>() == 2 && nk > 0) {
    // tiles two K steps ahead in registers (two stage slots, the loop unrolled by two so
    // the slots are static): step t loads tile t + 2 (clamped to the last tile, so the
    // loads are unconditional) into the slot tile t left, and stores tile t + 1. Measured
    // on the cfg2 step: GEMM 916 -> 902 us (the split waits for a tile issued a step
    // earlier instead of during the same step's MFMAs)
    Stage<BM, AK, NTH> sa2;
    Stage<BN, BKM, NTH> sb2;
    load_a(sa, kz0);
    load_b(sb, kz0);
    const int k1c = kz0 + min(1, nk - 1) * KS;
    load_a(sa2, k1c);
    load_b(sb2, k1c);
    if (do_rs) sa.rowsum(rs);
    sa.template store<IA>(lds, tid);
    sb.template store<IB>(lds + 3 * IA, tid);
    __syncthreads();
    // loads sit outside every branch (only MFMAs and stores are conditional), so the
    // compiler's wait counts stay exact across the loop
    auto kstep = [&](int t, Stage<BM, AK, NTH>& la, Stage<BN, BKM, NTH>& lb, Stage<BM, AK, NTH>& na, Stage<BN, BKM, NTH>& nb) {
      const int cur = t & 1;
      const int kl = kz0 + min(t + 2, nk - 1) * KS;
      load_a(la, kl);
      load_b(lb, kl);
      if (t < nk) {
        const uint16_t* As = lds + cur * BUF;
        mfmas(As, As + 3 * IA);
      }
      if (t + 1 < nk) {
        if (do_rs) na.rowsum(rs);
        uint16_t* nx = lds + (cur ^ 1) * BUF;
        na.template store<IA>(nx, tid);
        nb.template store<IB>(nx + 3 * IA, tid);
      }
      __syncthreads();
    };
    for (int t = 0; t < nk; t += 2) {
      kstep(t, sa, sb, sa2, sb2);
      kstep(t + 1, sa2, sb2, sa, sb);
    }
  } else if (nk > 0) {
    X3_STAMP(0, 0);
    load_a(sa, kz0);
    load_b(sb, kz0);
    if (do_rs) sa.rowsum(rs);
    sa.template store<IA>(lds, tid);
    sb.template store<IB>(lds + 3 * IA, tid);
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
      const int cur = t & 1;
      const bool more = t + 1 < nk;
      X3_STAMP(t + 1, 0);
      if (more) {
        load_a(sa, kz0 + (t + 1) * KS);
        load_b(sb, kz0 + (t + 1) * KS);
      }
      const uint16_t* As = lds + cur * BUF;
      mfmas(As, As + 3 * IA);
      X3_STAMP(t + 1, 1);
#if PG_X3_STAMP
      __builtin_amdgcn_s_waitcnt((0 & 15) | (7 << 4) | (15 << 8));  // vmcnt(0): the next tile's loads
      X3_STAMP(t + 1, 3);
#endif
      if (more) {
        if (do_rs) sa.rowsum(rs);
        uint16_t* nx = lds + (cur ^ 1) * BUF;
        sa.template store<IA>(nx, tid);
        sb.template store<IB>(nx + 3 * IA, tid);
      }
      X3_STAMP(t + 1, 2);
      __syncthreads();  // the next buffer is complete; every wave is past its reads of this one
    }
  }

  // row sums of op(A) (float64 partials per thread, combined in a fixed order)
  if (do_rs) {
    double* red = reinterpret_cast<double*>(lds);
    if constexpr (!AK) {
      // row image: unit i of thread tid is row (tid + i NTH) / 4, k-quarter tid % 4
#pragma unroll
      for (int i = 0; i < Stage<BM, AK, NTH>::RSN; ++i) red[tid + i * NTH] = rs[i];  // = 4 row + k-quarter
      __syncthreads();
      if (tid < BM && m0 + tid < M) {
        const double t = (red[4 * tid] + red[4 * tid + 1]) + (red[4 * tid + 2] + red[4 * tid + 3]);
        if constexpr (SPLIT) ws_rowsum[(int64_t)kz * M + m0 + tid] = (float)t;
        else rowsum[m0 + tid] = (float)t;
      }
    } else {
      // k image: thread tid holds rows 4 (tid % (BM / 4)) .. + 3 for the k-rows tid / (BM / 4)
      constexpr int G = NTH / (BM / 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) red[(tid / (BM / 4)) * BM + 4 * (tid % (BM / 4)) + e] = rs[e];
      __syncthreads();
      if (tid < BM && m0 + tid < M) {
        double t = 0.0;
        for (int g = 0; g < G; ++g) t += red[g * BM + tid];
        if constexpr (SPLIT) ws_rowsum[(int64_t)kz * M + m0 + tid] = (float)t;
        else rowsum[m0 + tid] = (float)t;
      }
    }
    __syncthreads();
  }

  X3_STAMP(65, 0);
  x3_store<BM, BN, EPI, PASSES, NTH>(acc, reinterpret_cast<float*>(lds), tid, m0, n0, M, N, kz, alpha, beta, C, ldc,
                                bias, slope, dact, lddact, ws);
  X3_STAMP(65, 1);
}

// XCD-aware order over `items` (slice-major within a product): workgroup b runs on XCD
// b % 8, which takes one contiguous range of the items, so the workgroups sharing a K
// slice's operand rows share that XCD's L2 (as gemm.hip's DMA kernel)
__device__ __forceinline__ int x3_item(int items) {
  const int b = blockIdx.x;
  const int q8 = items / 8, r8 = items % 8, x8 = b % 8;
  return (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + b / 8;
}

template <int BM, int BN, bool TA, bool TB, int EPI>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(x3_waves<BM, BN>())))
void gemm_x3_kernel(
    int M, int N, int K, int k_per_split, int tiles_n, int tiles, float alpha,
    const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb, float beta,
    float* __restrict__ C, int64_t ldc, const float* __restrict__ bias, float slope,
    const float* __restrict__ dact, int64_t lddact, float* __restrict__ rowsum,
    float* __restrict__ ws, float* __restrict__ ws_rowsum, int n_split) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[x3_lds_u16<BM, BN>()];
  const int item = x3_item(tiles * n_split);
  const int kz = item / tiles, tile = item % tiles;
  x3_tile<BM, BN, TA, TB, EPI>(lds, M, N, K, k_per_split, kz, tile / tiles_n, tile % tiles_n, alpha, A, lda, B,
                               ldb, beta, C, ldc, bias, slope, dact, lddact, rowsum, ws, ws_rowsum);
}

// K-concatenated operands (X3Cat), no split-K: the drop-in layers' products
template <int BM, int BN, bool TA, bool TB, int EPI>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(x3_waves<BM, BN>())))
void gemm_x3_cat_kernel(
    int M, int N, int K, int tiles_n, int tiles, float alpha,
    const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb, float beta,
    float* __restrict__ C, int64_t ldc, const float* __restrict__ bias, float slope,
    const float* __restrict__ dact, int64_t lddact, X3Cat cat) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[x3_lds_u16<BM, BN>()];
  const int tile = x3_item(tiles);
  x3_tile<BM, BN, TA, TB, EPI, true>(lds, M, N, K, K, 0, tile / tiles_n, tile % tiles_n, alpha, A, lda, B, ldb, beta, C,
                                     ldc, bias, slope, dact, lddact, nullptr, nullptr, nullptr, cat);
}

// Grouped split-K partials: the items of every part (its tiles x its K slices, slice-major)
// laid end to end, one launch for all of them (the step's weight gradients: the slab bytes
// then scale with the group's workgroups, not with each product's).
#ifndef PG_X3_GROUP_THREADS
#define PG_X3_GROUP_THREADS 256  // variant builds: 512 = 2 x 4 waves of 64 x 64 per 128 x 256 tile
#endif
#ifndef PG_X3_GROUP_WAVES
#define PG_X3_GROUP_WAVES (PG_X3_GROUP_THREADS == 512 ? 4 : x3_waves<BM, BN>())
#endif
template <int BM, int BN, bool TA, bool TB>
__global__ __launch_bounds__(PG_X3_GROUP_THREADS) __attribute__((amdgpu_waves_per_eu(PG_X3_GROUP_WAVES)))
void gemm_x3_group_kernel(X3Group g) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[x3_lds_u16<BM, BN>()];
  const int item = x3_item(g.items);
  int k = 0;
  while (k + 1 < g.n && item >= g.p[k + 1].first_item) ++k;
  const X3Part& p = g.p[k];
  const int local = item - p.first_item;
  const int kz = local / p.tiles, tile = local % p.tiles;
  x3_tile<BM, BN, TA, TB, EPI_SPLIT, false, PG_X3_GROUP_THREADS>(lds, p.M, p.N, p.K, p.kps, kz, tile / p.tiles_n,
                                                                 tile % p.tiles_n, 1.f, p.A,
                                     p.lda, p.B, p.ldb, 0.f, nullptr, 0, nullptr, 0.f, nullptr, 0, p.rowsum, p.ws,
                                     p.ws_rowsum);
}



template <int BM, int BN, bool TA, bool TB>
int launch_epi(const X3Args& a, hipStream_t st) {
  const dim3 grid((unsigned)(a.tiles * a.n_split)), block(NT);
#define PG_L(EPI_)                                                                                   \
  hipLaunchKernelGGL((gemm_x3_kernel<BM, BN, TA, TB, EPI_>), grid, block, 0, st, a.M, a.N, a.K, a.kps, \
                     a.tiles_n, a.tiles, a.alpha, a.A, a.lda, a.B, a.ldb, a.beta, a.C, a.ldc, a.bias,   \
                     a.slope, a.dact, a.lddact, a.rowsum, a.ws, a.ws_rowsum, a.n_split)
  switch (a.epi) {
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

template <int BM, int BN>
int launch_trans(const X3Args& a, hipStream_t st) {
  if (!a.ta && !a.tb) return launch_epi<BM, BN, false, false>(a, st);
  if (!a.ta && a.tb) return launch_epi<BM, BN, false, true>(a, st);
  if (a.ta && !a.tb) return launch_epi<BM, BN, true, false>(a, st);
  return launch_epi<BM, BN, true, true>(a, st);
}

}  // namespace

namespace pg_gemm {

int gemm_x3_group_launch(const X3Group& g, bool ta, bool tb, hipStream_t st) {
  const dim3 grid((unsigned)g.items), block(PG_X3_GROUP_THREADS);
#define PG_G(TA_, TB_) \
  hipLaunchKernelGGL((gemm_x3_group_kernel<kX3GroupBM, kX3GroupBN, TA_, TB_>), grid, block, 0, st, g)
  if (ta && !tb) PG_G(true, false);
  else if (!ta && !tb) PG_G(false, false);
  else if (!ta && tb) PG_G(false, true);
  else PG_G(true, true);
#undef PG_G
  return PG_OK;
}

#if PG_X3_BUFLOAD
template <int BM, int BN>
int launch_cat(const X3Args& a, const X3Cat& c, hipStream_t st) {
  if (a.ta || (a.epi != EPI_NONE && a.epi != EPI_LEAKY)) return PG_ERR_UNSUPPORTED;
  const dim3 grid((unsigned)a.tiles), block(NT);
#define PG_C(TB_, EPI_)                                                                                  \
  hipLaunchKernelGGL((gemm_x3_cat_kernel<BM, BN, false, TB_, EPI_>), grid, block, 0, st, a.M, a.N, a.K, \
                     a.tiles_n, a.tiles, a.alpha, a.A, a.lda, a.B, a.ldb, a.beta, a.C, a.ldc, a.bias, a.slope, \
                     a.dact, a.lddact, c)
  if (a.tb) {
    if (a.epi == EPI_NONE) PG_C(true, EPI_NONE); else PG_C(true, EPI_LEAKY);
  } else {
    if (a.epi == EPI_NONE) PG_C(false, EPI_NONE); else PG_C(false, EPI_LEAKY);
  }
#undef PG_C
  return PG_OK;
}

int gemm_x3_cat_launch(const X3Args& a, const float* A2, int64_t lda2, const float* B2, int64_t ldb2, int kcat,
                       hipStream_t st) {
  const X3Cat c{A2, lda2, B2, ldb2, kcat};
  if (a.bm == 128 && a.bn == 128) return launch_cat<128, 128>(a, c, st);
  if (a.bm == 128 && a.bn == 64) return launch_cat<128, 64>(a, c, st);
  if (a.bm == 64 && a.bn == 128) return launch_cat<64, 128>(a, c, st);
  if (a.bm == 64 && a.bn == 64) return launch_cat<64, 64>(a, c, st);
  return PG_ERR_UNSUPPORTED;  // a tile with no cat instantiation: the caller concatenates
}
#else
int gemm_x3_cat_launch(const X3Args&, const float*, int64_t, const float*, int64_t, int, hipStream_t) {
  return PG_ERR_UNSUPPORTED;
}
#endif

int gemm_x3_launch(const X3Args& a, hipStream_t st) {
  if (a.bm == 128 && a.bn == 128) return launch_trans<128, 128>(a, st);
  if (a.bm == 128 && a.bn == 64) return launch_trans<128, 64>(a, st);
  if (a.bm == 64 && a.bn == 128) return launch_trans<64, 128>(a, st);
  if (a.bm == 64 && a.bn == 64) return launch_trans<64, 64>(a, st);
  return PG_ERR_INVALID;
}

}  // namespace pg_gemm

#if PG_X3_STAMP
extern "C" int pg_x3_stamps(void* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(pg_x3_stamp), sizeof(pg_x3_stamp), 0, hipMemcpyDeviceToHost);
}
#endif
