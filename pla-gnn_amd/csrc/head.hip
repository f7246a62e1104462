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

#include <algorithm>
#include <cmath>

#include "adam_step.hpp"
#include "common.hpp"
#include "x3_split.hpp"

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
                                                                float* __restrict__ loss, float* adam_state = nullptr,
                                                                double lr = 0.0, double beta1 = 0.0,
                                                                double beta2 = 0.0) {
  // (optional) the step's Adam scalars, pg_adam_prepare's work, so the step has one tiny
  // launch fewer: it runs once per step here as there, before pg_adam_apply
  if (adam_state && blockIdx.x == 1 && threadIdx.x == 0) pg_adam::step_scalars(adam_state, lr, beta1, beta2);
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

// ---- liner1 + head + liner1's input gradient, fused (f32) --------------------------------
// The MLP on top of the last SAGE layer for one block of kL1Rows rows, in one pass:
//   A4  = leaky(H3 W1^T + b1)                (code/model.py:26-27; written out: liner2's weight
//                                             gradient reads it)
//   z, prob, loss terms, dz, dA4            (head_kernel above, on A4 held in LDS)
//   dH3 = (dA4 W1) * leaky'(H3)              (liner1's input gradient with the top SAGE layer's
//                                             activation backward: that layer's dY)
// Both products run as the three-piece GEMM does (gemm_x3.hip): the same split, the same
// 16-k steps in the same order, the same six MFMAs per block, zero past K; so A4 and dH3
// are bitwise the x3 GEMM's (and the head's outputs bitwise head_kernel's). Before, these
// were three launches (fwd.liner1, the head, dgrad.liner1: ~60 us per cfg2 step, the two
// GEMMs at ~60 TF/s: N = 104 columns on 64 x 64 tiles, K = 104 in 7 steps) that each
// streamed A3 / A4 / dA4 through memory.
// Block: 4 waves, kL1Rows = 32 rows. Phase 1: wave w owns A4 columns [32w, 32w + 32) (one
// 32 x 32 tile); the H3 rows go through LDS as three bf16 pieces in chunks of kL1Kc columns,
// W1's rows come straight from L2 into registers (each W1 element feeds one lane). Phase 3:
// wave w owns dH3 columns [64w, 64w + 64) of each 256-column chunk (two tiles); dA4's pieces
// sit in LDS, W1's columns come from L2 (8 rows x 32 consecutive columns per fragment).
constexpr int kL1Rows = 32;
constexpr int kL1Kc = 128;               // phase-1 K chunk staged in LDS
constexpr int kL1SA = kL1Kc + 8;         // piece row stride (u16): ds_read_b128 rows 4 banks apart
constexpr int kL1K1 = 128;               // liner1 width max (4 waves x 32 columns)
constexpr int kL1PD = 4;                 // W1 fragments in flight per wave (K steps ahead)
#ifndef PG_L1_WAVES
#define PG_L1_WAVES 3  // waves per SIMD the registers must allow (LDS: three blocks per CU)
#endif

using pg_x3::bf16x8;
using pg_x3::f32x16;

// dynamic LDS of one block (bytes) for liner1 width K1: the region that holds phase 1's H3
// pieces, then A4 (-> dA4) f32 [32][S] and dA4's pieces [3][32][K16 + 8]
__host__ __device__ inline int l1_region_bytes(int K1) {
  const int S = (K1 + 3) / 4 * 4 + 4, K16 = (K1 + 15) / 16 * 16;
  const int p1 = 3 * kL1Rows * kL1SA * 2;
  const int p23 = kL1Rows * S * 4 + 3 * kL1Rows * (K16 + 8) * 2;
  return (p1 > p23 ? p1 : p23 + 15) / 16 * 16;
}

// 8 consecutive floats -> the three bf16x8 fragments (pieces)
__device__ __forceinline__ void split8(const float4 lo, const float4 hi, bf16x8 (&f)[3]) {
  uint2 a[3], b[3];
  pg_x3::split4(lo, a);
  pg_x3::split4(hi, b);
#pragma unroll
  for (int p = 0; p < 3; ++p) f[p] = __builtin_bit_cast(bf16x8, make_uint4(a[p].x, a[p].y, b[p].x, b[p].y));
}

#ifndef PG_L1_SKIP
#define PG_L1_SKIP 0  // probe builds only (timing, wrong results): 1 / 2 / 3 skip that phase's products
#endif
#ifndef PG_L1_PRESPLIT
#define PG_L1_PRESPLIT 1  // W1's pieces split once per call in the fragments' own layout
#endif
// W1 [K1][F3] split once per call into its three bf16 pieces, stored fragment-native: for
// each piece, blocks of 32 rows x 8 k of 512 B, lane l of a fragment read owning the 16 B
// of row l (so a fragment read is one 512-B run per lane half):
//   p1: rows n < 128 (W1 rows, zero past K1), k < F16 (W1 columns, zero past F3): phase 1
//   p3: rows c < F32 (W1 columns, F3 rounded up to 32), k < K16 (W1 rows, zero past K1):
//       W1^T for phase 3
// (the same split4 as every other split: bitwise the pieces each block formed itself)
__host__ __device__ inline int64_t l1_p1_plane(int F3) { return (int64_t)kL1K1 * ((F3 + 15) / 16 * 16); }
__host__ __device__ inline int64_t l1_p3_plane(int F3, int K1) {
  return (int64_t)((F3 + 31) / 32 * 32) * ((K1 + 15) / 16 * 16);
}
__global__ __launch_bounds__(kBlock) void l1_split_kernel(const float* __restrict__ w1, int64_t ldw1, int K1, int F3,
                                                          uint16_t* __restrict__ p1, uint16_t* __restrict__ p3) {
  const int F16 = (F3 + 15) / 16 * 16, K16 = (K1 + 15) / 16 * 16, F32 = (F3 + 31) / 32 * 32;
  const int n1u = kL1K1 * (F16 / 8), n3u = F32 * (K16 / 8);
  const int u = blockIdx.x * kBlock + threadIdx.x;
  if (u >= n1u + n3u) return;
  float v[8];
  uint16_t* dst;
  int64_t plane;
  if (u < n1u) {  // unit (row block, k block, lane) -> W1[n][k0 .. k0 + 7]
    const int l = u & 31, kb = (u >> 5) % (F16 / 8), nb = (u >> 5) / (F16 / 8);
    const int n = 32 * nb + l, k0 = 8 * kb;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = n < K1 && k0 + i < F3 ? w1[(int64_t)n * ldw1 + k0 + i] : 0.f;
    dst = p1 + (int64_t)u * 8;
    plane = l1_p1_plane(F3);
  } else {        // -> W1[j0 .. j0 + 7][c]
    const int w = u - n1u;
    const int l = w & 31, kb = (w >> 5) % (K16 / 8), cb = (w >> 5) / (K16 / 8);
    const int c = 32 * cb + l, j0 = 8 * kb;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = c < F3 && j0 + i < K1 ? w1[(int64_t)(j0 + i) * ldw1 + c] : 0.f;
    dst = p3 + (int64_t)w * 8;
    plane = l1_p3_plane(F3, K1);
  }
  uint2 a[3], b[3];
  pg_x3::split4(make_float4(v[0], v[1], v[2], v[3]), a);
  pg_x3::split4(make_float4(v[4], v[5], v[6], v[7]), b);
#pragma unroll
  for (int p = 0; p < 3; ++p) *reinterpret_cast<uint4*>(dst + p * plane) = make_uint4(a[p].x, a[p].y, b[p].x, b[p].y);
}

// one f32 value's three pieces, as split4 forms each lane of its quad
__device__ __forceinline__ void split1(float x, uint16_t (&q)[3]) {
#pragma unroll
  for (int piece = 0; piece < 3; ++piece) {
    const uint32_t pk = pg_x3::pk_bf16(x, 0.f);
    q[piece] = (uint16_t)(pk & 0xFFFFu);
    if (piece < 2) x = x - pg_x3::lo_f(pk);
  }
}

// Adam over the flat parameters (pg_adam_apply's update, pg_adam::elem) that also keeps W1's
// pieces current: the thread that writes W1[r][k] (k < F3, r < K1) stores its three pieces at
// that element's places in both fragment-native layouts (l1_split_kernel's p1 and p3). W1's
// elements go to the first blocks of the grid, the other parameters to the rest. The
// pieces' zero pads are never touched, so one pg_mlp_l1_split before the first step keeps
// them. Replaces the split launch that each fused-head call made before (the step's W1
// changes only here).
__global__ __launch_bounds__(kBlock) void adam_apply_l1_kernel(
    float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v, int64_t n,
    const float* __restrict__ state, float beta1, float beta2, float a1, float a2, float eps, float wd,
    int64_t w1_off, int ldw1, int K1, int F3, uint16_t* __restrict__ p1, uint16_t* __restrict__ p3, int nb1) {
  const float step_size = state[1];
  const float bc2s = state[2];
  const int64_t nw1 = (int64_t)K1 * ldw1;
  if ((int)blockIdx.x < nb1) {
    // the first nb1 blocks: W1's elements (their piece stores are the slow part, so these
    // blocks start first)
    const int F16 = (F3 + 15) / 16 * 16, K16 = (K1 + 15) / 16 * 16;
    const int64_t pl1 = l1_p1_plane(F3), pl3 = l1_p3_plane(F3, K1);
    for (int64_t j = blockIdx.x * (int64_t)kBlock + threadIdx.x; j < nw1; j += (int64_t)nb1 * kBlock) {
      const float pi = pg_adam::elem(p, g, m, v, w1_off + j, step_size, bc2s, beta1, beta2, a1, a2, eps, wd);
      const int r = (int)(j / ldw1), k = (int)(j - (int64_t)r * ldw1);
      if (k < F3) {
        uint16_t q[3];
        split1(pi, q);
        // p1: block (r / 32, k / 8), lane r % 32, element k % 8
        const int64_t e1 = ((int64_t)((r >> 5) * (F16 / 8) + (k >> 3)) * 32 + (r & 31)) * 8 + (k & 7);
        // p3 (W1^T): block (k / 32, r / 8), lane k % 32, element r % 8
        const int64_t e3 = ((int64_t)((k >> 5) * (K16 / 8) + (r >> 3)) * 32 + (k & 31)) * 8 + (r & 7);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          p1[e1 + c * pl1] = q[c];
          p3[e3 + c * pl3] = q[c];
        }
      }
    }
    return;
  }
  // the rest: every other parameter, as pg_adam_apply
  const int64_t nrest = n - nw1;
  const int nb = (int)gridDim.x - nb1;
  for (int64_t u = (blockIdx.x - nb1) * (int64_t)kBlock + threadIdx.x; u < nrest; u += (int64_t)nb * kBlock) {
    const int64_t i = u < w1_off ? u : u + nw1;
    pg_adam::elem(p, g, m, v, i, step_size, bc2s, beta1, beta2, a1, a2, eps, wd);
  }
}

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(PG_L1_WAVES))) void mlp_l1_head_kernel(
    const float* __restrict__ h3, int64_t ldh, int n, int F3, const float* __restrict__ w1, int64_t ldw1,
    const float* __restrict__ b1, int K1, float* __restrict__ a4g, int64_t lda4,
    const float* __restrict__ w2, int64_t ldw, const float* __restrict__ b2, int C,
    const float* __restrict__ labels, int64_t ldl, const float* __restrict__ cw,
    const int8_t* __restrict__ row_set, float inv_n_train, float* __restrict__ prob, int64_t ldp,
    float* __restrict__ dz, int64_t lddz, float* __restrict__ da4g, int64_t ldg,
    float* __restrict__ dh3, int64_t lddh, float slope, float* __restrict__ part, int nb,
    const uint16_t* __restrict__ p1, const uint16_t* __restrict__ p3) {
  extern __shared__ __attribute__((aligned(16))) unsigned char region[];
  __shared__ __attribute__((aligned(16))) float w[kMaxC * (kMaxK + 4)];
  __shared__ float g[kRows][kMaxC];
  __shared__ float terms[2][kRows][kMaxC];
  static_assert(kRows == kL1Rows, "head rows");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int K4 = (K1 + 3) / 4 * 4, S = K4 + 4, K16 = (K1 + 15) / 16 * 16, SD = K16 + 8;
  uint16_t* sp = reinterpret_cast<uint16_t*>(region);                       // phase 1: [3][32][kL1SA]
  float* a = reinterpret_cast<float*>(region);                              // phase 2: A4 -> dA4 [32][S]
  uint16_t* sd = reinterpret_cast<uint16_t*>(region + kL1Rows * S * 4);     // phase 3: [3][32][SD]
  const int r0 = blockIdx.x * kL1Rows;
  const int nr = min(kL1Rows, n - r0);

  // W2 into LDS (the head's operand), issued first
  {
    const int uw = C * (K4 / 4);
    for (int u = tid; u < uw; u += kBlock) {
      const int c = u / (K4 / 4), k = (u - c * (K4 / 4)) * 4;
      *reinterpret_cast<float4*>(w + c * S + k) = ld4(w2, (int64_t)c * ldw, k, K1);
    }
  }
  for (int i = tid; i < 2 * kRows * kMaxC; i += kBlock) (&terms[0][0][0])[i] = 0.f;
  // the head's per-thread inputs (class c = tid % 16 of rows tid / 16 and tid / 16 + 16),
  // loaded now so that phase 2 does not wait on them
  constexpr int kHH = kRows / (kBlock / kMaxC);
  int hset[kHH];
  float hlab[kHH];
  const int hc = min(tid % kMaxC, C - 1);
  const float hwc = cw[2 * hc], hwp1 = cw[2 * hc + 1], hb2 = b2[hc];
#pragma unroll
  for (int hh = 0; hh < kHH; ++hh) {
    const int64_t r = min(r0 + tid / kMaxC + hh * (kBlock / kMaxC), n - 1);
    hset[hh] = row_set[r];
    hlab[hh] = labels[r * ldl + hc];
  }

  // ---- phase 1: A4 = leaky(H3 W1^T + b1) ----
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int n1 = 32 * wave + l32;                       // this lane's A4 column (W1 row)
  const bool live1 = n1 < K1;
#if !PG_L1_PRESPLIT
  // W1 through a buffer descriptor over its K1 rows: rows past K1 read 0 (the range check
  // covers the VGPR offset, which therefore carries the whole offset); every offset fits 32
  // bits (the host checks the extents). Each block splits the W1 fragments it reads (a
  // version reading pieces split once per call, in these layouts, was slower: 62 vs 44 us
  // per cfg2 call, the transposed pieces' rows being 224 B apart)
  const __amdgpu_buffer_rsrc_t rw1 = pg_x3::rsrc(w1, (uint32_t)K1 * (uint32_t)ldw1 * 4u);
  const int vo1 = (n1 * (int)ldw1 + 8 * h) * 4;
  // W1 row n1 at k = 16 s + 8 h .. + 7 (zero past F3)
  auto ldb1 = [&](int s, float4& lo, float4& hi) {
    const int k = 16 * s + 8 * h;
    const float4 x = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rw1, vo1 + 64 * s, 0, 0));
    const float4 y = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rw1, vo1 + 64 * s + 16, 0, 0));
    lo = k < F3 ? x : make_float4(0.f, 0.f, 0.f, 0.f);
    hi = k + 4 < F3 ? y : make_float4(0.f, 0.f, 0.f, 0.f);
  };
#endif
  const int steps1 = (F3 + 15) / 16;
#if PG_L1_PRESPLIT
  // p1's fragment of step s: block (wave, 2 s + h), this lane's 16 B, per piece
  const __amdgpu_buffer_rsrc_t rp1 = pg_x3::rsrc(p1, (uint32_t)(3 * l1_p1_plane(F3) * 2));
  const int pl1 = (int)(l1_p1_plane(F3) * 2), kb1 = (F3 + 15) / 16 * 2;
  auto ldf1 = [&](int s, bf16x8 (&f)[3]) {
    const int off = ((wave * kb1 + 2 * s + h) * 32 + l32) * 16;
#pragma unroll
    for (int p = 0; p < 3; ++p)
      f[p] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rp1, off + p * pl1, 0, 0));
  };
  bf16x8 bq[kL1PD][3];
#pragma unroll
  for (int i = 0; i < kL1PD; ++i) ldf1(min(i, steps1 - 1), bq[i]);
#else
  float4 bq[kL1PD][2];
#pragma unroll
  for (int i = 0; i < kL1PD; ++i) ldb1(min(i, steps1 - 1), bq[i][0], bq[i][1]);
#endif
  // H3[r0 .. r0 + 31][kc .. kc + kL1Kc) in registers, one chunk ahead (the next chunk's
  // loads are in flight during this chunk's MFMAs); zero past F3, rows past n read a clamped
  // valid row (never stored)
  constexpr int kPer = kL1Rows * kL1Kc / 4 / kBlock;  // 4 float4 units per thread
  float4 hv[kPer];
  auto ldh3 = [&](int kc) {
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int u = tid + q * kBlock, row = u / (kL1Kc / 4), k4 = (u % (kL1Kc / 4)) * 4;
      const float4 x = *reinterpret_cast<const float4*>(h3 + (int64_t)min(r0 + row, n - 1) * ldh + min(kc + k4, F3 - 4));
      hv[q] = kc + k4 < F3 ? x : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  ldh3(0);
  for (int kc = 0; kc < F3; kc += kL1Kc) {
    // stage the chunk as pieces, then start the next chunk's loads
    {
      float4* v = hv;
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        const int u = tid + q * kBlock, row = u / (kL1Kc / 4), k4 = (u % (kL1Kc / 4)) * 4;
        uint2 pc[3];
        pg_x3::split4(v[q], pc);
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(sp + (p * kL1Rows + row) * kL1SA + k4) = pc[p];
      }
    }
    __syncthreads();
    if (kc + kL1Kc < F3) ldh3(kc + kL1Kc);
    // the chunk's K steps (kL1Kc / 16 = 8, a multiple of kL1PD); W1 fragments kL1PD steps
    // ahead in a register ring (loads unconditional, clamped; the MFMAs of steps past F3 skipped)
    const int sc = kc / 16;
#pragma nounroll
    for (int i0 = 0; i0 < kL1Kc / 16; i0 += kL1PD) {
#pragma unroll
      for (int j = 0; j < kL1PD; ++j) {
        const int i = i0 + j, s = sc + i;
#if PG_L1_PRESPLIT
        if (s < steps1 && PG_L1_SKIP != 1) {
          bf16x8 fa[3];
#pragma unroll
          for (int p = 0; p < 3; ++p)
            fa[p] = *reinterpret_cast<const bf16x8*>(sp + (p * kL1Rows + l32) * kL1SA + 16 * i + 8 * h);
          pg_x3::mfma6(acc, fa, bq[j]);
        }
        if (PG_L1_SKIP != 1) ldf1(min(s + kL1PD, steps1 - 1), bq[j]);
#else
        bf16x8 fb[3];
        split8(bq[j][0], bq[j][1], fb);
        ldb1(min(s + kL1PD, steps1 - 1), bq[j][0], bq[j][1]);
        if (s < steps1) {
          bf16x8 fa[3];
#pragma unroll
          for (int p = 0; p < 3; ++p)
            fa[p] = *reinterpret_cast<const bf16x8*>(sp + (p * kL1Rows + l32) * kL1SA + 16 * i + 8 * h);
          pg_x3::mfma6(acc, fa, fb);
        }
#endif
        __builtin_amdgcn_sched_barrier(0);  // one step's fragments live at a time
      }
    }
    __syncthreads();  // the pieces are restaged (next chunk) or reused (phase 2)
  }
  // epilogue: + b1, leaky (as x3_store: 1 * acc, + bias, act); A4 to LDS and out
  {
    const float bb = live1 ? b1[n1] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
      float o = 1.f * acc[r];
      o = o + bb;
      o = o > 0.f ? o : o * slope;
      if (n1 < K4) a[row * S + n1] = live1 ? o : 0.f;
      if (live1 && row < nr) a4g[(int64_t)(r0 + row) * lda4 + n1] = o;
    }
  }
  __syncthreads();

  // ---- phase 2: the head (head_kernel's arithmetic, A4 from LDS) ----
  {
    const int c = tid % kMaxC, rg = tid / kMaxC;
#pragma unroll
    for (int hh = 0; hh < kRows / (kBlock / kMaxC); ++hh) {
      const int ri = rg + hh * (kBlock / kMaxC);
      if (c < C && ri < nr) {
        const int64_t r = r0 + ri;
        const int set = hset[hh];
        const float t = hlab[hh];
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
        zz = zz + hb2;
        const float pr = 1.f / (1.f + expf(-zz));
        if (prob) prob[r * ldp + c] = pr;
        float gz = 0.f;
        if (set != 0) {
          const float wc = hwc;
          const float wp1 = hwp1;
          const float cp = fminf(fmaxf(pr, 1e-9f), 10.f);
          const float q = 1.f - pr;
          const float cq = fminf(fmaxf(q, 1e-9f), 10.f);
          const float la = logf(cp), lb = logf(cq);
          terms[set - 1][ri][c] = ((t * la) * wc + (1.f - t) * lb) / wp1 * 2.f;
          if (set == 1) {
            float gg = -inv_n_train;
            gg = gg * 2.f;
            gg = gg / wp1;
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
      } else {
        g[ri][c] = 0.f;
      }
    }
  }
  __syncthreads();
  if (tid < 2 * C) {
    const int set = tid / C, c = tid % C;
    float s = 0.f;
    for (int ri = 0; ri < nr; ++ri) s += terms[set][ri][c];
    part[((int64_t)set * C + c) * nb + blockIdx.x] = s;
  }
  // dA4 = (dz W2) * leaky'(A4), in place of A4 (each element read and written by one thread)
  {
    const int j = tid % kMaxK, r2 = tid / kMaxK;
    if (j < K4) {
      float wj[kMaxC];
#pragma unroll
      for (int c = 0; c < kMaxC; ++c) wj[c] = c < C && j < K1 ? w[c * S + j] : 0.f;
      for (int ri = r2; ri < kL1Rows; ri += kBlock / kMaxK) {
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < kMaxC; ++c) s = fmaf(g[ri][c], wj[c], s);
        const float y = a[ri * S + j];
        const float d = y > 0.f ? s : s * slope;
        a[ri * S + j] = j < K1 ? d : 0.f;
        if (j < K1 && ri < nr) da4g[(int64_t)(r0 + ri) * ldg + j] = d;
      }
    }
  }
  __syncthreads();
  // dA4's pieces (zero past K1, up to the 16-k steps' end)
  for (int u = tid; u < kL1Rows * (K16 / 4); u += kBlock) {
    const int row = u / (K16 / 4), k4 = (u % (K16 / 4)) * 4;
    const float4 x = k4 < K4 ? *reinterpret_cast<const float4*>(a + row * S + k4) : make_float4(0.f, 0.f, 0.f, 0.f);
    uint2 pc[3];
    pg_x3::split4(x, pc);
#pragma unroll
    for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(sd + (p * kL1Rows + row) * SD + k4) = pc[p];
  }
  __syncthreads();

  // ---- phase 3: dH3 = (dA4 W1) * leaky'(H3), one 32-column tile per wave and pass ----
  const int steps3 = K16 / 16;
  for (int c0 = 32 * wave; c0 < (PG_L1_SKIP == 3 ? 0 : F3); c0 += 128) {
    const int col = c0 + l32;
    const int colc = min(col, F3 - 1);
#if !PG_L1_PRESPLIT
    // W1[k][col], k = 16 s + 8 h + i (i < 8): one strided column piece per fragment (each load
    // instruction: 32 consecutive floats of one W1 row per lane half); rows past K1 read 0
    // through the descriptor
    const int vo3 = (8 * h * (int)ldw1 + colc) * 4;
    auto ldb3 = [&](int s, float (&v)[8]) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        v[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw1, vo3 + (16 * s + i) * (int)ldw1 * 4, 0, 0));
    };
#endif
    // the activation operand of the epilogue, loaded first (used last); rows past n read 0
    float y[16];
    {
      const __amdgpu_buffer_rsrc_t rh = pg_x3::rsrc(h3, (uint32_t)n * (uint32_t)ldh * 4u);
      const int voy = (4 * h * (int)ldh + colc) * 4;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = r0 + (r & 3) + 8 * (r >> 2);
        y[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rh, voy + rr * (int)ldh * 4, 0, 0));
      }
    }
    f32x16 acc3;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc3[r] = 0.f;
    // every K step's W1 fragment of this tile in flight at once (K1 <= 128: at most 8 steps;
    // steps past K16 read zeros and are not multiplied)
#if PG_L1_PRESPLIT
    // p3's fragment of step s: block (c0 / 32, 2 s + h), this lane's 16 B, per piece;
    // kL1PD steps ahead in a register ring
    const __amdgpu_buffer_rsrc_t rp3 = pg_x3::rsrc(p3, (uint32_t)(3 * l1_p3_plane(F3, K1) * 2));
    const int pl3 = (int)(l1_p3_plane(F3, K1) * 2), kb3 = K16 / 8;
    auto ldf3 = [&](int s, bf16x8 (&f)[3]) {
      const int off = (((c0 >> 5) * kb3 + 2 * s + h) * 32 + l32) * 16;
#pragma unroll
      for (int p = 0; p < 3; ++p)
        f[p] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rp3, off + p * pl3, 0, 0));
    };
    bf16x8 bv[kL1PD][3];
#pragma unroll
    for (int i = 0; i < kL1PD; ++i) ldf3(min(i, steps3 - 1), bv[i]);
#pragma nounroll
    for (int s0 = 0; s0 < steps3; s0 += kL1PD) {
#pragma unroll
      for (int i = 0; i < kL1PD; ++i) {
        const int s = s0 + i;
        if (s < steps3) {
          bf16x8 fa[3];
#pragma unroll
          for (int p = 0; p < 3; ++p)
            fa[p] = *reinterpret_cast<const bf16x8*>(sd + (p * kL1Rows + l32) * SD + 16 * s + 8 * h);
          pg_x3::mfma6(acc3, fa, bv[i]);
        }
        ldf3(min(s + kL1PD, steps3 - 1), bv[i]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#else
    float bv[kL1K1 / 16][8];
#pragma unroll
    for (int s = 0; s < kL1K1 / 16; ++s) ldb3(s, bv[s]);
#pragma unroll
    for (int s = 0; s < kL1K1 / 16; ++s) {
      if (s < steps3) {
        bf16x8 fb[3], fa[3];
        split8(make_float4(bv[s][0], bv[s][1], bv[s][2], bv[s][3]), make_float4(bv[s][4], bv[s][5], bv[s][6], bv[s][7]),
               fb);
#pragma unroll
        for (int p = 0; p < 3; ++p)
          fa[p] = *reinterpret_cast<const bf16x8*>(sd + (p * kL1Rows + l32) * SD + 16 * s + 8 * h);
        pg_x3::mfma6(acc3, fa, fb);
      }
    }
#endif
    // epilogue: act'(H3) (as x3_store's EPI_DLEAKY: 1 * acc, then y > 0 ? x : x slope)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
      const float o = 1.f * acc3[r];
      if (row < nr && col < F3) dh3[(int64_t)(r0 + row) * lddh + col] = y[r] > 0.f ? o : o * slope;
    }
  }
}

bool l1_shape_ok(int32_t F3, int32_t K1) { return F3 > 0 && F3 % 4 == 0 && F3 <= 4096 && K1 > 0 && K1 <= kL1K1; }
void l1_split_launch(const float* w1, int64_t ldw1, int32_t F3, int32_t K1, uint16_t* p1, uint16_t* p3,
                     hipStream_t st) {
  const int units = (int)(kL1K1 * ((F3 + 15) / 16 * 2) + ((F3 + 31) / 32 * 32) * ((K1 + 15) / 16 * 2));
  hipLaunchKernelGGL(l1_split_kernel, dim3((units + kBlock - 1) / kBlock), dim3(kBlock), 0, st, w1, ldw1, (int)K1,
                     (int)F3, p1, p3);
}
uint16_t* l1_p3_of(void* pieces, int32_t F3) {
  return (uint16_t*)pieces + ((size_t)(3 * l1_p1_plane(F3) * 2 + 255) / 256 * 256) / 2;
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

size_t pg_mlp_l1_head_workspace(int64_t n, int32_t C, int32_t F3, int32_t K1) {
  const size_t head = (pg_mlp_head_workspace(n, C) + 255) / 256 * 256;
  if (!PG_L1_PRESPLIT || F3 <= 0 || K1 <= 0) return head;
  const size_t p1 = (size_t)(3 * l1_p1_plane(F3) * 2 + 255) / 256 * 256;
  return head + p1 + (size_t)(3 * l1_p3_plane(F3, K1) * 2);
}

size_t pg_mlp_l1_pieces_bytes(int32_t F3, int32_t K1) {
  if (F3 <= 0 || K1 <= 0) return 0;
  return (size_t)(3 * l1_p1_plane(F3) * 2 + 255) / 256 * 256 + (size_t)(3 * l1_p3_plane(F3, K1) * 2);
}

int pg_mlp_l1_split(const float* w1, int64_t ldw1, int32_t F3, int32_t K1, void* pieces, pg_stream_t stream) {
  if (!l1_shape_ok(F3, K1) || ldw1 < F3) return pg::set_error(PG_ERR_INVALID, "pg_mlp_l1_split: bad shape");
  if (!w1 || !pieces || ((uintptr_t)pieces & 255))
    return pg::set_error(PG_ERR_INVALID, "pg_mlp_l1_split: NULL W1, or pieces not 256-B aligned");
  l1_split_launch(w1, ldw1, F3, K1, (uint16_t*)pieces, l1_p3_of(pieces, F3), (hipStream_t)stream);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pg::set_error((int)e, "pg_mlp_l1_split: launch failed: %s", hipGetErrorString(e));
  return pg::ok();
}

int pg_adam_apply_l1(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                     const float* state, double beta1, double beta2, double eps, double weight_decay,
                     int64_t w1_offset, int64_t ldw1, int32_t F3, int32_t K1, void* pieces, pg_stream_t stream) {
  if (n < 0 || !state) return pg::set_error(PG_ERR_INVALID, "pg_adam_apply_l1: bad arguments");
  if (!l1_shape_ok(F3, K1) || ldw1 < F3 || ldw1 > INT32_MAX || w1_offset < 0 || w1_offset + (int64_t)K1 * ldw1 > n)
    return pg::set_error(PG_ERR_INVALID, "pg_adam_apply_l1: W1 [K1][ldw1] must lie inside the n parameters");
  if (!param || !grad || !exp_avg || !exp_avg_sq || !pieces || ((uintptr_t)pieces & 255))
    return pg::set_error(PG_ERR_INVALID, "pg_adam_apply_l1: NULL buffer, or pieces not 256-B aligned");
  const int64_t nw1 = (int64_t)K1 * ldw1;
  const int nb1 = (int)std::min<int64_t>((nw1 + kBlock - 1) / kBlock, 4096);
  const int64_t blocks = nb1 + std::max<int64_t>(1, std::min<int64_t>((n - nw1 + kBlock - 1) / kBlock, 32768));
  hipLaunchKernelGGL(adam_apply_l1_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream, param,
                     grad, exp_avg, exp_avg_sq, n, state, (float)beta1, (float)beta2, (float)(1.0 - beta1),
                     (float)(1.0 - beta2), (float)eps, (float)weight_decay, w1_offset, (int)ldw1, (int)K1, (int)F3,
                     (uint16_t*)pieces, l1_p3_of(pieces, F3), nb1);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pg::set_error((int)e, "pg_adam_apply_l1: launch failed: %s", hipGetErrorString(e));
  return pg::ok();
}

static int mlp_l1_head_impl(const float* h3, int64_t ldh, int64_t n, int32_t F3, const float* w1, int64_t ldw1,
                   const float* b1, int32_t K1, float* a4, int64_t lda4, const float* w2, int64_t ldw,
                   const float* b2, int32_t C, const float* labels, int64_t ldl, const float* class_w,
                   const int8_t* row_set, int64_t n_train, int64_t n_val, float* prob, int64_t ldp,
                   float* dz, int64_t lddz, float* da4, int64_t ldg, float* dh3, int64_t lddh, float slope,
                   float* loss2, void* ws, size_t ws_bytes, float* adam_state, double lr, double beta1,
                   double beta2, const void* pieces, pg_stream_t stream) {
  if (n < 0 || n > INT32_MAX || F3 <= 0 || F3 % 4 != 0 || F3 > 4096 || K1 <= 0 || K1 > kL1K1 || K1 > kMaxK ||
      C <= 0 || C > kMaxC || ldh < F3 || ldw1 < F3 || lda4 < K1 || ldw < K1 || ldl < C || (prob && ldp < C) ||
      (dz && lddz < C) || ldg < K1 || lddh < F3)
    return pg::set_error(PG_ERR_INVALID, "pg_mlp_l1_head: bad shape (F3 %% 4 == 0, F3 <= 4096, K1 <= %d, C <= %d)",
                         kL1K1, kMaxC);
  if (n == 0) return pg::ok();
  if (!h3 || !w1 || !b1 || !a4 || !w2 || !b2 || !labels || !class_w || !row_set || !da4 || !dh3 || !loss2 || !ws)
    return pg::set_error(PG_ERR_INVALID, "pg_mlp_l1_head: NULL buffer");
  if (((uintptr_t)h3 & 15) || (ldh & 3) || ((uintptr_t)w1 & 15) || (ldw1 & 3) || ((uintptr_t)w2 & 15) || (ldw & 3) ||
      ((uintptr_t)ws & 255))
    return pg::set_error(PG_ERR_INVALID, "pg_mlp_l1_head: H3, W1, W2 need 16-B aligned rows, ws 256-B alignment");
  if ((double)n * (double)ldh * 4.0 >= 2147483648.0 || (double)K1 * (double)ldw1 * 4.0 >= 2147483648.0)
    return pg::set_error(PG_ERR_UNSUPPORTED, "pg_mlp_l1_head: H3 / W1 of 2 GiB or more");
  if (ws_bytes < pg_mlp_l1_head_workspace(n, C, F3, K1))
    return pg::set_error(PG_ERR_WORKSPACE, "pg_mlp_l1_head: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int nb = (int)((n + kL1Rows - 1) / kL1Rows);
  float* part = (float*)ws;
  uint16_t* p1 = nullptr;
  uint16_t* p3 = nullptr;
  if (pieces) {  // kept current by the caller (pg_mlp_l1_split, pg_adam_apply_l1)
    if (!PG_L1_PRESPLIT || ((uintptr_t)pieces & 255))
      return pg::set_error(PG_ERR_INVALID, "pg_mlp_l1_head_ex: pieces not 256-B aligned");
    p1 = (uint16_t*)pieces;
    p3 = l1_p3_of((void*)pieces, F3);
  } else if (PG_L1_PRESPLIT) {
    p1 = (uint16_t*)((char*)ws + (pg_mlp_head_workspace(n, C) + 255) / 256 * 256);
    p3 = l1_p3_of(p1, F3);
    l1_split_launch(w1, ldw1, F3, K1, p1, p3, st);
  }
  const float inv_n = n_train > 0 ? 1.0f / (float)n_train : 0.f;
  hipLaunchKernelGGL(mlp_l1_head_kernel, dim3(nb), dim3(kBlock), (unsigned)l1_region_bytes(K1), st, h3, ldh, (int)n,
                     (int)F3, w1, ldw1, b1, (int)K1, a4, lda4, w2, ldw, b2, (int)C, labels, ldl, class_w, row_set, inv_n,
                     prob, ldp, dz, lddz, da4, ldg, dh3, lddh, slope, part, nb, (const uint16_t*)p1,
                     (const uint16_t*)p3);
  hipLaunchKernelGGL(head_final_kernel, dim3(2), dim3(64 * kMaxC), 0, st, (const float*)part, nb, (int)C, n_train,
                     n_val, loss2, adam_state, lr, beta1, beta2);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pg::set_error((int)e, "pg_mlp_l1_head: launch failed: %s", hipGetErrorString(e));
  return pg::ok();
}

int pg_mlp_l1_head(const float* h3, int64_t ldh, int64_t n, int32_t F3, const float* w1, int64_t ldw1,
                   const float* b1, int32_t K1, float* a4, int64_t lda4, const float* w2, int64_t ldw,
                   const float* b2, int32_t C, const float* labels, int64_t ldl, const float* class_w,
                   const int8_t* row_set, int64_t n_train, int64_t n_val, float* prob, int64_t ldp,
                   float* dz, int64_t lddz, float* da4, int64_t ldg, float* dh3, int64_t lddh, float slope,
                   float* loss2, void* ws, size_t ws_bytes, float* adam_state, double lr, double beta1,
                   double beta2, pg_stream_t stream) {
  return mlp_l1_head_impl(h3, ldh, n, F3, w1, ldw1, b1, K1, a4, lda4, w2, ldw, b2, C, labels, ldl, class_w, row_set,
                          n_train, n_val, prob, ldp, dz, lddz, da4, ldg, dh3, lddh, slope, loss2, ws, ws_bytes,
                          adam_state, lr, beta1, beta2, nullptr, stream);
}

int pg_mlp_l1_head_ex(const float* h3, int64_t ldh, int64_t n, int32_t F3, const float* w1, int64_t ldw1,
                      const float* b1, int32_t K1, float* a4, int64_t lda4, const float* w2, int64_t ldw,
                      const float* b2, int32_t C, const float* labels, int64_t ldl, const float* class_w,
                      const int8_t* row_set, int64_t n_train, int64_t n_val, float* prob, int64_t ldp,
                      float* dz, int64_t lddz, float* da4, int64_t ldg, float* dh3, int64_t lddh, float slope,
                      float* loss2, void* ws, size_t ws_bytes, float* adam_state, double lr, double beta1,
                      double beta2, const void* w1_pieces, pg_stream_t stream) {
  if (!w1_pieces) return pg::set_error(PG_ERR_INVALID, "pg_mlp_l1_head_ex: NULL pieces");
  return mlp_l1_head_impl(h3, ldh, n, F3, w1, ldw1, b1, K1, a4, lda4, w2, ldw, b2, C, labels, ldl, class_w, row_set,
                          n_train, n_val, prob, ldp, dz, lddz, da4, ldg, dh3, lddh, slope, loss2, ws, ws_bytes,
                          adam_state, lr, beta1, beta2, w1_pieces, stream);
}

}  // extern "C"
