// Message-passing kernels for gfx950 (MI355X): CSR SpMM with max/argmax (DGL
// SpMMCmpCsr<copy_lhs|u_mul_e, Max>, reached from SAGEConv('pool') at
// code/model.py:20/22/24), its backward (DGL GSpMM.backward scatter_add_ through argX,
// reached from code/train.py:204), and the sum/mean variants.
//
// Work decomposition: one 64-lane wave per schedule item {row, k0, k1, slot}. A row
// longer than the schedule's chunk is cut into several items whose partial results go
// to workspace slots and are combined in chunk order by a merge kernel, so hub rows do
// not serialise on one wave. Items are ordered longest first (pg_schedule_build).
// Inside a wave each lane owns W consecutive features (W = 4: float4 loads, 1 KiB per
// wave-instruction; W = 1: scalar path for unaligned rows) in NC chunks of 64*W.
// Row indices and weights are wave-uniform and come through the scalar cache.
//
// Numerics: the max is a selection (bit-exact); ties keep the earlier entry (strict >),
// matching DGL's in-order loop. Backward sums run in ascending destination order, the
// same order as a sequential scatter_add_, so unsplit rows are bit-exact against it.
// Build with -ffp-contract=off (no silent FMA contraction).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <type_traits>

#include "common.hpp"
#include "x3_split.hpp"

namespace {

// global agent-scope words (split-row tickets) and the buffer builtins' vector types
typedef __attribute__((address_space(1))) uint32_t pg_gu32;
typedef uint32_t pg_u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t pg_u32x2 __attribute__((ext_vector_type(2)));

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kMaxNC = 4;       // vector path: F <= 4 * 256 per launch
constexpr int kMaxNCScalar = 16; // scalar path: F <= 16 * 64 per launch

template <typename A>
__device__ __forceinline__ int arg_none();
template <>
__device__ __forceinline__ int arg_none<uint16_t>() { return 0xFFFF; }
template <>
__device__ __forceinline__ int arg_none<int32_t>() { return -1; }

__device__ __forceinline__ int wave_id_uniform() {
  return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// ---- element types: float, or bf16 storage (uint16_t bits) computed in f32 ------------
__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }
template <typename T>
__device__ __forceinline__ T from_f(float x);
template <>
__device__ __forceinline__ float from_f<float>(float x) { return x; }
template <>
__device__ __forceinline__ uint16_t from_f<uint16_t>(float x) {  // round to nearest even
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(x));
}

// ---- per-lane feature tile access ----------------------------------------------------
template <int W, typename T = float>
__device__ __forceinline__ void load_tile(const T* __restrict__ row, int f, int F,
                                          float (&r)[W], float fill) {
  if constexpr (W == 4) {
    if (f < F) {
      if constexpr (sizeof(T) == 4) {
        const float4 t = *reinterpret_cast<const float4*>(row + f);
        r[0] = t.x; r[1] = t.y; r[2] = t.z; r[3] = t.w;
      } else {
        const uint2 t = *reinterpret_cast<const uint2*>(row + f);
        r[0] = to_f((uint16_t)(t.x & 0xFFFF)); r[1] = to_f((uint16_t)(t.x >> 16));
        r[2] = to_f((uint16_t)(t.y & 0xFFFF)); r[3] = to_f((uint16_t)(t.y >> 16));
      }
    } else {
      r[0] = r[1] = r[2] = r[3] = fill;
    }
  } else {
    r[0] = f < F ? to_f(row[f]) : fill;
  }
}

template <int W, typename T = float>
__device__ __forceinline__ void store_tile(T* __restrict__ row, int f, int F,
                                           const float (&r)[W]) {
  if constexpr (W == 4) {
    if (f < F) {
      if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<float4*>(row + f) = make_float4(r[0], r[1], r[2], r[3]);
      } else {
        uint2 t;
        t.x = (uint32_t)from_f<uint16_t>(r[0]) | ((uint32_t)from_f<uint16_t>(r[1]) << 16);
        t.y = (uint32_t)from_f<uint16_t>(r[2]) | ((uint32_t)from_f<uint16_t>(r[3]) << 16);
        *reinterpret_cast<uint2*>(row + f) = t;
      }
    }
  } else {
    if (f < F) row[f] = from_f<T>(r[0]);
  }
}

template <int W, typename A>
__device__ __forceinline__ void load_arg(const A* __restrict__ row, int f, int F, int (&r)[W]) {
  if constexpr (W == 4) {
    if (f < F) {
      if constexpr (sizeof(A) == 2) {
        const uint2 t = *reinterpret_cast<const uint2*>(row + f);
        r[0] = t.x & 0xFFFF; r[1] = t.x >> 16; r[2] = t.y & 0xFFFF; r[3] = t.y >> 16;
      } else {
        const int4 t = *reinterpret_cast<const int4*>(row + f);
        r[0] = t.x; r[1] = t.y; r[2] = t.z; r[3] = t.w;
      }
    } else {
      r[0] = r[1] = r[2] = r[3] = arg_none<A>();
    }
  } else {
    r[0] = f < F ? (int)row[f] : arg_none<A>();
  }
}

template <int W, typename A>
__device__ __forceinline__ void store_arg(A* __restrict__ row, int f, int F, const int (&r)[W]) {
  if constexpr (W == 4) {
    if (f < F) {
      if constexpr (sizeof(A) == 2) {
        uint2 t;
        t.x = (uint32_t)(r[0] & 0xFFFF) | ((uint32_t)r[1] << 16);
        t.y = (uint32_t)(r[2] & 0xFFFF) | ((uint32_t)r[3] << 16);
        *reinterpret_cast<uint2*>(row + f) = t;
      } else {
        *reinterpret_cast<int4*>(row + f) = make_int4(r[0], r[1], r[2], r[3]);
      }
    }
  } else {
    if (f < F) row[f] = (A)r[0];
  }
}

// ---- edge windows ---------------------------------------------------------------------
// A wave walks its item's entries in windows of 64: one coalesced vector load brings 64
// column ids (and per-entry scalars) into a VGPR, and each edge's id is broadcast with
// v_readlane (a uniform lane select), so no per-edge scalar-load round trip sits in front
// of the row loads. Inside a window, U edges are in flight at once: all their row loads
// are issued before any is consumed. The last batch of a window is padded by repeating
// its last valid edge for the loads; its compute is skipped by a uniform branch.
__device__ __forceinline__ int bcast(int v, int j) { return __builtin_amdgcn_readlane(v, j); }
__device__ __forceinline__ float bcastf(float v, int j) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), j));
}

#ifndef PG_EDGE_U
#define PG_EDGE_U 8  // edges in flight per wave for feature tiles of <= 8 values per lane
#endif
template <int W, int NC>
struct EdgeU {
  static constexpr int value = (NC * W <= 8) ? PG_EDGE_U : 4;
};

// ---- max forward ---------------------------------------------------------------------
constexpr int kPackWaveMax = 256;  // longest row grouped by one wave (forward chunk)

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// In-launch combine of split rows for the whole-row forward (MERGE; replaces
// max_merge_kernel's launch), the max backward's hand-off (max_bwd_pull_kernel): every piece
// stores its partial maxima and positions write-through (sc1), drains them and draws a
// ticket from its (row, feature tile) counter (zeroed by a clear launch ahead); the piece
// that draws the last ticket reads the row's slots with sc1 loads and takes the maximum in
// slot order with strict > (the earliest maximal edge wins, as in max_merge_kernel).
struct FwdMerge {
  int chunk;            // the schedule's chunk
  uint32_t* tickets;    // [n_slots x n_ftiles]
  uint32_t val_bytes;   // the slot regions (< 2 GiB each, checked on the host)
  uint32_t arg_bytes;
};

template <int W, int NC, bool HAS_W, typename A, typename T = float, bool MERGE = false>
__global__ __launch_bounds__(kBlock) void max_fwd_kernel(
    const int32_t* __restrict__ ptr, const int32_t* __restrict__ col,
    const int32_t* __restrict__ eslot, const float* __restrict__ ew,
    const int4* __restrict__ items, int n_items, const T* __restrict__ X, int64_t ldx, int F,
    T* __restrict__ out, int64_t ldo, A* __restrict__ arg, int64_t lda,
    float* __restrict__ ws_val, A* __restrict__ ws_arg, int64_t ldw, int n_ftiles, int ftile, int dead_none,
    FwdMerge fm = {}) {
  constexpr int U = EdgeU<W, NC>::value;
  float* const val_base = ws_val;
  A* const arg_base = ws_arg;
  int ft = 0, f0 = 0;
  // n_ftiles > 1: all feature tiles of F in one launch, block b -> (item block b / n_ftiles,
  // tile b % n_ftiles), so every tile's longest items start first
  int bx = blockIdx.x;
  if (n_ftiles > 1) {
    const int t = bx % n_ftiles;
    ft = t;
    bx /= n_ftiles;
    f0 = t * ftile;
    X += f0;
    out += f0;
    arg += f0;
    if (ws_val) ws_val += f0;
    if (ws_arg) ws_arg += f0;
    F = min(ftile, F - f0);
  }
  const int it = bx * kWavesPerBlock + wave_id_uniform();
  if (it >= n_items) return;
  const int4 item = items[it];
  const int row = item.x, k0 = item.y, k1 = item.z, slot = item.w;
  const int rs = ptr[row];
  const int lane = lane_id();
  const float ninf = -std::numeric_limits<float>::infinity();

  float best[NC][W];
  int bpos[NC][W];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < W; ++i) {
      best[c][i] = ninf;
      bpos[c][i] = arg_none<A>();
    }

  for (int kw = k0; kw < k1; kw += kWave) {
    const int nw = min(kWave, k1 - kw);
    const int kl = kw + min(lane, nw - 1);
    const int idxv = col[kl];
    float wv = 1.f;
    if constexpr (HAS_W) wv = ew[eslot ? eslot[kl] : kl];
    for (int j = 0; j < nw; j += U) {
      const int nv = min(U, nw - j);
      float v[U][NC][W];
#pragma unroll
      for (int e = 0; e < U; ++e) {
        const T* xr = X + (int64_t)bcast(idxv, j + min(e, nv - 1)) * ldx;
#pragma unroll
        for (int c = 0; c < NC; ++c) load_tile<W, T>(xr, (c * kWave + lane) * W, F, v[e][c], ninf);
      }
#pragma unroll
      for (int e = 0; e < U; ++e) {
        if (e < nv) {
          const int pos = kw + j + e - rs;
          float w = 1.f;
          if constexpr (HAS_W) w = bcastf(wv, j + e);
#pragma unroll
          for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int i = 0; i < W; ++i) {
              const float m = HAS_W ? v[e][c][i] * w : v[e][c][i];
              if (m > best[c][i]) {
                best[c][i] = m;
                bpos[c][i] = pos;
              }
            }
        }
      }
    }
  }

  if (slot < 0) {
    // whole row: finalise (+-inf -> 0, empty row -> 0 / none)
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < W; ++i)
        if (__builtin_isinf(best[c][i])) best[c][i] = 0.f;
    if (dead_none) {  // PG_ARG_DEAD_NONE: a zero maximum records no winner
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int i = 0; i < W; ++i)
          if (best[c][i] == 0.f) bpos[c][i] = arg_none<A>();
    }
    T* orow = out + (int64_t)row * ldo;
    A* arow = arg + (int64_t)row * lda;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int f = (c * kWave + lane) * W;
      store_tile<W, T>(orow, f, F, best[c]);
      store_arg<W, A>(arow, f, F, bpos[c]);
    }
  } else if constexpr (MERGE && W == 4) {
    const __amdgpu_buffer_rsrc_t rv = pg_x3::rsrc(val_base, fm.val_bytes);
    const __amdgpu_buffer_rsrc_t ra = pg_x3::rsrc(arg_base, fm.arg_bytes);
    auto voff = [&](int sl, int f) { return ((uint32_t)sl * (uint32_t)ldw + (uint32_t)(f0 + f)) * 4u; };
    auto aoff = [&](int sl, int f) { return ((uint32_t)sl * (uint32_t)ldw + (uint32_t)(f0 + f)) * (uint32_t)sizeof(A); };
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int f = (c * kWave + lane) * W;
      if (f < F) {
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(pg_u32x4, make_float4(best[c][0], best[c][1], best[c][2], best[c][3])), rv,
            voff(slot, f), 0, 16);
        if constexpr (sizeof(A) == 2) {
          const pg_u32x2 a2 = {(uint32_t)(bpos[c][0] & 0xFFFF) | ((uint32_t)bpos[c][1] << 16),
                               (uint32_t)(bpos[c][2] & 0xFFFF) | ((uint32_t)bpos[c][3] << 16)};
          __builtin_amdgcn_raw_buffer_store_b64(a2, ra, aoff(slot, f), 0, 16);
        } else {
          const pg_u32x4 a4 = {(uint32_t)bpos[c][0], (uint32_t)bpos[c][1], (uint32_t)bpos[c][2], (uint32_t)bpos[c][3]};
          __builtin_amdgcn_raw_buffer_store_b128(a4, ra, aoff(slot, f), 0, 16);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every payload store drained before the ticket
    const int re = ptr[row + 1];
    const int s0 = slot - (k0 - rs) / fm.chunk;
    const int ns = (re - rs + fm.chunk - 1) / fm.chunk;
    uint32_t ticket = 0;
    if (lane == 0)
      ticket = __hip_atomic_fetch_add((pg_gu32*)(fm.tickets + (int64_t)s0 * n_ftiles + ft), 1u, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
    ticket = __builtin_amdgcn_readfirstlane(ticket);
    if ((int)ticket != ns - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the ticket
    T* orow = out + (int64_t)row * ldo;
    A* arow = arg + (int64_t)row * lda;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int f = (c * kWave + lane) * W;
      float bv[4] = {ninf, ninf, ninf, ninf};
      int bp[4] = {arg_none<A>(), arg_none<A>(), arg_none<A>(), arg_none<A>()};
      // 4 slots in flight, positions kept packed: the tail stays inside the main loop's
      // registers (8 slots and unpacked positions took the kernel from 46 to 68 VGPRs and
      // one wave per SIMD less for every item)
      constexpr int kS = 4;
      using AV = std::conditional_t<sizeof(A) == 2, pg_u32x2, pg_u32x4>;
      for (int sb = s0; sb < s0 + ns; sb += kS) {
        float4 v[kS];
        AV a[kS];
#pragma unroll
        for (int e = 0; e < kS; ++e) {
          const int sl = min(sb + e, s0 + ns - 1);
          v[e] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rv, voff(sl, f), 0, 16));
          if constexpr (sizeof(A) == 2) a[e] = __builtin_amdgcn_raw_buffer_load_b64(ra, aoff(sl, f), 0, 16);
          else a[e] = __builtin_amdgcn_raw_buffer_load_b128(ra, aoff(sl, f), 0, 16);
        }
#pragma unroll
        for (int e = 0; e < kS; ++e)
          if (sb + e < s0 + ns) {
            const float ve[4] = {v[e].x, v[e].y, v[e].z, v[e].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              int ai;
              if constexpr (sizeof(A) == 2) ai = (int)((a[e][i >> 1] >> (16 * (i & 1))) & 0xFFFF);
              else ai = (int)a[e][i];
              if (ve[i] > bv[i]) {
                bv[i] = ve[i];
                bp[i] = ai;
              }
            }
          }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (__builtin_isinf(bv[i])) bv[i] = 0.f;
        if (dead_none && bv[i] == 0.f) bp[i] = arg_none<A>();
      }
      store_tile<4, T>(orow, f, F, bv);
      store_arg<4, A>(arow, f, F, bp);
    }
  } else {
    float* orow = ws_val + (int64_t)slot * ldw;
    A* arow = ws_arg + (int64_t)slot * ldw;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int f = (c * kWave + lane) * W;
      store_tile<W>(orow, f, F, best[c]);
      store_arg<W, A>(arow, f, F, bpos[c]);
    }
  }
}

// ---- max forward over XCD column slices ---------------------------------------------
// The feature columns are cut into slices of LPR * 4 columns; every workgroup of one XCD
// (blockIdx % 8 labels the XCD) works on the same slice, so the part of X that XCD gathers
// (N rows x one slice) is small enough to stay in its 4 MiB L2 instead of crossing the
// fabric to the Infinity Cache for every edge. A wave holds 64 / LPR items side by side
// (LPR lanes each; neighbouring items have similar lengths: the schedule is longest-first)
// and walks each item's edges in order, U row pieces in flight, so ties keep the first
// maximal edge exactly as max_fwd_kernel. Slice s of item block i: s = g + 8 * pass,
// i = blockIdx / 8 within the pass (n_slices >= 8), or the n_slices < 8 slices shared out
// over the eight XCD labels.
// Measured in the cfg2 step: 256-B slices take F = 256 from 96 to 82 us and F = 504 from
// 184 to 156 us (about 16 TB/s of gathered row bytes, close to the 17-19 TB/s the
// microarchitecture guide measures for gathers served by L2); 128-B slices, whose part of X
// fits an L2 whole, are no faster; on cfg5's 384 656-row bf16 graph slicing loses (8.1 ->
// 12.1 ms per step), hence the size gate. The XCD mapping is what pays: the same kernel
// with each slice spread over all XCDs (-DPG_FWD_SLICE_NOXCD) takes 113 us at F = 256.
#ifndef PG_FWD_SLICE
#define PG_FWD_SLICE 256  // bytes of a row per slice (0: whole-row tiles only)
#endif
#ifndef PG_FWD_SLICE_NO_WIDE
#define PG_FWD_SLICE_NO_WIDE 0  // variant builds: 1 keeps widths that need wider slices on whole rows
#endif
#ifndef PG_SLICE_U_FIXED
#define PG_SLICE_U_FIXED 0  // variant builds: 8 keeps 8 pieces in flight for every slice count
#endif
#ifndef PG_FWD_SLICE_MAXTAB
#define PG_FWD_SLICE_MAXTAB (32ll << 20)  // largest slice of X (rows x slice bytes) sliced
#endif
// (slice, item block) of workgroup b over n_iblk item blocks, XCD-affine (see above)
__device__ __forceinline__ void slice_of_block(int b, int n_slices, int n_iblk, int& slice, int& iblk) {
#ifdef PG_FWD_SLICE_NOXCD  // probe builds: slice-major order, each slice spread over the XCDs
  slice = b / n_iblk;
  iblk = b % n_iblk;
#else
  const int g = b % 8, v = b / 8;
  if (n_slices >= 8) {
    slice = g + 8 * (v / n_iblk);
    iblk = v % n_iblk;
  } else {
    const int rep = 8 / n_slices;
    slice = g % n_slices;
    iblk = v * rep + g / n_slices;
  }
#endif
}

// One lane group's running maximum over `len` edges from in-CSR slot k0 (positions
// relative to rs), LPR edges' ids per load, UE row pieces in flight. (A macro, not a
// function: passed by reference the running maxima took 109-126 registers against 72-75
// written out in the kernel.) It reads the enclosing kernel's `lane`, `col`, `eslot`, `ew`,
// `X`, `ldx`, `f`, `F`, `ninf` and updates its `best[4]` / `bpos[4]`.
#define PG_SLICE_RUN(LPR, UE, HAS_W, T, k0_, len_, rs_)                                              \
  do {                                                                                               \
    constexpr int U_ = (UE) < (LPR) ? (UE) : (LPR);                                                  \
    static_assert((LPR) <= 32 && (LPR) % U_ == 0, "slice lanes");                                    \
    const int sk0 = (k0_), slen = (len_), srs = (rs_);                                               \
    const int q_ = lane % (LPR);                                                                     \
    const int gbase = 4 * (lane - q_);                                                               \
    for (int j = 0; j < slen; j += (LPR)) {                                                          \
      const int kq = sk0 + j + min(q_, slen - j - 1);                                                \
      const int idv = col[kq];                                                                       \
      float wv = 1.f;                                                                                \
      if constexpr (HAS_W) wv = ew[eslot ? eslot[kq] : kq];                                          \
      _Pragma("unroll") for (int e0 = 0; e0 < (LPR); e0 += U_) {                                     \
        if (j + e0 >= slen) break;                                                                   \
        float x[U_][4];                                                                              \
        _Pragma("unroll") for (int e = 0; e < U_; ++e) {                                             \
          const int id = __builtin_amdgcn_ds_bpermute(gbase + 4 * (e0 + e), idv);                    \
          load_tile<4, T>(X + (int64_t)id * ldx, f, F, x[e], ninf);                                  \
        }                                                                                            \
        _Pragma("unroll") for (int e = 0; e < U_; ++e) {                                             \
          if (j + e0 + e < slen) {                                                                   \
            const int pos = sk0 + j + e0 + e - srs;                                                  \
            float w = 1.f;                                                                           \
            if constexpr (HAS_W)                                                                     \
              w = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(gbase + 4 * (e0 + e),       \
                                                                          __builtin_bit_cast(int, wv))); \
            _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                          \
              const float m = HAS_W ? x[e][i] * w : x[e][i];                                         \
              if (m > best[i]) {                                                                     \
                best[i] = m;                                                                         \
                bpos[i] = pos;                                                                       \
              }                                                                                      \
            }                                                                                        \
          }                                                                                          \
        }                                                                                            \
      }                                                                                              \
    }                                                                                                \
  } while (0)

template <int LPR, typename A, typename T>
__device__ __forceinline__ void slice_store(T* __restrict__ out, int64_t ldo, A* __restrict__ arg, int64_t lda,
                                            int row, int f, int F, float (&best)[4], int (&bpos)[4],
                                            int dead_none) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (__builtin_isinf(best[i])) best[i] = 0.f;
    if (dead_none && best[i] == 0.f) bpos[i] = arg_none<A>();
  }
  store_tile<4, T>(out + (int64_t)row * ldo, f, F, best);
  store_arg<4, A>(arg + (int64_t)row * lda, f, F, bpos);
}

// Rows longer than the schedule's chunk (its split rows, `merges`, longest first) take the
// first hub_grid workgroups of the launch, one workgroup per (row, slice): its lane groups
// take contiguous runs of the row's edges, in order, and combine their maxima through LDS
// in run order (strict >: the earliest maximal edge wins, as in one sequential pass), so
// no partial slots and no merge launch. The other workgroups take the schedule's items and
// skip its pieces of those rows. (As a launch of its own before the other rows, the split
// rows' tail ran alone: 0.350 vs 0.301 ms per cfg2 step.)
template <int LPR, int UE, bool HAS_W, typename A, typename T = float>
__global__ __launch_bounds__(kBlock) void max_fwd_slice_kernel(
    const int32_t* __restrict__ ptr, const int32_t* __restrict__ col,
    const int32_t* __restrict__ eslot, const float* __restrict__ ew,
    const int4* __restrict__ items, int n_items, const int4* __restrict__ hubs, int n_hub, int hub_grid,
    const T* __restrict__ X, int64_t ldx, int F, T* __restrict__ out, int64_t ldo, A* __restrict__ arg,
    int64_t lda, int n_slices, int n_iblk, int dead_none) {
  constexpr int RPW = kWave / LPR;
  constexpr int CS = LPR * 4;
  constexpr int NG = RPW * kWavesPerBlock;  // lane groups per workgroup
  __shared__ float hv[NG][CS];
  __shared__ int hp[NG][CS];
  const int lane = lane_id();
  const float ninf = -std::numeric_limits<float>::infinity();
  float best[4] = {ninf, ninf, ninf, ninf};
  int bpos[4] = {arg_none<A>(), arg_none<A>(), arg_none<A>(), arg_none<A>()};
  int b = blockIdx.x;
  int slice, iblk;
  if (b < hub_grid) {
    // a split row, whole: the workgroup's lane groups take contiguous runs of its edges
    slice_of_block(b, n_slices, n_hub, slice, iblk);
    if (slice >= n_slices || iblk >= n_hub) return;  // uniform over the workgroup
    const int row = hubs[iblk].x;
    const int rs = ptr[row], deg = ptr[row + 1] - rs;
    const int grp = wave_id_uniform() * RPW + lane / LPR;
    const int run = (deg + NG - 1) / NG;
    const int k0 = min(deg, grp * run);
    const int len = min(deg, k0 + run) - k0;
    const int c = (lane % LPR) * 4;
    const int f = slice * CS + c;
    PG_SLICE_RUN(LPR, UE, HAS_W, T, rs + k0, len, rs);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      hv[grp][c + i] = best[i];
      hp[grp][c + i] = bpos[i];
    }
    __syncthreads();
    if (grp == 0) {
      for (int r = 1; r < NG; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (hv[r][c + i] > best[i]) {
            best[i] = hv[r][c + i];
            bpos[i] = hp[r][c + i];
          }
      slice_store<LPR, A, T>(out, ldo, arg, lda, row, f, F, best, bpos, dead_none);
    }
    return;
  }
  slice_of_block(b - hub_grid, n_slices, n_iblk, slice, iblk);
  if (slice >= n_slices || iblk >= n_iblk) return;
  const int it = (iblk * kWavesPerBlock + wave_id_uniform()) * RPW + lane / LPR;
  if (it >= n_items) return;
  const int4 item = items[it];
  if (item.w >= 0) return;  // a piece of a split row: taken whole above
  const int row = item.x;
  const int f = slice * CS + (lane % LPR) * 4;
  PG_SLICE_RUN(LPR, UE, HAS_W, T, item.y, item.z - item.y, ptr[row]);
  slice_store<LPR, A, T>(out, ldo, arg, lda, row, f, F, best, bpos, dead_none);
}

// Combine the partial maxima of split rows in chunk order (earlier chunk wins ties).
// One workgroup per split row, one thread per feature; slot loads batched.
template <typename A, typename T = float>
__global__ __launch_bounds__(kBlock) void max_merge_kernel(const int4* __restrict__ merges,
                                                           int n_merges, int F,
                                                           const float* __restrict__ ws_val,
                                                           const A* __restrict__ ws_arg,
                                                           int64_t ldw, T* __restrict__ out,
                                                           int64_t ldo, A* __restrict__ arg,
                                                           int64_t lda, int dead_none) {
  const int4 m = merges[blockIdx.x];
  const int row = m.x, s0 = m.y, ns = m.z;
  for (int f = threadIdx.x; f < F; f += kBlock) {
    float best = -std::numeric_limits<float>::infinity();
    int bp = arg_none<A>();
    for (int s = s0; s < s0 + ns; s += 8) {
      float v[8];
      int a[8];  // loaded with the values: no dependent load behind each compare
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int64_t o = (int64_t)min(s + e, s0 + ns - 1) * ldw + f;
        v[e] = ws_val[o];
        a[e] = (int)ws_arg[o];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (s + e < s0 + ns && v[e] > best) {
          best = v[e];
          bp = a[e];
        }
    }
    if (__builtin_isinf(best)) best = 0.f;
    if (dead_none && best == 0.f) bp = arg_none<A>();
    out[(int64_t)row * ldo + f] = from_f<T>(best);
    arg[(int64_t)row * lda + f] = (A)bp;
  }
}

// ---- max backward, deterministic gather over the transposed CSR ----------------------
// Wave per source row u: for every out-edge (u -> v) at in-row position p (ascending v),
// read v's argmax record; features whose winner is p take dout[v, f] (* w). The record
// loads of U edges are issued together, then their dout loads together (lanes with no
// match read row 0 at the same column instead of branching: a cache hit, no divergence).
template <int W, int NC, bool HAS_W, typename A>
__global__ __launch_bounds__(kBlock) void max_bwd_kernel(
    const float* __restrict__ ew, const int32_t* __restrict__ tcol,
    const int32_t* __restrict__ tslot, const int32_t* __restrict__ tpos,
    const int4* __restrict__ items, int n_items, const A* __restrict__ arg, int64_t lda,
    const float* __restrict__ dout, int64_t ldd, int F, const float* __restrict__ mask,
    int64_t ldm, float* __restrict__ dx, int64_t ldx, float* __restrict__ ws, int64_t ldw) {
  constexpr int U = EdgeU<W, NC>::value;
  const int it = blockIdx.x * kWavesPerBlock + wave_id_uniform();
  if (it >= n_items) return;
  const int4 item = items[it];
  const int row = item.x, t0 = item.y, t1 = item.z, slot = item.w;
  const int lane = lane_id();

  float acc[NC][W];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < W; ++i) acc[c][i] = 0.f;

  for (int tw = t0; tw < t1; tw += kWave) {
    const int nw = min(kWave, t1 - tw);
    const int tl = tw + min(lane, nw - 1);
    const int vv = tcol[tl];
    const int pv = tpos[tl];
    float wv = 1.f;
    if constexpr (HAS_W) wv = ew[tslot[tl]];
    for (int j = 0; j < nw; j += U) {
      const int nv = min(U, nw - j);
      int a[U][NC][W];
#pragma unroll
      for (int e = 0; e < U; ++e) {
        const A* ar = arg + (int64_t)bcast(vv, j + min(e, nv - 1)) * lda;
#pragma unroll
        for (int c = 0; c < NC; ++c) load_arg<W, A>(ar, (c * kWave + lane) * W, F, a[e][c]);
      }
      float d[U][NC][W];
#pragma unroll
      for (int e = 0; e < U; ++e) {
        const int je = j + min(e, nv - 1);
        const int p = bcast(pv, je);
        const float* dr = dout + (int64_t)bcast(vv, je) * ldd;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          bool any = false;
#pragma unroll
          for (int i = 0; i < W; ++i) any |= (a[e][c][i] == p);
          load_tile<W>(any ? dr : dout, (c * kWave + lane) * W, F, d[e][c], 0.f);
        }
      }
#pragma unroll
      for (int e = 0; e < U; ++e) {
        if (e < nv) {
          const int p = bcast(pv, j + e);
          float w = 1.f;
          if constexpr (HAS_W) w = bcastf(wv, j + e);
#pragma unroll
          for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int i = 0; i < W; ++i)
              if (a[e][c][i] == p) acc[c][i] += HAS_W ? w * d[e][c][i] : d[e][c][i];
        }
      }
    }
  }

  if (slot < 0) {
    float* xr = dx + (int64_t)row * ldx;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int f = (c * kWave + lane) * W;
      if (mask) {
        float mk[W];
        load_tile<W>(mask + (int64_t)row * ldm, f, F, mk, 0.f);
#pragma unroll
        for (int i = 0; i < W; ++i)
          if (!(mk[i] > 0.f)) acc[c][i] = 0.f;
      }
      store_tile<W>(xr, f, F, acc[c]);
    }
  } else {
    float* wr = ws + (int64_t)slot * ldw;
#pragma unroll
    for (int c = 0; c < NC; ++c) store_tile<W>(wr, (c * kWave + lane) * W, F, acc[c]);
  }
}

// ---- max backward, grouped form (default for u16 records and F <= 1024) ---------------
// Pass 1 (pack), per destination row v: group v's live entries (v, f) by their winning
// in-row position p, giving
//   rec[v F + i]    = {w * dout[v,f], f}, grouped by p (any order inside a group; 8-B
//                     records, or 4-B {bf16 dout, f} for bf16 storage without weights),
//   glist[s]        = start_p | count_p << 16 for the edge at in-CSR slot s = ptr[v] + p:
//                     4 B, the start relative to the row's run v F (a row's descriptors are
//                     contiguous: coalesced stores).
// Rows of in-degree <= kPackWaveMax: one wave per row (wave-private LDS histogram, wave
// scan, LDS-atomic placement); longer rows: one workgroup per row (block histogram, or a
// bitonic sort of (p << 16 | f) keys past kHistMax entries).
// Pass 2 (pull), one wave per source row item: for each out-edge of u, ascending
// destination v (the transposed CSR order), read its descriptor glist[tslot[t]] and add
// its records into an LDS row accumulator (max_bwd_pull_kernel). Traffic per edge: its
// 4-B slot and destination (coalesced), one 4-B descriptor (random; 8 B {v F + start,
// count} before: twice the footprint for the caches to hold) and one short contiguous run
// of records (~F/deg entries).
// Transposed descriptors (round 5; when the caller gives the in-CSR slots' transposed
// indices, g->epos): the descriptor of slot s is stored at its transposed index einv[s],
// and only for edges that win something (about half win nothing: their descriptors stay
// the zero the launch clears the array to). The pull then reads its out-edges' descriptors
// in order, coalesced, and fetches lists only for the edges that have one: one random
// access per live edge instead of two per edge. (Round 3 stored every descriptor at the
// transposed index, empty ones included: pull 35.6 vs 43.5 us, pack 28.3 vs 15.9 us at
// F = 256, no gain. A source-ordered record layout, DESIGN.md §7, measured slower still.)
constexpr int kHistMax = 4096;
constexpr int kGroupMaxF = 1024;  // (starts and counts <= F fit the descriptor's 16-bit halves)

__device__ __forceinline__ uint32_t desc_make(int start, int count) {
  return (uint32_t)start | ((uint32_t)count << 16);
}

// Where the pack puts a descriptor: at the in-CSR slot (TR = false), or at the slot's
// transposed index when the list is not empty (TR = true; the array was cleared first).
template <bool TR>
struct DescOut {
  uint32_t* glist;
  const int32_t* einv;
  // the transposed index of slot s, loaded ahead of the write (TR only)
  __device__ __forceinline__ int pre(int s) const {
    if constexpr (TR) return einv[s];
    else return s;
  }
  __device__ __forceinline__ void put(int pre_s, int start, int count) const {
    if constexpr (TR) {
      if (count > 0) glist[pre_s] = desc_make(start, count);
    } else {
      glist[pre_s] = desc_make(start, count);
    }
  }
};
#ifndef PG_BWD_TRANS
#define PG_BWD_TRANS 1  // variant builds: 0 keeps the descriptors at the in-CSR slots
#endif
#ifndef PG_BWD_DIRECT
#define PG_BWD_DIRECT 0
#endif

// one record per list entry, one contiguous run per list (one line for the pull to fetch
// where two arrays cost two). GPack: {value f32, feature u32} (8 B); the value carries the
// edge weight already (w * dout[v,f], the product the pull formed before). GPack4 (bf16
// storage without edge weights): the bf16 upstream gradient itself and the feature,
// {value bf16, feature u16} (4 B); exact, since the value is a bf16 number.
struct GPack {
  using W = uint2;
  W* __restrict__ r;
  __device__ static __forceinline__ W make(int f, float d) { return make_uint2(__float_as_uint(d), (uint32_t)f); }
  __device__ __forceinline__ void put(int64_t pos, int f, float d) const { r[pos] = make(f, d); }
  __device__ __forceinline__ void get(int64_t pos, int& f, float& d) const {
    const W x = r[pos];
    d = __uint_as_float(x.x);
    f = (int)x.y;
  }
};
struct GPack4 {
  using W = uint32_t;
  W* __restrict__ r;
  __device__ static __forceinline__ W make(int f, float d) {
    return (__float_as_uint(d) & 0xFFFF0000u) | (uint32_t)f;
  }
  __device__ __forceinline__ void put(int64_t pos, int f, float d) const { r[pos] = make(f, d); }
  __device__ __forceinline__ void get(int64_t pos, int& f, float& d) const {
    const W x = r[pos];
    d = __uint_as_float(x & 0xFFFF0000u);
    f = (int)(x & 0xFFFFu);
  }
};

#ifndef PG_SCAN_DPP
#define PG_SCAN_DPP 1
#endif
// inclusive prefix sum over the 64 lanes: DPP row shifts, then row broadcasts 15 and 31
// (six VALU ops; the __shfl_up form is six dependent ds_bpermute round trips)
__device__ __forceinline__ int wave_incl_add(int x) {
#if PG_SCAN_DPP
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
#else
  const int lane = (int)(threadIdx.x & 63);
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  return x;
#endif
}

__device__ int block_exclusive_scan(int* s, int n, int* wsum) {
  const int per = (n + kBlock - 1) / kBlock;
  const int b = threadIdx.x * per;
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  int local = 0;
  for (int i = 0; i < per; ++i)
    if (b + i < n) local += s[b + i];
  int x = local;
  x = wave_incl_add(x);
  if (lane == kWave - 1) wsum[wave] = x;
  __syncthreads();
  int pre = 0;
  for (int w = 0; w < wave; ++w) pre += wsum[w];
  int run = pre + x - local;
  for (int i = 0; i < per; ++i)
    if (b + i < n) {
      const int t = s[b + i];
      s[b + i] = run;
      run += t;
    }
  const int total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  return total;
}

template <typename A, typename T, typename R, typename D>
__device__ __forceinline__ void pack_short_row(
    int v, int wave, const int32_t* __restrict__ ptr,
    const A* __restrict__ arg, int64_t lda, int F, const T* __restrict__ dout, int64_t ldd,
    const T* __restrict__ fout, int64_t ldf, const float* __restrict__ ew, R gp, D dsc,
    int* __restrict__ lds) {
  constexpr int MAXW = kGroupMaxF / kWave;  // features per lane
  const int lane = lane_id();
  // every independent load first: the row bounds, the argmax record and the upstream
  // gradient (each lane its own features, coalesced), then the list descriptors' slots
  const int rs = ptr[v];
  const int re = ptr[v + 1];
  const A* ar = arg + (int64_t)v * lda;
  const T* dr = dout + (int64_t)v * ldd;
  int a[MAXW];
  float d[MAXW];
#pragma unroll
  for (int i = 0; i < MAXW; ++i) {
    const int f = lane + i * kWave;
    a[i] = f < F ? (int)ar[f] : arg_none<A>();
    d[i] = f < F ? to_f(dr[f]) : 0.f;
  }
  if (fout) {  // a zero maximum: its winner's relu mask is 0, the entry contributes nothing
    const T* fr = fout + (int64_t)v * ldf;
    float m[MAXW];
#pragma unroll
    for (int i = 0; i < MAXW; ++i) m[i] = to_f(fr[min(lane + i * kWave, F - 1)]);
#pragma unroll
    for (int i = 0; i < MAXW; ++i)
      if (m[i] == 0.f) a[i] = arg_none<A>();
  }
  const int deg = re - rs;
  if (deg > kPackWaveMax || deg == 0) return;
  const int B = (deg + kWave - 1) / kWave;  // bins per lane, <= 4
  int ei[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = lane * B + q;
    ei[q] = dsc.pre((q < B && p < deg) ? rs + p : rs);
  }
  int* hist = lds + wave * (kPackWaveMax + 4);
  for (int p = lane; p < deg; p += kWave) hist[p] = 0;
  wave_lds_sync();
#pragma unroll
  for (int i = 0; i < MAXW; ++i)
    if (a[i] != arg_none<A>()) atomicAdd(&hist[a[i]], 1);
  wave_lds_sync();
  // exclusive scan over the deg bins: lane owns bins [lane B, lane B + B)
  int c[4], local = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = lane * B + q;
    c[q] = (q < B && p < deg) ? hist[p] : 0;
    local += c[q];
  }
  int x = local;
  x = wave_incl_add(x);
  int run = x - local;
  const int vF = v * F;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = lane * B + q;
    if (q < B && p < deg) {
      hist[p] = run;
      dsc.put(ei[q], run, c[q]);
      run += c[q];
    }
  }
  wave_lds_sync();
  // placement: every winner straight to its list slot (the order inside a list is free)
#pragma unroll
  for (int i = 0; i < MAXW; ++i)
    if (a[i] != arg_none<A>()) {
      const int pos = vF + atomicAdd(&hist[a[i]], 1);
      gp.put(pos, lane + i * kWave, ew ? ew[rs + a[i]] * d[i] : d[i]);
    }
}

// The same for F <= 256 NV with rows of 4-aligned features: lane l owns the features
// 256 c + 4 l + i (c < NV, i < 4), loaded 4 at a time (argmax records 8 B, upstream
// gradient and forward output 16 B or 8 B), and one LDS atomic per live feature both
// counts its winning position and ranks it inside that position's list (the order inside
// a list is free); the list offsets come from one wave scan over the positions. The lists
// are assembled in LDS and copied out with coalesced stores (scattered 2-B global stores
// are read-modify-writes of partial lines): -6 % for the whole backward on cfg2.
template <int NV>
constexpr int pack_wave_ints() { return kPackWaveMax + 4 + NV * 512; }  // hist | records (8 B)

template <int NV, typename A, typename T, typename R, typename D>
__device__ __forceinline__ void pack_short_row_v(
    int v, int wave, const int32_t* __restrict__ ptr,
    const A* __restrict__ arg, int64_t lda, int F, const T* __restrict__ dout, int64_t ldd,
    const T* __restrict__ fout, int64_t ldf, const float* __restrict__ ew, R gp, D dsc,
    int* __restrict__ lds) {
  const int lane = lane_id();
  const int rs = ptr[v];
  const int deg = ptr[v + 1] - rs;
  if (deg > kPackWaveMax || deg == 0) return;
  int a[NV][4];
  float d[NV][4];
  // straight-line loads at clamped columns (F % 4 == 0 here), masked afterwards: no branch
  // between the record and gradient loads, so both are in flight before the first wait
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int f = (c * kWave + lane) * 4;
    const int fc = min(f, F - 4);
    int ac[4];
    float dc[4];
    load_arg<4, A>(arg + (int64_t)v * lda, fc, F, ac);
    load_tile<4, T>(dout + (int64_t)v * ldd, fc, F, dc, 0.f);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[c][i] = f < F ? ac[i] : arg_none<A>();
      d[c][i] = f < F ? dc[i] : 0.f;
    }
  }
  if (fout) {  // a zero maximum: its winner's relu mask is 0, the entry contributes nothing
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      float m[4];
      load_tile<4, T>(fout + (int64_t)v * ldf, (c * kWave + lane) * 4, F, m, 1.f);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (m[i] == 0.f) a[c][i] = arg_none<A>();
    }
  }
  const int B = (deg + kWave - 1) / kWave;  // bins per lane, <= 4
  int ei[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = lane * B + q;
    ei[q] = dsc.pre((q < B && p < deg) ? rs + p : rs);
  }
  int* hist = lds + wave * pack_wave_ints<NV>();
  typename R::W* lr = reinterpret_cast<typename R::W*>(hist + kPackWaveMax + 4);  // 16-B aligned: 260 ints
  for (int p = lane; p < deg; p += kWave) hist[p] = 0;
  wave_lds_sync();
  int rank[NV][4];
#pragma unroll
  for (int c = 0; c < NV; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      rank[c][i] = a[c][i] != arg_none<A>() ? atomicAdd(&hist[a[c][i]], 1) : 0;
  wave_lds_sync();
  int cq[4], local = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = lane * B + q;
    cq[q] = (q < B && p < deg) ? hist[p] : 0;
    local += cq[q];
  }
  int x = local;
  x = wave_incl_add(x);
  int run = x - local;
  const int vF = v * F;
  wave_lds_sync();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = lane * B + q;
    if (q < B && p < deg) {
      hist[p] = run;
      dsc.put(ei[q], run, cq[q]);
      run += cq[q];
    }
  }
  wave_lds_sync();
  if (ew) {  // the edge weight folded into the value: w * d, the product the pull formed
#pragma unroll
    for (int c = 0; c < NV; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) d[c][i] = ew[rs + (a[c][i] != arg_none<A>() ? a[c][i] : 0)] * d[c][i];
  }
#pragma unroll
  for (int c = 0; c < NV; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (a[c][i] != arg_none<A>()) {
        const int pos = hist[a[c][i]] + rank[c][i];
        lr[pos] = R::make((c * kWave + lane) * 4 + i, d[c][i]);
      }
  wave_lds_sync();
  const int total = __builtin_amdgcn_readlane(x, kWave - 1);
  // 16-B stores of 2 (8-B) or 4 (4-B) records per lane (vF and the LDS image are 16-B
  // aligned: F % 4 == 0)
  constexpr int RP = 16 / sizeof(typename R::W);
  for (int i = lane * RP; i < total; i += RP * kWave) {
    if (i + RP <= total) {
      *reinterpret_cast<uint4*>(gp.r + vF + i) = *reinterpret_cast<const uint4*>(lr + i);
    } else {
      for (int k = i; k < total; ++k) gp.r[vF + k] = lr[k];
    }
  }
}

template <typename A, typename T, typename R, typename D>
__device__ __forceinline__ void pack_long_row(
    int v, const int32_t* __restrict__ ptr,
    const A* __restrict__ arg, int64_t lda, int F, const T* __restrict__ dout, int64_t ldd,
    const T* __restrict__ fout, int64_t ldf, const float* __restrict__ ew, R gp, D dsc,
    int* __restrict__ lds) {
  int* hist = lds;
  uint16_t* feats = reinterpret_cast<uint16_t*>(lds + kHistMax + 8);
  int* wsum = lds + kHistMax + 8 + kGroupMaxF / 2;
  const int rs = ptr[v];
  const int deg = ptr[v + 1] - rs;
  if (deg <= kPackWaveMax) return;
  const A* ar = arg + (int64_t)v * lda;
  const int64_t vF = (int64_t)v * F;
  int total;
  if (deg <= kHistMax) {
    // independent loads first (each thread its own features), placement straight to the
    // list slots as in the wave form
    constexpr int FPT = kGroupMaxF / kBlock;
    const T* dr = dout + (int64_t)v * ldd;
    int a[FPT];
    float d[FPT];
#pragma unroll
    for (int i = 0; i < FPT; ++i) {
      const int f = threadIdx.x + i * kBlock;
      a[i] = f < F ? (int)ar[f] : arg_none<A>();
      d[i] = f < F ? to_f(dr[f]) : 0.f;
    }
    if (fout) {  // zero maxima contribute nothing (their winner's relu mask is 0)
      const T* fr = fout + (int64_t)v * ldf;
      float m[FPT];
#pragma unroll
      for (int i = 0; i < FPT; ++i) m[i] = to_f(fr[min((int)threadIdx.x + i * kBlock, F - 1)]);
#pragma unroll
      for (int i = 0; i < FPT; ++i)
        if (m[i] == 0.f) a[i] = arg_none<A>();
    }
    for (int p = threadIdx.x; p < deg; p += kBlock) hist[p] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FPT; ++i)
      if (a[i] != arg_none<A>()) atomicAdd(&hist[a[i]], 1);
    __syncthreads();
    total = block_exclusive_scan(hist, deg, wsum);
    for (int p0 = threadIdx.x; p0 < deg; p0 += 4 * kBlock) {
      int e[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = p0 + j * kBlock;
        e[j] = dsc.pre(p < deg ? rs + p : rs);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = p0 + j * kBlock;
        if (p < deg) {
          const int st = hist[p];
          const int en = p + 1 < deg ? hist[p + 1] : total;
          dsc.put(e[j], st, en - st);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FPT; ++i)
      if (a[i] != arg_none<A>()) {
        const int64_t pos = vF + atomicAdd(&hist[a[i]], 1);
        gp.put(pos, threadIdx.x + i * kBlock, ew ? ew[rs + a[i]] * d[i] : d[i]);
      }
    return;
  } else {
    // hub row: bitonic sort of (p << 16 | f) keys; "none" sorts last
    uint32_t* keys = reinterpret_cast<uint32_t*>(hist);
    int np = 1;
    while (np < F) np <<= 1;
    for (int i = threadIdx.x; i < np; i += kBlock) {
      uint32_t key = 0xFFFFFFFFu;
      if (i < F) {
        const int a = (int)ar[i];
        const bool live = !fout || to_f(fout[(int64_t)v * ldf + i]) != 0.f;
        if (a != arg_none<A>() && live) key = ((uint32_t)a << 16) | (uint32_t)i;
      }
      keys[i] = key;
    }
    __syncthreads();
    for (int k = 2; k <= np; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = threadIdx.x; i < np; i += kBlock) {
          const int ixj = i ^ j;
          if (ixj > i) {
            const uint32_t a = keys[i], b = keys[ixj];
            if ((a > b) == ((i & k) == 0)) {
              keys[i] = b;
              keys[ixj] = a;
            }
          }
        }
        __syncthreads();
      }
    auto lower = [&](uint32_t key) {
      int lo = 0, hi = np;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[mid] < key) lo = mid + 1; else hi = mid;
      }
      return lo;
    };
    for (int p = threadIdx.x; p < deg; p += kBlock) {
      const int es = dsc.pre(rs + p);
      const int st = lower((uint32_t)p << 16);
      const int en = lower((uint32_t)(p + 1) << 16);
      dsc.put(es, st, en - st);
    }
    if (threadIdx.x == 0) wsum[0] = lower(0xFFFFFFFFu);
    __syncthreads();
    total = wsum[0];
    for (int i = threadIdx.x; i < total; i += kBlock) feats[i] = (uint16_t)(keys[i] & 0xFFFFu);
    __syncthreads();
  }
  const T* dr = dout + (int64_t)v * ldd;
  for (int i = threadIdx.x; i < total; i += kBlock) {
    const int f = feats[i];
    const float dv = to_f(dr[f]);
    gp.put(vF + i, f, ew ? ew[rs + (int)(reinterpret_cast<const uint32_t*>(hist)[i] >> 16)] * dv : dv);
  }
}

// One launch for both: blocks [0, n_long) take the rows past kPackWaveMax (`rows` lists
// them, as {row, ...} int4 = the split-row merges of a schedule whose chunk is <=
// kPackWaveMax; NULL = every row, short ones exit at once) so the long rows start first;
// the remaining blocks take 4 rows each, one wave per row.
constexpr int kPackLds = kHistMax + 8 + kGroupMaxF / 2 + 4;
static_assert(kPackLds >= kWavesPerBlock * (kPackWaveMax + 4), "pack LDS");

template <typename A, typename T, int NV, typename R, bool TR>
__global__ __launch_bounds__(kBlock) void group_pack_kernel(
    const int4* __restrict__ rows, int n_long, int n_rows, const int32_t* __restrict__ ptr,
    const A* __restrict__ arg, int64_t lda, int F,
    const T* __restrict__ dout, int64_t ldd, const T* __restrict__ fout, int64_t ldf,
    const float* __restrict__ ew, R gp, uint32_t* __restrict__ glist, const int32_t* __restrict__ einv,
    uint32_t* __restrict__ tickets, int n_tickets) {
  // the pull's split-row ticket counters start every call at zero (this launch precedes it)
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < n_tickets; i += gridDim.x * kBlock) tickets[i] = 0u;
  const DescOut<TR> dsc{glist, einv};
  constexpr int kLds = NV > 0 && kWavesPerBlock * pack_wave_ints<NV>() > kPackLds
                           ? kWavesPerBlock * pack_wave_ints<NV>() : kPackLds;
  __shared__ __attribute__((aligned(16))) int lds[kLds];
  const int b = blockIdx.x;
  if (b < n_long) {
    pack_long_row<A, T, R>(rows ? rows[b].x : b, ptr, arg, lda, F, dout, ldd, fout, ldf, ew, gp, dsc, lds);
  } else {
    const int wave = wave_id_uniform();
    const int v = (b - n_long) * kWavesPerBlock + wave;
    if (v < n_rows)
    {
      if constexpr (NV > 0)
        pack_short_row_v<NV, A, T, R>(v, wave, ptr, arg, lda, F, dout, ldd, fout, ldf, ew, gp, dsc, lds);
      else
        pack_short_row<A, T, R>(v, wave, ptr, arg, lda, F, dout, ldd, fout, ldf, ew, gp, dsc, lds);
    }
  }
}

#ifndef PG_FWD_MERGE
#define PG_FWD_MERGE 1  // split rows combined inside the whole-row forward (0: the max_merge_kernel launch)
#endif

#ifndef PG_PULL_MERGE
#define PG_PULL_MERGE 1  // split rows combined inside the pull (0: the sum_merge_kernel launch)
#endif

#ifndef PG_PULL_U
#define PG_PULL_U 8  // list segments in flight per wave (4-8 best on S0, 16 +6 %, 32 +25 %)
#endif

// Pass 2 (pull): one wave per source-row item {u, t0, t1, slot}, its out-edges in windows
// of 64 (ascending destination); lane j holds window edge j's descriptor (loaded through its
// in-CSR slot tslot[t]: the descriptors one window ahead, the slots two). The records of
// each list are added into an LDS row accumulator. A list never repeats a feature, so the
// lanes of one segment add into distinct words, and every feature's terms are summed in
// ascending v, the order of the sequential scatter_add_ (bit-exact on rows that are not
// split across items). Dense segments across several lists, added in order by LDS
// compare-and-swap (the float LDS atomic, ds_add_f32, runs at 1/16 of the integer atomics'
// rate on gfx950: scripts/probes/lds_rmw_probe.hip), measured slower on the engine's data:
// a source that wins a feature at many destinations puts it many times into one segment,
// and the swaps serialise.
// In-launch combine of split rows (MERGE; replaces sum_merge_kernel's launch): the pieces of a
// row longer than the schedule's chunk store their partial rows write-through (sc1), drain
// them, and draw a ticket from the row's counter (one per first slot, zeroed by the pack);
// the piece that draws the last ticket reads every slot of the row with sc1 loads (no stale
// L1 or other-XCD L2 line can serve them, so no acquire fence) and sums them in slot order
// from +0, exactly sum_merge_kernel's order: the same bits whichever piece arrives last.
struct PullMerge {
  const int32_t* ptr;  // the transposed CSR's row pointers (piece index = (t0 - ptr[row]) / chunk)
  int chunk;           // the schedule's chunk (pg_schedule_build)
  uint32_t* tickets;   // [n_slots]
  uint32_t ws_bytes;   // the slot region (< 2 GiB, checked on the host)
};


template <typename T, typename R, bool TR, bool MERGE>
__global__ __launch_bounds__(kBlock) void max_bwd_pull_kernel(
    const int32_t* __restrict__ tslot, const int4* __restrict__ items, int n_items,
    const int32_t* __restrict__ tdst, const uint32_t* __restrict__ glist, R gp, int F,
    const T* __restrict__ mask, int64_t ldm, T* __restrict__ dx, int64_t ldx, float* __restrict__ ws,
    int64_t ldw, PullMerge pm) {
  constexpr int U = PG_PULL_U;
  __shared__ __attribute__((aligned(16))) float accs[kWavesPerBlock][kGroupMaxF];
  const int wave = wave_id_uniform();
  const int it = blockIdx.x * kWavesPerBlock + wave;
  if (it >= n_items) return;
  float* acc = accs[wave];
  const int4 item = items[it];
  const int row = item.x, t0 = item.y, t1 = item.z, slot = item.w;
  const int lane = lane_id();
  // (MERGE: the 16-B slot stores cover ldw = round_up(F, 4) columns)
  for (int f = lane; f < (MERGE ? (int)ldw : F); f += kWave) acc[f] = 0.f;
  // descriptors (and the destinations' record bases v F) one window ahead, their in-CSR
  // slots two windows ahead (an item with no out-edges reads nothing)
  auto tl_of = [&](int tw) { return tw + min(lane, t1 - tw - 1); };
  uint32_t dsc_next = 0;
  int vf_next = 0, ts_next = 0;
  // TR: the descriptors sit at the transposed indices themselves (coalesced, no slot loads)
  if (t1 > t0) {
    dsc_next = glist[TR ? tl_of(t0) : tslot[tl_of(t0)]];
    vf_next = tdst[tl_of(t0)] * F;
    if (!TR && t0 + kWave < t1) ts_next = tslot[tl_of(t0 + kWave)];
  }
  for (int tw = t0; tw < t1; tw += kWave) {
    const int nw = min(kWave, t1 - tw);
    // this window's edge (lane): its list's first record and its length
    const int2 dsc = make_int2(vf_next + (int)(dsc_next & 0xFFFFu), (int)(dsc_next >> 16));
    if (tw + kWave < t1) {
      dsc_next = glist[TR ? tl_of(tw + kWave) : ts_next];
      vf_next = tdst[tl_of(tw + kWave)] * F;
      if (!TR && tw + 2 * kWave < t1) ts_next = tslot[tl_of(tw + 2 * kWave)];
    }
    // segments: 64-entry pieces of single lists, U segments' loads in flight. Segment t
    // belongs to the edge i with excl_i <= t < excl_i + nseg_i, i.e.
    // i = popcount(ballot(excl <= t)) - 1.
    {
      const int nseg = lane < nw ? (dsc.y + kWave - 1) / kWave : 0;
      const int incl = wave_incl_add(nseg);
      const int excl = incl - nseg;
      const int nseg_all = bcast(incl, kWave - 1);
      for (int s0 = 0; s0 < nseg_all; s0 += U) {
        const int nv = min(U, nseg_all - s0);
        int fe[U], ne[U];
        float de[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int t = s0 + min(u, nv - 1);
          const int i = __popcll(__ballot(excl <= t)) - 1;
          const int seg = t - bcast(excl, i);
          const int base = bcast(dsc.x, i) + seg * kWave;
          const int n = min(kWave, bcast(dsc.y, i) - seg * kWave);
          ne[u] = n;
          // straight-line loads (lanes past n load a valid entry of the same segment), so
          // the waits are counted instead of a vmcnt(0) behind each branch
          gp.get(base + min(lane, n - 1), fe[u], de[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (u < nv && lane < ne[u]) acc[fe[u]] += de[u];
      }
    }
  }
  wave_lds_sync();
  if (slot < 0) {
    T* xr = dx + (int64_t)row * ldx;
    const T* mr = mask ? mask + (int64_t)row * ldm : nullptr;
    for (int f = lane; f < F; f += kWave) {
      float a = acc[f];
      if (mr && !(to_f(mr[f]) > 0.f)) a = 0.f;
      xr[f] = from_f<T>(a);
    }
  } else if constexpr (MERGE) {
    const __amdgpu_buffer_rsrc_t rs = pg_x3::rsrc(ws, pm.ws_bytes);
    const uint32_t sbase = (uint32_t)slot * (uint32_t)ldw * 4u;
    for (int f = lane * 4; f < F; f += kWave * 4)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(pg_u32x4, *reinterpret_cast<const float4*>(acc + f)), rs, sbase + (uint32_t)f * 4u,
                                             0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every payload store drained before the ticket
    const int rb = pm.ptr[row], re = pm.ptr[row + 1];
    const int s0 = slot - (t0 - rb) / pm.chunk;
    const int ns = (re - rb + pm.chunk - 1) / pm.chunk;
    uint32_t ticket = 0;
    if (lane == 0)
      ticket = __hip_atomic_fetch_add((pg_gu32*)(pm.tickets + s0), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ticket = __builtin_amdgcn_readfirstlane(ticket);
    if ((int)ticket != ns - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the ticket
    T* xr = dx + (int64_t)row * ldx;
    const T* mr = mask ? mask + (int64_t)row * ldm : nullptr;
    for (int f = lane * 4; f < F; f += kWave * 4) {
      float a[4] = {0.f, 0.f, 0.f, 0.f};
      for (int s = s0; s < s0 + ns; s += 8) {
        float4 v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          v[e] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
              rs, (uint32_t)min(s + e, s0 + ns - 1) * (uint32_t)ldw * 4u + (uint32_t)f * 4u, 0, 16));
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (s + e < s0 + ns) {
            a[0] += v[e].x; a[1] += v[e].y; a[2] += v[e].z; a[3] += v[e].w;
          }
      }
      if (mr) {
        float mk[4];
        load_tile<4, T>(mr, f, F, mk, 0.f);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (!(mk[i] > 0.f)) a[i] = 0.f;
      }
      store_tile<4, T>(xr, f, F, a);
    }
  } else {
    float* wr = ws + (int64_t)slot * ldw;
    for (int f = lane; f < F; f += kWave) wr[f] = acc[f];
  }
}

// Sum partial slots in order; optional relu' mask (bwd) or 1/deg (mean fwd).
// One workgroup per split row, one thread per feature.
template <typename T = float>
__global__ __launch_bounds__(kBlock) void sum_merge_kernel(
    const int4* __restrict__ merges, int n_merges, int F, const float* __restrict__ ws,
    int64_t ldw, const int32_t* __restrict__ ptr, int divide_by_deg,
    const T* __restrict__ mask, int64_t ldm, T* __restrict__ out, int64_t ldo) {
  const int4 m = merges[blockIdx.x];
  const int row = m.x, s0 = m.y, ns = m.z;
  const float deg = divide_by_deg ? (float)(ptr[row + 1] - ptr[row]) : 1.f;
  // 4 features per thread (float4 slot loads) when every row is 4-aligned: the same
  // per-feature order, bitwise the same result
  constexpr uintptr_t kTa = 4 * sizeof(T) - 1;
  const bool vec = (F % 4) == 0 && (ldw % 4) == 0 && (ldo % 4) == 0 && ((uintptr_t)ws & 15) == 0 &&
                   ((uintptr_t)out & kTa) == 0 && (!mask || ((ldm % 4) == 0 && ((uintptr_t)mask & kTa) == 0));
  if (vec) {
    for (int f = threadIdx.x * 4; f < F; f += kBlock * 4) {
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      for (int s = s0; s < s0 + ns; s += 8) {
        float4 v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          v[e] = *reinterpret_cast<const float4*>(ws + (int64_t)min(s + e, s0 + ns - 1) * ldw + f);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (s + e < s0 + ns) {
            acc[0] += v[e].x; acc[1] += v[e].y; acc[2] += v[e].z; acc[3] += v[e].w;
          }
      }
      if (divide_by_deg)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = acc[i] / deg;
      if (mask) {
        float mk[4];
        load_tile<4, T>(mask + (int64_t)row * ldm, f, F, mk, 0.f);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (!(mk[i] > 0.f)) acc[i] = 0.f;
      }
      store_tile<4, T>(out + (int64_t)row * ldo, f, F, acc);
    }
    return;
  }
  for (int f = threadIdx.x; f < F; f += kBlock) {
    float acc = 0.f;
    for (int s = s0; s < s0 + ns; s += 8) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ws[(int64_t)min(s + e, s0 + ns - 1) * ldw + f];
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (s + e < s0 + ns) acc += v[e];
    }
    if (divide_by_deg) acc = acc / deg;
    if (mask && !(to_f(mask[(int64_t)row * ldm + f]) > 0.f)) acc = 0.f;
    out[(int64_t)row * ldo + f] = from_f<T>(acc);
  }
}

// ---- sum / mean / weighted SpMM ------------------------------------------------------
template <int W, int NC, bool HAS_W, int NORM>
__global__ __launch_bounds__(kBlock) void sum_kernel(
    const int32_t* __restrict__ ptr, const int32_t* __restrict__ col,
    const int32_t* __restrict__ eslot, const float* __restrict__ ew,
    const int32_t* __restrict__ norm_ptr, const int4* __restrict__ items, int n_items,
    const float* __restrict__ X, int64_t ldx, int F, float* __restrict__ out, int64_t ldo,
    float* __restrict__ ws, int64_t ldw) {
  constexpr int U = EdgeU<W, NC>::value;
  const int it = blockIdx.x * kWavesPerBlock + wave_id_uniform();
  if (it >= n_items) return;
  const int4 item = items[it];
  const int row = item.x, k0 = item.y, k1 = item.z, slot = item.w;
  const int lane = lane_id();
  float acc[NC][W];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < W; ++i) acc[c][i] = 0.f;

  for (int kw = k0; kw < k1; kw += kWave) {
    const int nw = min(kWave, k1 - kw);
    const int kl = kw + min(lane, nw - 1);
    const int idxv = col[kl];
    float wv = 1.f, dv = 1.f;
    if constexpr (HAS_W) wv = ew[eslot ? eslot[kl] : kl];
    if constexpr (NORM == 2) dv = (float)(norm_ptr[idxv + 1] - norm_ptr[idxv]);
    for (int j = 0; j < nw; j += U) {
      const int nv = min(U, nw - j);
      float v[U][NC][W];
#pragma unroll
      for (int e = 0; e < U; ++e) {
        const float* xr = X + (int64_t)bcast(idxv, j + min(e, nv - 1)) * ldx;
#pragma unroll
        for (int c = 0; c < NC; ++c) load_tile<W>(xr, (c * kWave + lane) * W, F, v[e][c], 0.f);
      }
#pragma unroll
      for (int e = 0; e < U; ++e) {
        if (e < nv) {
          float w = 1.f, dc = 1.f;
          if constexpr (HAS_W) w = bcastf(wv, j + e);
          if constexpr (NORM == 2) dc = bcastf(dv, j + e);
#pragma unroll
          for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int i = 0; i < W; ++i) {
              float tv = HAS_W ? v[e][c][i] * w : v[e][c][i];
              if constexpr (NORM == 2) tv = tv / dc;
              acc[c][i] += tv;
            }
        }
      }
    }
  }
  if (slot < 0) {
    if constexpr (NORM == 1) {
      const int d = ptr[row + 1] - ptr[row];
      if (d > 0) {
        const float fd = (float)d;
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
          for (int i = 0; i < W; ++i) acc[c][i] = acc[c][i] / fd;
      }
    }
    float* orow = out + (int64_t)row * ldo;
#pragma unroll
    for (int c = 0; c < NC; ++c) store_tile<W>(orow, (c * kWave + lane) * W, F, acc[c]);
  } else {
    float* wr = ws + (int64_t)slot * ldw;
#pragma unroll
    for (int c = 0; c < NC; ++c) store_tile<W>(wr, (c * kWave + lane) * W, F, acc[c]);
  }
}

// ---- DGL-form scatter backward (float atomics) ----------------------------------------
__global__ __launch_bounds__(kBlock) void clear_u4_kernel(uint4* __restrict__ x, int64_t n4) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kBlock)
    x[i] = make_uint4(0u, 0u, 0u, 0u);
}

__global__ __launch_bounds__(kBlock) void fill2d_kernel(float* __restrict__ x, int64_t ldx,
                                                        int64_t rows, int cols, float val) {
  const int64_t n = rows * (int64_t)cols;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t r = i / cols;
    const int c = (int)(i - r * cols);
    x[r * ldx + c] = val;
  }
}

template <typename A, bool HAS_W>
__global__ __launch_bounds__(kBlock) void max_bwd_scatter_kernel(
    const int32_t* __restrict__ ptr, const int32_t* __restrict__ col,
    const int32_t* __restrict__ eslot, const float* __restrict__ ew, int64_t n_rows,
    const A* __restrict__ arg, int64_t lda, const float* __restrict__ dout, int64_t ldd, int F,
    float* __restrict__ dx, int64_t ldx) {
  const int64_t row = (int64_t)blockIdx.x * kWavesPerBlock + wave_id_uniform();
  if (row >= n_rows) return;
  const int rs = ptr[row];
  for (int f = lane_id(); f < F; f += kWave) {
    const int a = (int)arg[row * lda + f];
    if (a == arg_none<A>()) continue;
    const int k = rs + a;
    const int u = col[k];
    float d = dout[row * ldd + f];
    if (HAS_W) d = ew[eslot ? eslot[k] : k] * d;
    atomicAdd(dx + (int64_t)u * ldx + f, d);
  }
}

template <typename A>
__global__ __launch_bounds__(kBlock) void argpos_to_src_kernel(
    const int32_t* __restrict__ ptr, const int32_t* __restrict__ col, int64_t n_rows,
    const A* __restrict__ arg, int64_t lda, int F, int64_t* __restrict__ argx, int64_t ldx) {
  const int64_t n = n_rows * (int64_t)F;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t v = i / F;
    const int f = (int)(i - v * F);
    const int a = (int)arg[v * lda + f];
    argx[v * ldx + f] = a == arg_none<A>() ? -1 : (int64_t)col[ptr[v] + a];
  }
}

// ---- host-side dispatch helpers --------------------------------------------------------
inline int grid_for(int64_t n_work) {
  return (int)((n_work + kWavesPerBlock - 1) / kWavesPerBlock);
}

inline int hip_status(const char* who) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return pg::set_error((int)e, "%s: launch failed: %s", who, hipGetErrorString(e));
  return pg::ok();
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }
inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// workspace layout: [values: n_slots x ldw floats][args: n_slots x ldw A], 256-B aligned
inline int64_t ws_ld(int64_t F) { return round_up(F, 4); }

// Feature tiles per launch: the kernel is instantiated for F <= kFTile; wider F is
// processed in tiles by offsetting the feature pointers.
constexpr int kFTileVec = kMaxNC * kWave * 4;        // 1024
constexpr int kFTileScalar = kMaxNCScalar * kWave;   // 1024

template <typename Fn>
int dispatch_nc_vec(int nc, Fn&& fn) {
  switch (nc) {
    case 1: return fn(std::integral_constant<int, 1>{});
    case 2: return fn(std::integral_constant<int, 2>{});
    case 3: return fn(std::integral_constant<int, 3>{});
    case 4: return fn(std::integral_constant<int, 4>{});
  }
  return PG_ERR_UNSUPPORTED;
}

template <typename Fn>
int dispatch_nc_scalar(int nc, Fn&& fn) {
  switch (nc) {
    case 1: return fn(std::integral_constant<int, 1>{});
    case 2: return fn(std::integral_constant<int, 2>{});
    case 3: return fn(std::integral_constant<int, 3>{});
    case 4: return fn(std::integral_constant<int, 4>{});
    case 5: return fn(std::integral_constant<int, 5>{});
    case 6: return fn(std::integral_constant<int, 6>{});
    case 7: return fn(std::integral_constant<int, 7>{});
    case 8: return fn(std::integral_constant<int, 8>{});
    case 9: return fn(std::integral_constant<int, 9>{});
    case 10: return fn(std::integral_constant<int, 10>{});
    case 11: return fn(std::integral_constant<int, 11>{});
    case 12: return fn(std::integral_constant<int, 12>{});
    case 13: return fn(std::integral_constant<int, 13>{});
    case 14: return fn(std::integral_constant<int, 14>{});
    case 15: return fn(std::integral_constant<int, 15>{});
    case 16: return fn(std::integral_constant<int, 16>{});
  }
  return PG_ERR_UNSUPPORTED;
}

struct TilePlan {
  bool vec;
  int64_t tile;
};

// Feature columns per launch on the vector path (a multiple of 256 up to 1024; variant
// builds: -DPG_SPMM_FTILE=...): narrower tiles mean fewer registers per wave (higher
// occupancy) at the price of re-reading the column ids once per tile. 256 measured best.
#ifndef PG_SPMM_FTILE
#define PG_SPMM_FTILE 256
#endif
static_assert(PG_SPMM_FTILE >= 256 && PG_SPMM_FTILE <= kFTileVec && PG_SPMM_FTILE % 256 == 0, "feature tile");
constexpr int64_t vec_ftile() { return PG_SPMM_FTILE; }

inline TilePlan plan_tiles(int64_t F, std::initializer_list<int64_t> lds,
                           std::initializer_list<const void*> ptrs) {
  bool vec = (F % 4) == 0;
  for (int64_t l : lds) vec = vec && (l % 4) == 0;
  for (const void* p : ptrs) vec = vec && (p == nullptr || aligned16(p));
  return {vec, vec ? vec_ftile() : (int64_t)kFTileScalar};
}

template <typename A, typename T>
int launch_max_fwd(const pg_csr_t* g, const T* X, int64_t ldx, int64_t F, T* out,
                   int64_t ldo, A* arg, int64_t lda, float* ws_val, A* ws_arg, int64_t ldw,
                   int dead_none, hipStream_t st, uint32_t* tickets) {
  // argpos rows: u16 x4 = 8 B -> need 8-B alignment only; treat via the same 16-B check on
  // the float operands and an 8-B check on arg.
  TilePlan tp = plan_tiles(F, {ldx, ldo, lda}, {X, out, ws_val});
  if (tp.vec && (((uintptr_t)arg & (4 * sizeof(A) - 1)) != 0 ||
                 ((uintptr_t)ws_arg & (4 * sizeof(A) - 1)) != 0))
    tp.vec = false;
  if (!tp.vec) tp.tile = kFTileScalar;
  const bool has_w = g->ew != nullptr;
  const int blocks = grid_for(g->n_items);
  // every feature tile in one launch (blocks interleaved over the tiles), one merge launch
  // over the whole F
  const int n_ft = (int)((F + tp.tile - 1) / tp.tile);
  if constexpr (PG_FWD_SLICE > 0) if (tp.vec && g->n_items > 0 && (g->n_merges == 0 || g->merges)) {
    // XCD column slices (max_fwd_slice_kernel); split rows whole, first. The slices must share
    // out over the 8 XCDs (1, 2, 4 or a multiple of 8 of them): a width whose PG_FWD_SLICE-byte
    // slices do not (F = 400 f32: 7 of 64 columns) tries slices twice as wide (4 of 128).
    auto try_slices = [&](auto lpr_c) -> bool {
      constexpr int LPR = decltype(lpr_c)::value;
      constexpr int RPW = kWave / LPR;
      const int n_sl = (int)((F + 4 * LPR - 1) / (4 * LPR));
      if (!(n_sl % 8 == 0 || n_sl == 1 || n_sl == 2 || n_sl == 4) ||
          g->n_cols * (int64_t)(4 * LPR * sizeof(T)) > PG_FWD_SLICE_MAXTAB)
        return false;
      auto grid_of = [&](int64_t n_iblk) -> int64_t {
        if (n_iblk == 0) return 0;
        return n_sl >= 8 ? n_iblk * n_sl : 8 * ((n_iblk + 8 / n_sl - 1) / (8 / n_sl));
      };
      const int n_iblk = (int)((g->n_items + RPW * kWavesPerBlock - 1) / (RPW * kWavesPerBlock));
      const int n_hub = (int)g->n_merges;
      // row pieces in flight per lane group: 4 with one slice per XCD and no edge weights
      // (cfg2's F = 512: 147.8-148.2 vs 151.8 us), else 8 (F = 256: 81.6 vs 88.5 us; cfg3's
      // weighted F = 512: 169-171 vs 177-180 us)
      auto go = [&](auto hw_c, auto ue_c) {
        constexpr bool HW = decltype(hw_c)::value;
        constexpr int UE = decltype(ue_c)::value;
        const int64_t hub_grid = grid_of(n_hub);
        hipLaunchKernelGGL((max_fwd_slice_kernel<LPR, UE, HW, A, T>), dim3((unsigned)(hub_grid + grid_of(n_iblk))),
                           dim3(kBlock), 0, st, g->ptr, g->col, g->eslot, g->ew, (const int4*)g->items,
                           (int)g->n_items, (const int4*)g->merges, n_hub, (int)hub_grid, X, ldx, (int)F, out, ldo,
                           arg, lda, n_sl, n_iblk, dead_none);
      };
      using U4 = std::integral_constant<int, 4>;
      using U8 = std::integral_constant<int, 8>;
      if (n_sl >= 8 && !has_w && PG_SLICE_U_FIXED != 8) {
        go(std::false_type{}, U4{});
      } else {
        if (has_w) go(std::true_type{}, U8{}); else go(std::false_type{}, U8{});
      }
      return true;
    };
    constexpr int LPR0 = std::min(32, PG_FWD_SLICE / (4 * (int)sizeof(T)));
    bool done = try_slices(std::integral_constant<int, LPR0>{});
    if constexpr (2 * LPR0 <= 32 && !PG_FWD_SLICE_NO_WIDE)
      if (!done) done = try_slices(std::integral_constant<int, 2 * LPR0>{});
    if (done) return hip_status("pg_spmm_max_fwd");
  }
  {
    const int64_t f0 = 0;
    const int Ft = (int)std::min<int64_t>(tp.tile, F);
    // split rows combined inside the launch (max_merge_kernel's launch otherwise): the vector
    // path, the schedule's chunk known, slot regions a 32-bit buffer offset covers
    const size_t vbytes = round_up(g->n_slots * ldw * 4, 256), abytes = round_up(g->n_slots * ldw * (int64_t)sizeof(A), 256);
    const bool merge_in = PG_FWD_MERGE && tp.vec && g->n_merges > 0 && g->chunk > 0 && tickets &&
                          vbytes < ((size_t)1 << 31) && abytes < ((size_t)1 << 31);
    if (merge_in) {  // the tickets start at zero: [n_slots x n_ft] words, a 256-B padded block
      const int64_t n4 = round_up(g->n_slots * n_ft * 4, 256) / 16;
      hipLaunchKernelGGL(clear_u4_kernel, dim3((unsigned)std::min<int64_t>(2048, (n4 + kBlock - 1) / kBlock)),
                         dim3(kBlock), 0, st, reinterpret_cast<uint4*>(tickets), n4);
    }
    const FwdMerge fm{g->chunk, tickets, (uint32_t)vbytes, (uint32_t)abytes};
    auto go = [&](auto nc_c, auto w_c, auto hw_c) -> int {
      constexpr int NC = decltype(nc_c)::value;
      constexpr int W = decltype(w_c)::value;
      constexpr bool HW = decltype(hw_c)::value;
      if (merge_in)
        hipLaunchKernelGGL((max_fwd_kernel<W, NC, HW, A, T, true>), dim3((unsigned)blocks * n_ft), dim3(kBlock), 0,
                           st, g->ptr, g->col, g->eslot, g->ew, (const int4*)g->items, (int)g->n_items,
                           X, ldx, n_ft > 1 ? (int)F : Ft, out, ldo, arg, lda, ws_val, ws_arg, ldw, n_ft,
                           (int)tp.tile, dead_none, fm);
      else
        hipLaunchKernelGGL((max_fwd_kernel<W, NC, HW, A, T, false>), dim3((unsigned)blocks * n_ft), dim3(kBlock), 0,
                           st, g->ptr, g->col, g->eslot, g->ew, (const int4*)g->items, (int)g->n_items,
                           X, ldx, n_ft > 1 ? (int)F : Ft, out, ldo, arg, lda, ws_val, ws_arg, ldw, n_ft,
                           (int)tp.tile, dead_none, fm);
      return PG_OK;
    };
    int rc;
    if (tp.vec) {
      const int nc = (Ft + 255) / 256;
      rc = has_w ? dispatch_nc_vec(nc, [&](auto n) { return go(n, std::integral_constant<int, 4>{}, std::true_type{}); })
                 : dispatch_nc_vec(nc, [&](auto n) { return go(n, std::integral_constant<int, 4>{}, std::false_type{}); });
    } else {
      const int nc = (Ft + 63) / 64;
      rc = has_w ? dispatch_nc_scalar(nc, [&](auto n) { return go(n, std::integral_constant<int, 1>{}, std::true_type{}); })
                 : dispatch_nc_scalar(nc, [&](auto n) { return go(n, std::integral_constant<int, 1>{}, std::false_type{}); });
    }
    if (rc != PG_OK) return pg::set_error(rc, "pg_spmm_max_fwd: unsupported feature tile");
    if (g->n_merges > 0 && !merge_in) {
      hipLaunchKernelGGL((max_merge_kernel<A, T>), dim3((unsigned)g->n_merges), dim3(kBlock), 0, st,
                         (const int4*)g->merges, (int)g->n_merges, (int)F, ws_val + f0, ws_arg + f0,
                         ldw, out + f0, ldo, arg + f0, lda, dead_none);
    }
  }
  return hip_status("pg_spmm_max_fwd");
}

template <typename A>
int launch_max_bwd(const pg_csr_t* g, const pg_csr_t* gt, const A* arg, int64_t lda,
                   const float* dout, int64_t ldd, int64_t F, const float* mask, int64_t ldm,
                   float* dx, int64_t ldx, float* ws, int64_t ldw, hipStream_t st) {
  TilePlan tp = plan_tiles(F, {lda, ldd, ldx, mask ? ldm : 4}, {dout, dx, mask, ws});
  if (tp.vec && ((uintptr_t)arg & (4 * sizeof(A) - 1)) != 0) tp.vec = false;
  if (!tp.vec) tp.tile = kFTileScalar;
  const bool has_w = g->ew != nullptr;
  const int blocks = grid_for(gt->n_items);
  for (int64_t f0 = 0; f0 < F; f0 += tp.tile) {
    const int Ft = (int)std::min<int64_t>(tp.tile, F - f0);
    auto go = [&](auto nc_c, auto w_c, auto hw_c) -> int {
      constexpr int NC = decltype(nc_c)::value;
      constexpr int W = decltype(w_c)::value;
      constexpr bool HW = decltype(hw_c)::value;
      hipLaunchKernelGGL((max_bwd_kernel<W, NC, HW, A>), dim3(blocks), dim3(kBlock), 0, st,
                         g->ew, gt->col, gt->eslot, gt->epos, (const int4*)gt->items,
                         (int)gt->n_items, arg + f0, lda, dout + f0, ldd, Ft,
                         mask ? mask + f0 : nullptr, ldm, dx + f0, ldx, ws ? ws + f0 : nullptr,
                         ldw);
      return PG_OK;
    };
    int rc;
    if (tp.vec) {
      const int nc = (Ft + 255) / 256;
      rc = has_w ? dispatch_nc_vec(nc, [&](auto n) { return go(n, std::integral_constant<int, 4>{}, std::true_type{}); })
                 : dispatch_nc_vec(nc, [&](auto n) { return go(n, std::integral_constant<int, 4>{}, std::false_type{}); });
    } else {
      const int nc = (Ft + 63) / 64;
      rc = has_w ? dispatch_nc_scalar(nc, [&](auto n) { return go(n, std::integral_constant<int, 1>{}, std::true_type{}); })
                 : dispatch_nc_scalar(nc, [&](auto n) { return go(n, std::integral_constant<int, 1>{}, std::false_type{}); });
    }
    if (rc != PG_OK) return pg::set_error(rc, "pg_spmm_max_bwd: unsupported feature tile");
    if (gt->n_merges > 0) {
      hipLaunchKernelGGL(sum_merge_kernel<float>, dim3((unsigned)gt->n_merges), dim3(kBlock), 0, st,
                         (const int4*)gt->merges, (int)gt->n_merges, Ft, ws + f0, ldw, gt->ptr, 0,
                         mask ? mask + f0 : nullptr, ldm, dx + f0, ldx);
    }
  }
  return hip_status("pg_spmm_max_bwd");
}

int check_ws(size_t have, size_t need, const char* who) {
  if (have < need)
    return pg::set_error(PG_ERR_WORKSPACE, "%s: workspace %zu B < required %zu B", who, have, need);
  return PG_OK;
}

}  // namespace

extern "C" {

size_t pg_spmm_max_fwd_workspace(const pg_csr_t* g, int64_t F, int arg_kind) {
  if (!g || g->n_slots <= 0 || F <= 0) return 0;
  const int64_t ldw = ws_ld(F);
  const size_t vals = round_up(g->n_slots * ldw * 4, 256);
  const size_t args = round_up(g->n_slots * ldw * (int64_t)pg::arg_bytes(arg_kind & ~PG_ARG_DEAD_NONE), 256);
  // the whole-row kernel's split-row tickets: one word per slot and 256-column feature tile
  const size_t tickets = round_up(g->n_slots * ((F + 255) / 256) * 4, 256);
  return vals + args + tickets;
}

}  // extern "C"

namespace {

template <typename T>
int max_fwd_entry(const pg_csr_t* g, const T* X, int64_t ldx, int64_t F, T* out, int64_t ldo,
                  void* argpos, int64_t lda, int arg_kind, void* ws, size_t ws_bytes,
                  pg_stream_t stream) {
  PG_TRY(pg::check_csr(g, "pg_spmm_max_fwd", true));
  const int dead_none = (arg_kind & PG_ARG_DEAD_NONE) != 0;
  arg_kind &= ~PG_ARG_DEAD_NONE;
  if (!pg::valid_arg_kind(arg_kind))
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_fwd: bad arg_kind %d", arg_kind);
  if (F < 0 || ldx < F || ldo < F || lda < F)
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_fwd: bad F/leading dims");
  if (arg_kind == PG_ARG_U16 && g->max_deg >= 0xFFFF)
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_fwd: max degree %d needs PG_ARG_I32",
                         g->max_deg);
  if (F == 0 || g->n_rows == 0) return pg::ok();
  if (!X || !out || !argpos) return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_fwd: NULL buffer");
  const size_t need = pg_spmm_max_fwd_workspace(g, F, arg_kind);
  PG_TRY(check_ws(ws_bytes, need, "pg_spmm_max_fwd"));
  const int64_t ldw = ws_ld(F);
  float* ws_val = need ? (float*)ws : nullptr;
  void* ws_arg = need ? (char*)ws + round_up(g->n_slots * ldw * 4, 256) : nullptr;
  // [slot values | slot positions | split-row tickets]
  uint32_t* tickets = need ? (uint32_t*)((char*)ws_arg + round_up(g->n_slots * ldw * (int64_t)pg::arg_bytes(arg_kind), 256))
                           : nullptr;
  if (((uintptr_t)ws & 255) != 0) tickets = nullptr;  // (the in-launch combine wants aligned regions)
  hipStream_t st = (hipStream_t)stream;
  if (arg_kind == PG_ARG_U16)
    return launch_max_fwd<uint16_t, T>(g, X, ldx, F, out, ldo, (uint16_t*)argpos, lda, ws_val,
                                       (uint16_t*)ws_arg, ldw, dead_none, st, tickets);
  return launch_max_fwd<int32_t, T>(g, X, ldx, F, out, ldo, (int32_t*)argpos, lda, ws_val,
                                    (int32_t*)ws_arg, ldw, dead_none, st, tickets);
}

}  // namespace

extern "C" {

int pg_spmm_max_fwd(const pg_csr_t* g, const float* X, int64_t ldx, int64_t F, float* out,
                    int64_t ldo, void* argpos, int64_t lda, int arg_kind, void* ws,
                    size_t ws_bytes, pg_stream_t stream) {
  return max_fwd_entry<float>(g, X, ldx, F, out, ldo, argpos, lda, arg_kind, ws, ws_bytes, stream);
}

int pg_spmm_max_fwd_bf16(const pg_csr_t* g, const void* X, int64_t ldx, int64_t F, void* out,
                         int64_t ldo, void* argpos, int64_t lda, int arg_kind, void* ws,
                         size_t ws_bytes, pg_stream_t stream) {
  return max_fwd_entry<uint16_t>(g, (const uint16_t*)X, ldx, F, (uint16_t*)out, ldo, argpos, lda,
                                 arg_kind, ws, ws_bytes, stream);
}

// [split-row partials][grouped path: list records N x F x 8 B | glist nnz x 4 B | tickets n_slots x 4 B]
static size_t bwd_partials_bytes(const pg_csr_t* gt, int64_t F) {
  return gt->n_slots > 0 ? round_up(gt->n_slots * ws_ld(F) * 4, 256) : 0;
}

size_t pg_spmm_max_bwd_workspace(const pg_csr_t* gt, int64_t F) {
  if (!gt || F <= 0) return 0;
  size_t b = bwd_partials_bytes(gt, F);
  if (F <= kGroupMaxF) {
    const int64_t N = gt->n_cols;
    b += round_up(N * F * 8, 256) + round_up(gt->nnz * 4, 256);
    if (gt->n_slots > 0) b += round_up(gt->n_slots * 4, 256);  // the pull's split-row tickets
  }
  return b;
}

}  // extern "C"

namespace {

template <typename T>
int max_bwd_entry(const pg_csr_t* g, const pg_csr_t* gt, const void* argpos, int64_t lda,
                  int arg_kind, const T* dout, int64_t ldd, int64_t F, const T* mask_src,
                  int64_t ldm, const T* fwd_out, int64_t ldf, T* dx, int64_t ldx, void* ws,
                  size_t ws_bytes, pg_stream_t stream) {
  PG_TRY(pg::check_csr(g, "pg_spmm_max_bwd", false));
  PG_TRY(pg::check_csr(gt, "pg_spmm_max_bwd", true));
  // PG_ARG_DEAD_NONE: the records already leave out the zero maxima (fwd_out's filter)
  const bool dead_none = (arg_kind & PG_ARG_DEAD_NONE) != 0;
  arg_kind &= ~PG_ARG_DEAD_NONE;
  if (!pg::valid_arg_kind(arg_kind))
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_bwd: bad arg_kind %d", arg_kind);
  if (gt->n_cols != g->n_rows || gt->nnz != g->nnz)
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_bwd: gt is not the transpose of g");
  if (gt->nnz > 0 && (!gt->epos || !gt->eslot))
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_bwd: gt needs eslot and epos");
  if (F < 0 || ldd < F || ldx < F || lda < F || (mask_src && ldm < F) || (fwd_out && ldf < F))
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_bwd: bad F/leading dims");
  if ((fwd_out || dead_none) && !mask_src)
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_bwd: fwd_out / PG_ARG_DEAD_NONE needs mask_src");
  if (dead_none) fwd_out = nullptr;
  if (F == 0 || gt->n_rows == 0) return pg::ok();
  if (!argpos || !dout || !dx) return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_bwd: NULL buffer");
  const size_t need = pg_spmm_max_bwd_workspace(gt, F);
  PG_TRY(check_ws(ws_bytes, need, "pg_spmm_max_bwd"));
  hipStream_t st = (hipStream_t)stream;
  const size_t pbytes = bwd_partials_bytes(gt, F);
  float* w = pbytes ? (float*)ws : nullptr;
  const int64_t N = g->n_rows;
  // PG_BWD_DIRECT (variant builds): always the argmax-record gather over the transposed CSR
  if (arg_kind == PG_ARG_U16 && F <= kGroupMaxF && N * F < INT32_MAX && !PG_BWD_DIRECT) {
    char* p = (char*)ws + pbytes;
    // the records carry the upstream gradient as f32 (8 B), or for bf16 storage without edge
    // weights as its bf16 value (4 B); the sums are f32 either way (one rounding of dx at the
    // end, as the oracle's f32 sums)
    void* recs = p;
    p += round_up(N * F * 8, 256);
    uint32_t* glist = (uint32_t*)p;
    p += round_up(g->nnz * 4, 256);
    uint32_t* tickets = (uint32_t*)p;
    // split rows combined inside the pull (sum_merge_kernel's launch otherwise): vector rows,
    // the schedule's chunk known, a slot region a 32-bit buffer offset covers
    constexpr uintptr_t kTm = 4 * sizeof(T) - 1;
    const bool merge_in = PG_PULL_MERGE && gt->n_merges > 0 && gt->chunk > 0 && F % 4 == 0 && ldx % 4 == 0 &&
                          ((uintptr_t)dx & kTm) == 0 && ((uintptr_t)w & 15) == 0 && pbytes < ((size_t)1 << 31) &&
                          (!mask_src || dead_none || (ldm % 4 == 0 && ((uintptr_t)mask_src & kTm) == 0));
    const int n_tickets = merge_in ? (int)gt->n_slots : 0;
    const auto* arg16 = (const uint16_t*)argpos;
    // rows past kPackWaveMax: the schedule's split rows when its chunk guarantees they are
    // a superset, else every row
    const bool listed = g->merges != nullptr && g->chunk > 0 && g->chunk <= kPackWaveMax;
    const int n_long = (int)(listed ? g->n_merges : N);
    const int n_short_blocks = (int)((N + kWavesPerBlock - 1) / kWavesPerBlock);
    // 4 features per lane (vector loads) when every row is 4-aligned
    constexpr uintptr_t kTa = 4 * sizeof(T) - 1;
    const bool vec = F % 4 == 0 && lda % 4 == 0 && ldd % 4 == 0 && (!fwd_out || ldf % 4 == 0) &&
                     ((uintptr_t)argpos & 7) == 0 && ((uintptr_t)dout & kTa) == 0 && ((uintptr_t)fwd_out & kTa) == 0;
    const dim3 pgrid((unsigned)(n_long + n_short_blocks));
    const int4* prow = listed ? (const int4*)g->merges : nullptr;
    // transposed descriptors when the in-CSR slots' transposed indices are given (g->epos)
    const bool tr = g->epos != nullptr && PG_BWD_TRANS && ((uintptr_t)glist & 15) == 0;
    // cleared by a kernel of this library, not hipMemsetAsync: a memset issued while the
    // stream is being captured into a HIP graph did not clear the array on replays (the
    // engine's step graph trained on stale descriptors)
    if (tr && g->nnz > 0) {
      const int64_t n4 = (g->nnz + 3) / 4;  // glist is 256-B aligned and padded: whole uint4s
      hipLaunchKernelGGL(clear_u4_kernel, dim3((unsigned)std::min<int64_t>(2048, (n4 + kBlock - 1) / kBlock)),
                         dim3(kBlock), 0, st, reinterpret_cast<uint4*>(glist), n4);
    }
    auto run = [&](auto gp, auto tr_c) {
    using R = decltype(gp);
    constexpr bool TR = decltype(tr_c)::value;
    auto pack = [&](auto nv_c) {
      constexpr int NV = decltype(nv_c)::value;
      hipLaunchKernelGGL((group_pack_kernel<uint16_t, T, NV, R, TR>), pgrid, dim3(kBlock), 0, st, prow, n_long,
                         (int)N, g->ptr, arg16, lda, (int)F, dout, ldd, fwd_out, ldf, g->ew, gp, glist, g->epos,
                         tickets, n_tickets);
      return PG_OK;
    };
    if (vec) dispatch_nc_vec((int)((F + 255) / 256), pack);
    else pack(std::integral_constant<int, 0>{});
    const int blocks = grid_for(gt->n_items);
    // dead-none records imply the relu' mask (the contract: mask_src >= 0): every entry left
    // in the lists has a maximum X[u,f] w != 0, so X[u,f] > 0; an element with no entries
    // sums to +0, which the mask would leave +0. With fwd_out alone the mask is applied.
    if (dead_none) mask_src = nullptr;
    const PullMerge pm{gt->ptr, gt->chunk, tickets, (uint32_t)pbytes};
    if (merge_in)
      hipLaunchKernelGGL((max_bwd_pull_kernel<T, R, TR, true>), dim3(blocks), dim3(kBlock), 0, st, gt->eslot,
                         (const int4*)gt->items, (int)gt->n_items, gt->col, glist, gp, (int)F, mask_src, ldm,
                         dx, ldx, w, ws_ld(F), pm);
    else
      hipLaunchKernelGGL((max_bwd_pull_kernel<T, R, TR, false>), dim3(blocks), dim3(kBlock), 0, st, gt->eslot,
                         (const int4*)gt->items, (int)gt->n_items, gt->col, glist, gp, (int)F, mask_src, ldm,
                         dx, ldx, w, ws_ld(F), pm);
    if (gt->n_merges > 0 && !merge_in)
      hipLaunchKernelGGL(sum_merge_kernel<T>, dim3((unsigned)gt->n_merges), dim3(kBlock), 0, st,
                         (const int4*)gt->merges, (int)gt->n_merges, (int)F, w, ws_ld(F), gt->ptr, 0,
                         mask_src, ldm, dx, ldx);
    };
    auto run_tr = [&](auto gp) {
      if (tr) run(gp, std::true_type{});
      else run(gp, std::false_type{});
    };
    if (sizeof(T) == 2 && !g->ew) {
      GPack4 gp;
      gp.r = (uint32_t*)recs;
      run_tr(gp);
    } else {
      GPack gp;
      gp.r = (uint2*)recs;
      run_tr(gp);
    }
    return hip_status("pg_spmm_max_bwd");
  }
  if constexpr (sizeof(T) == 4) {
    if (arg_kind == PG_ARG_U16)
      return launch_max_bwd<uint16_t>(g, gt, (const uint16_t*)argpos, lda, dout, ldd, F, mask_src,
                                      ldm, dx, ldx, w, ws_ld(F), st);
    return launch_max_bwd<int32_t>(g, gt, (const int32_t*)argpos, lda, dout, ldd, F, mask_src, ldm,
                                   dx, ldx, w, ws_ld(F), st);
  } else {
    return pg::set_error(PG_ERR_UNSUPPORTED,
                         "pg_spmm_max_bwd_bf16: needs PG_ARG_U16 records and F <= %d (grouped path)",
                         kGroupMaxF);
  }
}

}  // namespace

extern "C" {

int pg_spmm_max_bwd(const pg_csr_t* g, const pg_csr_t* gt, const void* argpos, int64_t lda,
                    int arg_kind, const float* dout, int64_t ldd, int64_t F,
                    const float* mask_src, int64_t ldm, const float* fwd_out, int64_t ldf,
                    float* dx, int64_t ldx, void* ws, size_t ws_bytes, pg_stream_t stream) {
  return max_bwd_entry<float>(g, gt, argpos, lda, arg_kind, dout, ldd, F, mask_src, ldm, fwd_out, ldf,
                              dx, ldx, ws, ws_bytes, stream);
}

int pg_spmm_max_bwd_bf16(const pg_csr_t* g, const pg_csr_t* gt, const void* argpos, int64_t lda,
                         int arg_kind, const void* dout, int64_t ldd, int64_t F,
                         const void* mask_src, int64_t ldm, const void* fwd_out, int64_t ldf,
                         void* dx, int64_t ldx, void* ws, size_t ws_bytes, pg_stream_t stream) {
  return max_bwd_entry<uint16_t>(g, gt, argpos, lda, arg_kind, (const uint16_t*)dout, ldd, F,
                                 (const uint16_t*)mask_src, ldm, (const uint16_t*)fwd_out, ldf,
                                 (uint16_t*)dx, ldx, ws, ws_bytes, stream);
}

int pg_spmm_max_bwd_scatter(const pg_csr_t* g, const void* argpos, int64_t lda, int arg_kind,
                            const float* dout, int64_t ldd, int64_t F, float* dx, int64_t ldx,
                            int64_t n_src, pg_stream_t stream) {
  PG_TRY(pg::check_csr(g, "pg_spmm_max_bwd_scatter", false));
  if (!pg::valid_arg_kind(arg_kind))
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_bwd_scatter: bad arg_kind %d", arg_kind);
  if (F < 0 || ldd < F || ldx < F || lda < F || n_src < g->n_cols)
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_max_bwd_scatter: bad F/leading dims");
  if (F == 0) return pg::ok();
  hipStream_t st = (hipStream_t)stream;
  const int64_t n_fill = n_src * F;
  const int fill_blocks = (int)std::min<int64_t>(4096, (n_fill + kBlock - 1) / kBlock);
  if (fill_blocks > 0)
    hipLaunchKernelGGL(fill2d_kernel, dim3(fill_blocks), dim3(kBlock), 0, st, dx, ldx, n_src,
                       (int)F, 0.f);
  const int blocks = grid_for(g->n_rows);
  if (blocks > 0) {
    const bool hw = g->ew != nullptr;
    if (arg_kind == PG_ARG_U16) {
      if (hw)
        hipLaunchKernelGGL((max_bwd_scatter_kernel<uint16_t, true>), dim3(blocks), dim3(kBlock), 0, st,
                           g->ptr, g->col, g->eslot, g->ew, g->n_rows, (const uint16_t*)argpos, lda,
                           dout, ldd, (int)F, dx, ldx);
      else
        hipLaunchKernelGGL((max_bwd_scatter_kernel<uint16_t, false>), dim3(blocks), dim3(kBlock), 0, st,
                           g->ptr, g->col, g->eslot, g->ew, g->n_rows, (const uint16_t*)argpos, lda,
                           dout, ldd, (int)F, dx, ldx);
    } else {
      if (hw)
        hipLaunchKernelGGL((max_bwd_scatter_kernel<int32_t, true>), dim3(blocks), dim3(kBlock), 0, st,
                           g->ptr, g->col, g->eslot, g->ew, g->n_rows, (const int32_t*)argpos, lda,
                           dout, ldd, (int)F, dx, ldx);
      else
        hipLaunchKernelGGL((max_bwd_scatter_kernel<int32_t, false>), dim3(blocks), dim3(kBlock), 0, st,
                           g->ptr, g->col, g->eslot, g->ew, g->n_rows, (const int32_t*)argpos, lda,
                           dout, ldd, (int)F, dx, ldx);
    }
  }
  return hip_status("pg_spmm_max_bwd_scatter");
}

size_t pg_spmm_sum_workspace(const pg_csr_t* g, int64_t F) {
  if (!g || g->n_slots <= 0 || F <= 0) return 0;
  return round_up(g->n_slots * ws_ld(F) * 4, 256);
}

int pg_spmm_sum(const pg_csr_t* g, const float* X, int64_t ldx, int64_t F, int norm_mode,
                const int32_t* norm_ptr, float* out, int64_t ldo, void* ws, size_t ws_bytes,
                pg_stream_t stream) {
  PG_TRY(pg::check_csr(g, "pg_spmm_sum", true));
  if (F < 0 || ldx < F || ldo < F)
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_sum: bad F/leading dims");
  if (norm_mode < 0 || norm_mode > 2 || (norm_mode == 2 && !norm_ptr))
    return pg::set_error(PG_ERR_INVALID, "pg_spmm_sum: bad norm_mode %d", norm_mode);
  if (F == 0 || g->n_rows == 0) return pg::ok();
  if (!X || !out) return pg::set_error(PG_ERR_INVALID, "pg_spmm_sum: NULL buffer");
  const size_t need = pg_spmm_sum_workspace(g, F);
  PG_TRY(check_ws(ws_bytes, need, "pg_spmm_sum"));
  float* w = need ? (float*)ws : nullptr;
  const int64_t ldw = ws_ld(F);
  hipStream_t st = (hipStream_t)stream;
  TilePlan tp = plan_tiles(F, {ldx, ldo}, {X, out, w});
  const bool has_w = g->ew != nullptr;
  const int blocks = grid_for(g->n_items);
  for (int64_t f0 = 0; f0 < F; f0 += tp.tile) {
    const int Ft = (int)std::min<int64_t>(tp.tile, F - f0);
    auto go = [&](auto nc_c, auto w_c, auto hw_c, auto norm_c) -> int {
      constexpr int NC = decltype(nc_c)::value;
      constexpr int W = decltype(w_c)::value;
      constexpr bool HW = decltype(hw_c)::value;
      constexpr int NORM = decltype(norm_c)::value;
      hipLaunchKernelGGL((sum_kernel<W, NC, HW, NORM>), dim3(blocks), dim3(kBlock), 0, st, g->ptr,
                         g->col, g->eslot, g->ew, norm_ptr, (const int4*)g->items, (int)g->n_items,
                         X + f0, ldx, Ft, out + f0, ldo, w ? w + f0 : nullptr, ldw);
      return PG_OK;
    };
    auto by_norm = [&](auto nc_c, auto w_c, auto hw_c) -> int {
      switch (norm_mode) {
        case 0: return go(nc_c, w_c, hw_c, std::integral_constant<int, 0>{});
        case 1: return go(nc_c, w_c, hw_c, std::integral_constant<int, 1>{});
        default: return go(nc_c, w_c, hw_c, std::integral_constant<int, 2>{});
      }
    };
    int rc;
    if (tp.vec) {
      const int nc = (Ft + 255) / 256;
      rc = has_w ? dispatch_nc_vec(nc, [&](auto n) { return by_norm(n, std::integral_constant<int, 4>{}, std::true_type{}); })
                 : dispatch_nc_vec(nc, [&](auto n) { return by_norm(n, std::integral_constant<int, 4>{}, std::false_type{}); });
    } else {
      const int nc = (Ft + 63) / 64;
      rc = has_w ? dispatch_nc_scalar(nc, [&](auto n) { return by_norm(n, std::integral_constant<int, 1>{}, std::true_type{}); })
                 : dispatch_nc_scalar(nc, [&](auto n) { return by_norm(n, std::integral_constant<int, 1>{}, std::false_type{}); });
    }
    if (rc != PG_OK) return pg::set_error(rc, "pg_spmm_sum: unsupported feature tile");
    if (g->n_merges > 0)
      hipLaunchKernelGGL(sum_merge_kernel<float>, dim3((unsigned)g->n_merges), dim3(kBlock), 0, st,
                         (const int4*)g->merges, (int)g->n_merges, Ft, w + f0, ldw, g->ptr,
                         norm_mode == 1 ? 1 : 0, nullptr, 0, out + f0, ldo);
  }
  return hip_status("pg_spmm_sum");
}

int pg_argpos_to_src(const pg_csr_t* g, const void* argpos, int64_t lda, int arg_kind,
                     int64_t F, int64_t* argx, int64_t ldx, pg_stream_t stream) {
  PG_TRY(pg::check_csr(g, "pg_argpos_to_src", false));
  if (!pg::valid_arg_kind(arg_kind))
    return pg::set_error(PG_ERR_INVALID, "pg_argpos_to_src: bad arg_kind %d", arg_kind);
  if (F < 0 || lda < F || ldx < F)
    return pg::set_error(PG_ERR_INVALID, "pg_argpos_to_src: bad F/leading dims");
  const int64_t n = g->n_rows * F;
  if (n == 0) return pg::ok();
  const int blocks = (int)std::min<int64_t>(4096, (n + kBlock - 1) / kBlock);
  hipStream_t st = (hipStream_t)stream;
  if (arg_kind == PG_ARG_U16)
    hipLaunchKernelGGL((argpos_to_src_kernel<uint16_t>), dim3(blocks), dim3(kBlock), 0, st, g->ptr,
                       g->col, g->n_rows, (const uint16_t*)argpos, lda, (int)F, argx, ldx);
  else
    hipLaunchKernelGGL((argpos_to_src_kernel<int32_t>), dim3(blocks), dim3(kBlock), 0, st, g->ptr,
                       g->col, g->n_rows, (const int32_t*)argpos, lda, (int)F, argx, ldx);
  return hip_status("pg_argpos_to_src");
}

}  // extern "C"
