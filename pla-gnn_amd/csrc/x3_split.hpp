// The three-piece bf16 split of f32 values shared by the three-piece GEMM (gemm_x3.hip) and
// the fused MLP head (head.hip): a = a_h + a_m + a_l, each piece the round-to-nearest bf16
// of what the previous pieces leave (v_cvt_pk_bf16_f32). Elementwise, so any kernel that
// splits the same values and issues the same MFMA sequence gets bitwise the same products.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace pg_x3 {

using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using bf16x2 = __attribute__((ext_vector_type(2))) __bf16;
using f32x16 = __attribute__((ext_vector_type(16))) float;

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  const bf16x2 v = {static_cast<__bf16>(a), static_cast<__bf16>(b)};  // v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(uint32_t, v);
}
// low bf16 of a packed pair widened to f32 by v_perm_b32 (the shift form gets rewritten into
// an extra cvt)
__device__ __forceinline__ float lo_f(uint32_t p) { return __uint_as_float(__builtin_amdgcn_perm(0u, p, 0x01000c0cu)); }
__device__ __forceinline__ float hi_f(uint32_t p) { return __uint_as_float(p & 0xFFFF0000u); }

// three-piece split of 4 floats: out[piece] = 4 bf16 (8 B)
__device__ __forceinline__ void split4(const float4 v, uint2 (&out)[3]) {
  float r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int piece = 0; piece < 3; ++piece) {
    const uint32_t p0 = pk_bf16(r[0], r[1]), p1 = pk_bf16(r[2], r[3]);
    out[piece] = make_uint2(p0, p1);
    if (piece < 2) {
      r[0] = r[0] - lo_f(p0); r[1] = r[1] - hi_f(p0);
      r[2] = r[2] - lo_f(p1); r[3] = r[3] - hi_f(p1);
    }
  }
}

// A raw buffer descriptor (wave-uniform: built from readfirstlane'd inputs, so the compiler
// keeps it in SGPRs) covering `bytes` from P: loads at byte offsets past the range return 0.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* P, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(P);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* base = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// the six products of one 32 x 32 x 16 block, small terms first: (h,l) (l,h) (m,m) (h,m) (m,h) (h,h)
__device__ __forceinline__ void mfma6(f32x16& acc, const bf16x8 (&a)[3], const bf16x8 (&b)[3]) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
}

}  // namespace pg_x3
