// Micro-probe: sustained v_mfma_f32_32x32x2_f32 rate for NACC independent accumulation
// chains per wave, optionally with a ds_read_b128 + barrier step every 32 MFMAs (the shape of
// the GEMM K step). Prints TFLOP/s. Build: hipcc --offload-arch=gfx950 -O3 mfma_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
using f32x16 = __attribute__((ext_vector_type(16))) float;

template <int NACC, int MODE>
__global__ __launch_bounds__(256) void probe(float* out, int iters, float x) {
  __shared__ __attribute__((aligned(16))) float lds[256 * 36];
  f32x16 acc[NACC];
  for (int i = 0; i < NACC; ++i) for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  const int tid = threadIdx.x;
  lds[tid] = x;
  __syncthreads();
  float a = x + tid, b = x - tid;
  constexpr int PER = 32 / NACC;  // MFMAs per chain per step -> 32 MFMAs per step
  if constexpr (MODE >= 3) {
    // GEMM-shaped step: TM x TN = NACC tiles (TN = 1 or 2), 16 k-values per lane from
    // [row][36] LDS images, 16 * NACC MFMAs per step (x2 steps per iteration -> 32 * NACC)
    constexpr int TM = NACC >= 2 ? 2 : 1, TN = NACC / TM;
    const int l32 = tid & 31, h = (tid >> 5) & 1, wave = tid >> 6;
    for (int i = tid; i < 256 * 36; i += 256) {
      unsigned hsh = (unsigned)i * 2654435761u + (unsigned)blockIdx.x * 40503u;
      hsh ^= hsh >> 13; hsh *= 0x5bd1e995u; hsh ^= hsh >> 15;
      lds[i] = x * ((float)(hsh & 0xffffff) / 16777216.0f - 0.5f);  // uniform [-0.5, 0.5)
    }
    __syncthreads();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        float fa[TM][16], fb[TN][16];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 t = *reinterpret_cast<const float4*>(lds + ((wave & 1) * 64 + i * 32 + l32) * 36 + h * 16 + 4 * q);
            fa[i][4 * q] = t.x; fa[i][4 * q + 1] = t.y; fa[i][4 * q + 2] = t.z; fa[i][4 * q + 3] = t.w;
          }
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 t = *reinterpret_cast<const float4*>(lds + 128 * 36 + ((wave >> 1) * 64 + j * 32 + l32) * 36 + h * 16 + 4 * q);
            fb[j][4 * q] = t.x; fb[j][4 * q + 1] = t.y; fb[j][4 * q + 2] = t.z; fb[j][4 * q + 3] = t.w;
          }
#pragma unroll
        for (int s = 0; s < 16; ++s)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i * TN + j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc[i * TN + j], 0, 0, 0);
        __syncthreads();
        if constexpr (MODE == 4) {
          lds[(tid * 37) % (256 * 36)] = fa[0][half];
          __syncthreads();
        }
      }
    }
  } else
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE >= 1) {
      const float4 t = *reinterpret_cast<const float4*>(lds + ((tid & 31) * 36 + ((tid >> 5) & 1) * 16));
      a += t.x; b += t.y;
    }
    if constexpr (MODE == 2) __syncthreads();
#pragma unroll
    for (int s = 0; s < PER; ++s)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  }
  float t = 0.f;
  for (int i = 0; i < NACC; ++i) for (int r = 0; r < 16; ++r) t += acc[i][r];
  out[blockIdx.x * 256 + tid] = t;
}

template <int NACC, int MODE>
void run(int blocks_per_cu) {
  const int blocks = 256 * blocks_per_cu, iters = 2000;
  float* out;
  hipMalloc(&out, blocks * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  probe<NACC, MODE><<<blocks, 256>>>(out, 10, 1.f);
  hipEventRecord(e0);
  probe<NACC, MODE><<<blocks, 256>>>(out, iters, 1.f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double per = MODE >= 3 ? 32.0 * NACC : 32.0;  // MFMAs per wave per iteration
  const double fl = 2.0 * 32 * 32 * 2 * per * iters * 4 * blocks;
  printf("nacc %d mode %d blocks/cu %d: %.1f TF\n", NACC, MODE, blocks_per_cu, fl / ms / 1e9);
  hipFree(out);
}

int main() {
  for (int b : {1, 2, 3}) {
    run<2, 3>(b); run<4, 3>(b);
    run<2, 4>(b); run<4, 4>(b);
  }
  return 0;
}
