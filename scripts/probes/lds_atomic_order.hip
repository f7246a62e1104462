// Probe: in which order does one wave's ds_add_f32 apply lanes that hit the same LDS word?
// Each trial: 64 lanes, lane l adds v[l] (values chosen so the float sum depends on the
// order) to words addr[l] in {0..K-1}; the result is compared with the sums in ascending
// and in descending lane order. Build: hipcc --offload-arch=gfx950 -O2 lds_atomic_order.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kTrials = 4096;
constexpr int kWords = 8;

__global__ void probe(const float* v, const int* addr, float* out) {
  __shared__ float acc[4][kWords];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int t = blockIdx.x * 4 + w;
  if (lane < kWords) acc[w][lane] = 0.f;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  atomicAdd(&acc[w][addr[t * 64 + lane]], v[t * 64 + lane]);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (lane < kWords) out[t * kWords + lane] = acc[w][lane];
}

int main() {
  std::vector<float> v(kTrials * 64);
  std::vector<int> a(kTrials * 64);
  srand(7);
  for (int i = 0; i < kTrials * 64; ++i) {
    const float m = (rand() % 3 == 0) ? 1e7f : 1.f;
    v[i] = m * ((float)rand() / RAND_MAX - 0.5f);
    a[i] = rand() % ((i / 64) % 3 == 0 ? 1 : kWords);
  }
  float *dv, *dout;
  int* da;
  hipMalloc(&dv, v.size() * 4);
  hipMalloc(&da, a.size() * 4);
  hipMalloc(&dout, kTrials * kWords * 4);
  hipMemcpy(dv, v.data(), v.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(kTrials / 4), dim3(256), 0, 0, dv, da, dout);
  std::vector<float> o(kTrials * kWords);
  hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
  long asc = 0, desc = 0, other = 0, amb = 0;
  for (int t = 0; t < kTrials; ++t)
    for (int k = 0; k < kWords; ++k) {
      float sa = 0.f, sd = 0.f;
      for (int l = 0; l < 64; ++l)
        if (a[t * 64 + l] == k) sa += v[t * 64 + l];
      for (int l = 63; l >= 0; --l)
        if (a[t * 64 + l] == k) sd += v[t * 64 + l];
      const float g = o[t * kWords + k];
      if (sa == sd) { amb += g == sa; other += g != sa; continue; }
      if (g == sa) ++asc;
      else if (g == sd) ++desc;
      else ++other;
    }
  printf("words where the order shows: ascending-lane %ld, descending-lane %ld, neither %ld (order-free words matching %ld)\n",
         asc, desc, other, amb);
  return other == 0 && desc == 0 ? 0 : 1;
}
