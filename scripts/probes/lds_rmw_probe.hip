// Probe: throughput of LDS read-modify-write forms on gfx950, and which lane's value a
// plain LDS store keeps when several lanes of one instruction store to the same word.
// Build: hipcc --offload-arch=gfx950 -O3 -o lds_rmw_probe lds_rmw_probe.hip
// Each wave keeps a 256-float row in LDS and applies 64-lane groups whose addresses are
// random over the row (the max backward's stream pass: records of one source, features
// drawn from F = 256, so a group has a few same-address pairs).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kIters = 4096;

__device__ __forceinline__ unsigned hash(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

template <int MODE>
__global__ __launch_bounds__(256) void rmw_kernel(float* out, int fmask) {
  __shared__ float acc[4][256 + 64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* a = acc[wave];
  for (int f = lane; f < 256 + 64; f += 64) a[f] = 0.f;
  __builtin_amdgcn_wave_barrier();
  unsigned seed = hash(blockIdx.x * 256 + threadIdx.x);
  for (int it = 0; it < kIters; ++it) {
    seed = hash(seed + it);
    const int f = (int)(seed & (unsigned)fmask);
    const float v = (float)(seed >> 24) * 1e-3f;
    if constexpr (MODE == 0) {  // ds_add_f32 (no return)
      atomicAdd(&a[f], v);
    } else if constexpr (MODE == 1) {  // ds_add_u32 (no return)
      atomicAdd(reinterpret_cast<unsigned*>(&a[f]), (unsigned)(seed >> 28));
    } else if constexpr (MODE == 2) {  // ds_min_u32 (no return)
      atomicMin(reinterpret_cast<unsigned*>(&a[f]), (unsigned)lane);
    } else if constexpr (MODE == 3) {  // plain store
      a[f] = v;
    } else if constexpr (MODE == 4) {  // read, add, store (wrong under conflicts: timing only)
      a[f] = a[f] + v;
    } else {  // tag rounds: store the lane id, read it back, the survivors add (timing)
      reinterpret_cast<int*>(a)[f] = lane;
      __builtin_amdgcn_wave_barrier();
      if (reinterpret_cast<int*>(a)[f] == lane) a[f + 0] = a[f] + v;
    }
  }
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) out[blockIdx.x * 4 + wave] = a[7];
}

// which lane's value survives a same-word store: rec[trial] = 1 if the highest colliding
// lane always won, 2 if the lowest always won, 0 otherwise
__global__ __launch_bounds__(64) void order_kernel(int* rec, int trials) {
  __shared__ int tag[256];
  const int lane = threadIdx.x;
  for (int t = blockIdx.x; t < trials; t += gridDim.x) {
    const int f = (int)(hash(t * 64 + lane) & 31);  // 64 lanes over 32 words: many collisions
    tag[f] = -1;
    __builtin_amdgcn_wave_barrier();
    tag[f] = lane;
    __builtin_amdgcn_wave_barrier();
    const int won = tag[f];
    // the highest / lowest lane with the same f
    int hi = -1, lo = 64;
    for (int j = 0; j < 64; ++j) {
      const int fj = __shfl(f, j);
      if (fj == f) { hi = j > hi ? j : hi; lo = j < lo ? j : lo; }
    }
    const unsigned long long high_ok = __ballot(won == hi);
    const unsigned long long low_ok = __ballot(won == lo);
    if (lane == 0) rec[t] = (high_ok == ~0ull) ? 1 : (low_ok == ~0ull ? 2 : 0);
    __builtin_amdgcn_wave_barrier();
  }
}

template <int MODE>
float time_mode(float* out, int blocks, int fmask) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(rmw_kernel<MODE>, dim3(blocks), dim3(256), 0, 0, out, fmask);
  hipEventRecord(a);
  hipLaunchKernelGGL(rmw_kernel<MODE>, dim3(blocks), dim3(256), 0, 0, out, fmask);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 8;
  float* out;
  hipMalloc(&out, blocks * 4 * sizeof(float));
  const char* names[] = {"ds_add_f32", "ds_add_u32", "ds_min_u32", "store", "read+add+store", "tag round"};
  for (int fm : {255, 63}) {
    float t[6] = {time_mode<0>(out, blocks, fm), time_mode<1>(out, blocks, fm), time_mode<2>(out, blocks, fm),
                  time_mode<3>(out, blocks, fm), time_mode<4>(out, blocks, fm), time_mode<5>(out, blocks, fm)};
    const double instr = (double)blocks * 4 * kIters;  // wave instructions
    for (int m = 0; m < 6; ++m)
      printf("features %3d  %-16s %8.3f ms  %6.1f clk/instr per CU (2.4 GHz)\n", fm + 1, names[m], t[m],
             t[m] * 1e-3 * 2.4e9 / (instr / cus));
  }
  const int trials = 100000;
  int* rec;
  hipMalloc(&rec, trials * sizeof(int));
  hipLaunchKernelGGL(order_kernel, dim3(1024), dim3(64), 0, 0, rec, trials);
  std::vector<int> h(trials);
  hipMemcpy(h.data(), rec, trials * sizeof(int), hipMemcpyDeviceToHost);
  int n[3] = {0, 0, 0};
  for (int v : h) n[v]++;
  printf("same-word LDS stores over %d trials: highest lane kept %d, lowest kept %d, mixed %d\n", trials, n[1], n[2],
         n[0]);
  return 0;
}
