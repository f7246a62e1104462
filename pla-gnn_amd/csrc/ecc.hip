// Edge clustering coefficient on the GPU: the reference's
// edge_clustering_coefficients (code/data_preprocess.py:175-214) for a symmetric
// adjacency in CSR form with sorted, unique column ids:
//   ecc(i, j) = epsilon                    if min(deg_i, deg_j) - 1 == 0
//             = |N(i) ∩ N(j)| / (min(deg_i, deg_j) - 1)   otherwise (float64),
// deg = the row sums of the stored values (the reference's ppi[i].data.sum()).
//
// Each unordered pair {i, j} is counted once, by the row of larger degree (ties: larger
// id): that row's neighbour set is a bitmap over node ids in LDS and the other row's
// list is streamed against it, so a pair costs min(deg_i, deg_j) bit tests and a hub
// never streams its own long list per neighbour. The value is written to the pair's
// entry in both rows (mirror[k] = the index of the transposed entry). Persistent
// workgroups walk the rows (longest first) and clear only the bits they set, so the
// bitmap is zeroed once per workgroup. Integer counts and one f64 division per pair:
// bit-exact against the reference.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.hpp"

namespace {

constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void ecc_kernel(
    const int32_t* __restrict__ ptr, const int32_t* __restrict__ col,
    const int32_t* __restrict__ mirror, const double* __restrict__ deg,
    const int32_t* __restrict__ order, int64_t n, int words, double epsilon,
    double* __restrict__ ecc) {
  extern __shared__ uint32_t bits[];
  for (int w = threadIdx.x; w < words; w += kBlock) bits[w] = 0u;
  __syncthreads();
  for (int64_t r = blockIdx.x; r < n; r += gridDim.x) {
    const int i = order ? order[r] : (int)r;
    const int s = ptr[i], e = ptr[i + 1];
    for (int k = s + threadIdx.x; k < e; k += kBlock) {
      const int c = col[k];
      atomicOr(&bits[c >> 5], 1u << (c & 31));
    }
    __syncthreads();
    const double di = deg ? deg[i] : (double)(e - s);
    for (int k = s + threadIdx.x; k < e; k += kBlock) {
      const int j = col[k];
      if (j == i) {
        ecc[k] = 0.0;  // a diagonal entry is not an ECC entry (the reference skips j <= i)
        continue;
      }
      const int sj = ptr[j], ej = ptr[j + 1];
      const double dj = deg ? deg[j] : (double)(ej - sj);
      const int li = e - s, lj = ej - sj;
      // the pair belongs to the longer row (ties: the larger id)
      if (lj > li || (lj == li && j > i)) continue;
      int tri = 0;
      for (int q = sj; q < ej; ++q) {
        const int x = col[q];
        tri += (bits[x >> 5] >> (x & 31)) & 1u;
      }
      const double possible = fmin(di, dj) - 1.0;
      const double v = possible == 0.0 ? epsilon : (double)tri / possible;
      ecc[k] = v;
      ecc[mirror[k]] = v;
    }
    __syncthreads();
    for (int k = s + threadIdx.x; k < e; k += kBlock) {
      const int c = col[k];
      bits[c >> 5] = 0u;
    }
    __syncthreads();
  }
}

}  // namespace

extern "C" {

int pg_ecc(const int32_t* ptr, const int32_t* col, const int32_t* mirror, const double* deg,
           const int32_t* order, int64_t n, int64_t nnz, double epsilon, double* ecc,
           pg_stream_t stream) {
  if (n < 0 || nnz < 0 || n > (int64_t)1 << 22)
    return pg::set_error(PG_ERR_INVALID, "pg_ecc: n must be in [0, 2^22] (LDS bitmap)");
  if (n == 0 || nnz == 0) return pg::ok();
  if (!ptr || !col || !mirror || !ecc) return pg::set_error(PG_ERR_INVALID, "pg_ecc: NULL buffer");
  const int words = (int)((n + 31) / 32);
  const size_t lds = (size_t)words * 4;
  if (lds > 160 * 1024) return pg::set_error(PG_ERR_UNSUPPORTED, "pg_ecc: bitmap exceeds LDS");
  hipStream_t st = (hipStream_t)stream;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)ecc_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  // persistent workgroups: as many as fit (LDS-bound), at most one per row
  const int per_cu = std::max(1, std::min(8, (int)((160 * 1024) / std::max<size_t>(lds, 1))));
  const int blocks = (int)std::min<int64_t>(n, 256 * per_cu);
  hipLaunchKernelGGL(ecc_kernel, dim3(blocks), dim3(kBlock), lds, st, ptr, col, mirror, deg,
                     order, n, words, epsilon, ecc);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return pg::set_error((int)err, "pg_ecc: launch failed: %s", hipGetErrorString(err));
  return pg::ok();
}

}  // extern "C"
