// The optimizer's per-step scalars (torch 1.10 Adam, code/train.py:180, 205): state[0] the
// step count (incremented here), state[1] = lr / (1 - beta1^step), state[2] =
// sqrt(1 - beta2^step), formed in double and rounded to float once, like torch's scalar
// arguments. One thread runs it once per step, before pg_adam_apply (dense.hip's
// adam_prepare_kernel, or the fused head's final kernel, head.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace pg_adam {

__device__ __forceinline__ void step_scalars(float* state, double lr, double beta1, double beta2) {
  const float step = state[0] + 1.f;
  state[0] = step;
  const double bc1 = 1.0 - pow(beta1, (double)step);
  const double bc2 = 1.0 - pow(beta2, (double)step);
  state[1] = (float)(lr / bc1);  // step_size
  state[2] = (float)sqrt(bc2);   // sqrt(bias_correction2)
}

// one element's update (torch 1.10 Adam, _functional.adam): m, v and p written back, the new
// p returned. step_size = state[1], bc2s = state[2]; a1 = 1 - beta1, a2 = 1 - beta2.
__device__ __forceinline__ float elem(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                      float* __restrict__ v, int64_t i, float step_size, float bc2s, float beta1,
                                      float beta2, float a1, float a2, float eps, float wd) {
  float gi = g[i];
  if (wd != 0.f) gi = gi + wd * p[i];
  const float mi = m[i] * beta1 + a1 * gi;        // exp_avg.mul_(b1).add_(g, alpha=1-b1)
  const float vi = v[i] * beta2 + a2 * gi * gi;   // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
  const float denom = sqrtf(vi) / bc2s + eps;     // (sqrt / sqrt(bc2)).add_(eps)
  const float pi = p[i] + (-step_size) * (mi / denom);  // addcdiv_(m, denom, -step_size)
  p[i] = pi;
  m[i] = mi;
  v[i] = vi;
  return pi;
}

}  // namespace pg_adam
