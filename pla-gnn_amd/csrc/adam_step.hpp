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

}  // namespace pg_adam
