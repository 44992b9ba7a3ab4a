// Scrambled-Sobol N(0,1) base samples on the GPU.
//
// Reference: SobolQMCNormalSampler._construct_base_samples
// (botorch/sampling/normal.py:178-209) -> draw_sobol_normal_samples
// (botorch/utils/sampling.py:108-137) -> NormalQMCEngine(inv_transform=True)
// (botorch/sampling/qmc.py:60-98) over torch.quasirandom.SobolEngine
// (scramble=True, seed).  The scrambled direction numbers (dim x 30) and the
// digital shift are the engine's own state; point k of the sequence is
//   u_k = (shift XOR  XOR_{bit b of gray(k)} v_b) * 2^-30,   gray(k) = k ^ (k >> 1)
// (point 0 = shift), which is what the engine's sequential Gray-code update
// produces, so every point is generated independently in parallel.
//   z = sqrt(2) erfinv(2 v - 1),  v = 1/2 + (1 - eps)(u - 1/2).
#include "common.h"

namespace {

constexpr int MAXBIT = 30;

__global__ void sobol_normal_kernel(const int64_t* __restrict__ state,
                                    const int64_t* __restrict__ shift, int dim, int64_t n,
                                    int64_t skip, double* __restrict__ out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * dim) return;
  const int64_t i = idx / dim + skip;
  const int j = (int)(idx % dim);
  const uint64_t g = (uint64_t)i ^ ((uint64_t)i >> 1);
  int64_t v = shift[j];
  const int64_t* sj = state + (int64_t)j * MAXBIT;
#pragma unroll
  for (int b = 0; b < MAXBIT; ++b)
    if ((g >> b) & 1ull) v ^= sj[b];
  const double u = (double)v * (1.0 / 1073741824.0);
  const double eps = 2.220446049250313e-16;
  const double vv = 0.5 + (1.0 - eps) * (u - 0.5);
  out[idx] = erfinv(2.0 * vv - 1.0) * 1.4142135623730951;
}

}  // namespace

extern "C" int bo_sobol_normal(const int64_t* state, const int64_t* shift, int dim, int64_t n,
                               int64_t skip, double* out, void* stream) {
  BO_CHECK_ARG(dim > 0 && n >= 0 && skip >= 0, "bo_sobol_normal: bad shape");
  const int64_t tot = n * dim;
  if (tot == 0) return BO_OK;
  sobol_normal_kernel<<<(unsigned)ceil_div(tot, 256), 256, 0, as_stream(stream)>>>(
      state, shift, dim, n, skip, out);
  BO_LAUNCH_CHECK();
  return BO_OK;
}
