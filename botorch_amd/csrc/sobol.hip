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

// erfinv to ~1 ulp (torch's CPU erfinv is that accurate; the device library's
// double erfinv is not -- measured 3.7e-7 relative near 0 on gfx950): Giles'
// single-precision rational start, then three Halley steps on erf (erfc in
// the tails, where 1 - |y| is exact and erf would cancel).
__device__ double erfinv_accurate(double y) {
  const double ay = fabs(y);
  if (ay >= 1.0) return ay == 1.0 ? copysign(INFINITY, y) : NAN;
  double w = -log((1.0 - y) * (1.0 + y));
  double p;
  if (w < 5.0) {
    w -= 2.5;
    p = 2.81022636e-08;
    p = 3.43273939e-07 + p * w;
    p = -3.5233877e-06 + p * w;
    p = -4.39150654e-06 + p * w;
    p = 0.00021858087 + p * w;
    p = -0.00125372503 + p * w;
    p = -0.00417768164 + p * w;
    p = 0.246640727 + p * w;
    p = 1.50140941 + p * w;
  } else {
    w = sqrt(w) - 3.0;
    p = -0.000200214257;
    p = 0.000100950558 + p * w;
    p = 0.00134934322 + p * w;
    p = -0.00367342844 + p * w;
    p = 0.00573950773 + p * w;
    p = -0.0076224613 + p * w;
    p = 0.00943887047 + p * w;
    p = 1.00167406 + p * w;
    p = 2.83297682 + p * w;
  }
  double x = p * y;
  const double k = 1.1283791670955126;  // 2 / sqrt(pi)
  for (int it = 0; it < 3; ++it) {
    // erf(x) - y, written through erfc in the tails:  y > 0: (1 - y) - erfc(x),
    // y < 0: erfc(|x|) - (1 - |y|).
    const double f = (ay < 0.5) ? erf(x) - y
                                : (erfc(fabs(x)) - (1.0 - ay)) * (y < 0.0 ? 1.0 : -1.0);
    const double fp = k * exp(-x * x);
    x = x - f / (fp + x * f);
  }
  return x;
}

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
  // Same op order as the reference (no fma contraction): v = 1/2 + (1-eps)(u-1/2).
  const double t = __dmul_rn(1.0 - eps, u - 0.5);
  const double vv = __dadd_rn(0.5, t);
  out[idx] = erfinv_accurate(__dsub_rn(__dmul_rn(2.0, vv), 1.0)) * 1.4142135623730951;
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
