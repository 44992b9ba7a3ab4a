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

// Maclaurin series of erf for |x| <= 0.5 (terms fall by >= 4x: converged to
// the last bit in < 25 terms).
__device__ double erf_series(double x) {
  const double x2 = x * x;
  double term = x, sum = x;
  for (int n = 1; n < 40; ++n) {
    term *= -x2 / n;
    const double c = term / (2 * n + 1);
    sum += c;
    if (fabs(c) <= 1e-18 * fabs(sum)) break;
  }
  return 1.1283791670955126 * sum;
}

// erfinv to ~1 ulp (torch's CPU erfinv is that accurate; the device library's
// double erfinv is not -- measured 3.7e-7 relative near 0 on gfx950).  Start:
// Giles' single-precision rational form, or for 1 - |y| < 1e-6 the asymptotic
// erfc(x) ~ exp(-x^2) / (x sqrt(pi)); then Halley steps to convergence on
// erf(x) - y through the series for |y| < 1/2, and on erfc(|x|) - (1 - |y|)
// in the tails (1 - |y| is exact there, erf would cancel).
__device__ double erfinv_accurate(double y) {
  const double ay = fabs(y);
  if (ay >= 1.0) return ay == 1.0 ? copysign(INFINITY, y) : NAN;
  if (ay == 0.0) return y;
  const double t = 1.0 - ay;  // exact for ay >= 1/2
  double x;                   // |erfinv(y)|
  if (t < 1e-6) {
    x = sqrt(-log(t));
    for (int i = 0; i < 4; ++i) x = sqrt(-log(t * x * 1.7724538509055160273));
  } else {
    double w = -log((1.0 - ay) * (1.0 + ay));
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
    x = p * ay;
  }
  const double k = 1.1283791670955126;  // 2 / sqrt(pi)
  for (int it = 0; it < 60; ++it) {
    // g(x) = erf(x) - |y|  (= t - erfc(x) in the tails), g' = k exp(-x^2), g'' = -2 x g'
    const double g = (ay < 0.5) ? erf_series(x) - ay : t - erfc(x);
    const double gp = k * exp(-x * x);
    const double dx = g / (gp + x * g);
    x -= dx;
    if (fabs(dx) <= 2e-16 * fabs(x)) break;
  }
  return copysign(x, y);
}

__global__ void sobol_normal_kernel(const int64_t* __restrict__ state,
                                    const int64_t* __restrict__ shift, int dim, int64_t n,
                                    int64_t skip, int first_f32, double* __restrict__ out) {
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
  // torch's SobolEngine returns its first point as _first_point = quasi / 2**30
  // computed at construction in the default dtype (float32 unless changed),
  // so point 0 carries float32 rounding; every later point is exact.
  const double u = (i == 0 && first_f32) ? (double)((float)v) * (1.0 / 1073741824.0)
                                         : (double)v * (1.0 / 1073741824.0);
  const double eps = 2.220446049250313e-16;
  // Same op order as the reference (no fma contraction): v = 1/2 + (1-eps)(u-1/2).
  const double t = __dmul_rn(1.0 - eps, u - 0.5);
  const double vv = __dadd_rn(0.5, t);
  out[idx] = erfinv_accurate(__dsub_rn(__dmul_rn(2.0, vv), 1.0)) * 1.4142135623730951;
}

// Box-scaled raw designs: out[i][j] = lower[j % d] + range[j % d] * u_i[j]
// (draw_sobol_samples, botorch/utils/sampling.py:66-105: engine over q*d
// dimensions, draw(n, dtype=double), then lower + rng * raw -- product and sum
// rounded separately, as torch evaluates them).
__global__ void sobol_box_kernel(const int64_t* __restrict__ state,
                                 const int64_t* __restrict__ shift, int dim, int64_t n,
                                 int64_t skip, int first_f32, const double* __restrict__ lower,
                                 const double* __restrict__ range, int d,
                                 double* __restrict__ out) {
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
  const double u = (i == 0 && first_f32) ? (double)((float)v) * (1.0 / 1073741824.0)
                                         : (double)v * (1.0 / 1073741824.0);
  const int t = j % d;
  out[idx] = __dadd_rn(lower[t], __dmul_rn(range[t], u));
}

// Owen-type scramble of the direction numbers, as SobolEngine(scramble=True)
// applies it at construction (torch/quasirandom.py _scramble +
// torch._sobol_engine_scramble_): with L_d the random lower-triangular 30 x 30
// bit matrix of dimension d (unit diagonal) and row p packed MSB-first
// (bit 29 - k = L_d[p][k]),
//   state[d][j] bit (29 - p) = parity(L_d[p] & state0[d][j]),
//   shift[d] = sum_k s[d][k] 2^k.
// `bits` holds the engine's two randint draws in order: the dim x 30 shift bits,
// then the dim x 30 x 30 matrix bits (taken below/on the diagonal only).  One
// workgroup scrambles SDIM dimensions: the packed rows go through LDS.
constexpr int SDIM = 8;

__global__ void __launch_bounds__(256) sobol_scramble_kernel(
    int dim, const int64_t* __restrict__ state0, const uint8_t* __restrict__ bits,
    int64_t* __restrict__ state, int64_t* __restrict__ shift) {
  __shared__ unsigned rows[SDIM][MAXBIT];
  const int t = threadIdx.x;
  const int dl = t / MAXBIT, r = t % MAXBIT;
  const int d = blockIdx.x * SDIM + dl;
  const bool live = t < SDIM * MAXBIT && d < dim;
  if (live) {
    const uint8_t* row = bits + (int64_t)dim * MAXBIT + ((int64_t)d * MAXBIT + r) * MAXBIT;
    unsigned packed = 1u << (MAXBIT - 1 - r);
    for (int k = 0; k < r; ++k) packed |= (unsigned)(row[k] & 1) << (MAXBIT - 1 - k);
    rows[dl][r] = packed;
  }
  __syncthreads();
  if (!live) return;
  const unsigned v = (unsigned)state0[(int64_t)d * MAXBIT + r];
  unsigned out = 0;
#pragma unroll
  for (int p = 0; p < MAXBIT; ++p) out |= (unsigned)(__popc(rows[dl][p] & v) & 1) << (MAXBIT - 1 - p);
  state[(int64_t)d * MAXBIT + r] = (int64_t)out;
  if (r == 0) {
    int64_t s = 0;
    const uint8_t* sb = bits + (int64_t)d * MAXBIT;
    for (int k = 0; k < MAXBIT; ++k) s |= (int64_t)(sb[k] & 1) << k;
    shift[d] = s;
  }
}

}  // namespace

extern "C" int bo_sobol_scramble(int dim, const int64_t* state0, const uint8_t* bits,
                                 int64_t* state, int64_t* shift, void* stream) {
  BO_CHECK_ARG(dim > 0, "bo_sobol_scramble: bad dimension %d", dim);
  sobol_scramble_kernel<<<(unsigned)ceil_div(dim, SDIM), 256, 0, as_stream(stream)>>>(
      dim, state0, bits, state, shift);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

extern "C" int bo_sobol_box(const int64_t* state, const int64_t* shift, int dim, int64_t n,
                            int64_t skip, int first_f32, const double* lower, const double* range,
                            int d, double* out, void* stream) {
  BO_CHECK_ARG(dim > 0 && n >= 0 && skip >= 0 && d > 0 && dim % d == 0,
               "bo_sobol_box: bad shape (dim %d, d %d)", dim, d);
  const int64_t tot = n * dim;
  if (tot == 0) return BO_OK;
  sobol_box_kernel<<<(unsigned)ceil_div(tot, 256), 256, 0, as_stream(stream)>>>(
      state, shift, dim, n, skip, first_f32, lower, range, d, out);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

extern "C" int bo_sobol_normal(const int64_t* state, const int64_t* shift, int dim, int64_t n,
                               int64_t skip, int first_f32, double* out, void* stream) {
  BO_CHECK_ARG(dim > 0 && n >= 0 && skip >= 0, "bo_sobol_normal: bad shape");
  const int64_t tot = n * dim;
  if (tot == 0) return BO_OK;
  sobol_normal_kernel<<<(unsigned)ceil_div(tot, 256), 256, 0, as_stream(stream)>>>(
      state, shift, dim, n, skip, first_f32, out);
  BO_LAUNCH_CHECK();
  return BO_OK;
}
