// Device-resident multi-start L-BFGS-B: one 64-lane wave per restart runs the
// reverse-communication state machine of lbfgsb_core.h (scipy 1.15's L-BFGS-B,
// the optimiser of botorch's gen_candidates_scipy, botorch/generation/gen.py:
// 194-267) for one function evaluation per launch.
//
// The caller evaluates -acq and its gradient at every restart's trial point xt
// (one batched forward + backward of the fused acquisition kernels) and
// launches bo_lbfgsb_step, which consumes them and writes the next trial
// points.  Iterate, gradient, the compact-form memory (S, Y ring; SY, SS and
// the Cholesky factor of theta SS + L D^-1 L^T) and the line-search state stay
// in HBM between launches; the host reads only the status vector, every few
// evaluations.  Vector work (dot products over n = q d, the Cauchy breakpoint
// search, the free-set products of formk) is spread over the wave's lanes; the
// 2m x 2m algebra runs on lane 0 in LDS.  A restart that has stopped keeps
// xt = x, so it costs nothing but its slot in the batched evaluation.
#include "common.h"

#include <atomic>
#include <cstdlib>
#include <mutex>

// No multiply-add contraction: scipy's L-BFGS-B rounds every product and sum
// separately, and a fused a*b+c flips borderline line-search tests (measured:
// one restart in 16 took another trial point after 14 evaluations).  The step
// is latency-bound scalar work; the FMAs saved nothing.
#pragma clang fp contract(off)

// everything inlined into the kernel: a call keeps `this` (Step, Restart) on the
// stack, and every field access becomes a scratch load (374 of them)
#define BO_HD __device__ __attribute__((always_inline))
#include "lbfgsb_core.h"

namespace {

struct WaveCtx {
  static constexpr int NL = 64;
  int lane;
  __device__ void sync() { __syncthreads(); }
  __device__ unsigned long long clock() { return wall_clock64(); }
  __device__ double sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
  }
  __device__ double max(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
  }
  __device__ double min(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
  }
  __device__ void argmin(double& v, int& i) {  // ties to the smallest index
    for (int o = 32; o > 0; o >>= 1) {
      const double ov = __shfl_xor(v, o);
      const int oi = __shfl_xor(i, o);
      if (ov < v || (ov == v && oi < i)) {
        v = ov;
        i = oi;
      }
    }
  }
  __device__ int exscan(int v, int& total) {  // exclusive prefix sum in lane order
    int x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    total = __shfl(x, 63);
    return x - v;
  }
};

// NW waves as one lane context (NL = 64 NW lanes): the joint problem of
// gen.py:252-267 -- ONE L-BFGS-B over all restarts' b q d variables -- is a
// single restart with n in the thousands, so its dot products, breakpoint scans
// and formk products are spread over a whole workgroup.  Reductions: the wave
// butterfly, then the NW wave results through LDS in wave order (the same
// result on every lane, as WaveCtx's).
template <int NW_>
struct BlockCtx {
  static constexpr int NW = NW_;
  static constexpr int NL = 64 * NW;
  int lane;
  double* red;   // LDS, NW doubles
  int* redi;     // LDS, NW ints
  double* reds;  // LDS, NW x M2 doubles (sums)
  __device__ int wave() const { return lane >> 6; }
  __device__ int wlane() const { return lane & 63; }
  __device__ void sync() { __syncthreads(); }
  __device__ double wave_sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
  }
  // every entry of v summed over all NL lanes (waves in order), on every lane
  template <int K>
  __device__ void sums(double (&v)[K]) {
    static_assert(K <= bolb::M2, "sums: scratch holds M2 values per wave");
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = wave_sum(v[k]);
    __syncthreads();
    if (wlane() == 0)
#pragma unroll
      for (int k = 0; k < K; ++k) reds[wave() * bolb::M2 + k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {
      double r = reds[k];
      for (int w = 1; w < NW; ++w) r += reds[w * bolb::M2 + k];
      v[k] = r;
    }
  }
  __device__ int exscan(int v, int& total) {  // exclusive prefix sum in lane order
    int x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (wlane() >= o) x += y;
    }
    __syncthreads();
    if (wlane() == 63) redi[wave()] = x;
    __syncthreads();
    int before = 0;
    total = 0;
    for (int w = 0; w < NW; ++w) {
      if (w < wave()) before += redi[w];
      total += redi[w];
    }
    return before + x - v;
  }
  __device__ unsigned long long clock() { return wall_clock64(); }
  template <class F>
  __device__ double all(double v, F op) {
    for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o));
    __syncthreads();  // the previous reduction's reads are done
    if ((lane & 63) == 0) red[lane >> 6] = v;
    __syncthreads();
    double r = red[0];
    for (int w = 1; w < NW; ++w) r = op(r, red[w]);
    return r;
  }
  __device__ double sum(double v) { return all(v, [](double a, double b) { return a + b; }); }
  __device__ double max(double v) { return all(v, [](double a, double b) { return fmax(a, b); }); }
  __device__ double min(double v) { return all(v, [](double a, double b) { return fmin(a, b); }); }
  __device__ void argmin(double& v, int& i) {  // ties to the smallest index
    for (int o = 32; o > 0; o >>= 1) {
      const double ov = __shfl_xor(v, o);
      const int oi = __shfl_xor(i, o);
      if (ov < v || (ov == v && oi < i)) {
        v = ov;
        i = oi;
      }
    }
    __syncthreads();
    if ((lane & 63) == 0) {
      red[lane >> 6] = v;
      redi[lane >> 6] = i;
    }
    __syncthreads();
    v = red[0];
    i = redi[0];
    for (int w = 1; w < NW; ++w)
      if (red[w] < v || (red[w] == v && redi[w] < i)) {
        v = red[w];
        i = redi[w];
      }
  }
};

// Bytes of LDS a restart's working set takes (vectors, int vectors, S / Y ring).
inline size_t staged_bytes(int n, int m) {
  return sizeof(double) * ((size_t)bolb::V_COUNT * n + 2 * (size_t)m * n) +
         sizeof(int) * (size_t)bolb::IV_COUNT * n;
}
constexpr size_t STAGE_LIMIT = 64 * 1024 - sizeof(bolb::Shared);  // dynamic LDS budget
constexpr int JOINT_N = 1024;  // wider restarts run on a JOINT_W-wave workgroup
constexpr int JOINT_W = 8;
constexpr int JOINT_TB_LDS = 16384;  // breakpoints of a wide restart up to 128 KB of LDS

// One wave per restart.  With `staged`, the restart's vectors and ring are
// copied into LDS for the launch (coalesced, once) and back at the end: every
// dot product, breakpoint scan and formk product then reads LDS instead of
// chaining dependent HBM / L2 loads, which set the duration of the slowest
// restart (the launch's duration).
template <int NW>
__global__ __launch_bounds__(64 * NW) void lbfgsb_kernel(bolb::Problem P, double* __restrict__ xt,
                                                         const double* __restrict__ ft,
                                                         const double* __restrict__ gt,
                                                         double* __restrict__ v, int* __restrict__ iv,
                                                         double* __restrict__ ws,
                                                         double* __restrict__ wy,
                                                         double* __restrict__ mat,
                                                         double* __restrict__ ds, int* __restrict__ is,
                                                         int staged) {
  constexpr int NL = 64 * NW;
  __shared__ bolb::Shared S;
  __shared__ double red[NW];
  __shared__ int redi[NW];
  __shared__ double reds[NW > 1 ? NW * bolb::M2 : 1];
  extern __shared__ double lds_dyn[];
  const long b = blockIdx.x;
  const long n = P.n, m = P.m;
  const int lane = threadIdx.x;
  double* gv = v + b * bolb::V_COUNT * n;
  int* giv = iv + b * bolb::IV_COUNT * n;
  double* gws = ws + b * m * n;
  double* gwy = wy + b * m * n;
  bolb::Restart R{xt + b * n,
                  ft[b],
                  gt + b * n,
                  gv,
                  giv,
                  gws,
                  gwy,
                  mat + b * bolb::NMAT * bolb::MMAX * bolb::MMAX,
                  ds + b * bolb::DSLOTS,
                  is + b * bolb::ISLOTS};
  const long nv = bolb::V_COUNT * n, nr = m * n, ni = bolb::IV_COUNT * n;
  if (staged == 1) {
    double* lv = lds_dyn;
    double* lws = lv + nv;
    double* lwy = lws + nr;
    int* liv = reinterpret_cast<int*>(lwy + nr);
    for (long k = lane; k < nv; k += NL) lv[k] = gv[k];
    for (long k = lane; k < nr; k += NL) {
      lws[k] = gws[k];
      lwy[k] = gwy[k];
    }
    for (long k = lane; k < ni; k += NL) liv[k] = giv[k];
    __syncthreads();
    R.v = lv;
    R.ws = lws;
    R.wy = lwy;
    R.iv = liv;
  }
  if (staged == 2) R.tb_scratch = lds_dyn;  // the breakpoints in LDS (wide, unstaged)
  if constexpr (NW == 1) {
    WaveCtx c{lane};
    bolb::Step<WaveCtx> st(c, P, R, S);
    st.run(P.prof ? P.prof + b * bolb::PROF_SLOTS : nullptr);
  } else {
    BlockCtx<NW> c{lane, red, redi, reds};
    bolb::Step<BlockCtx<NW>> st(c, P, R, S);
    st.run(P.prof ? P.prof + b * bolb::PROF_SLOTS : nullptr);
  }
  if (staged == 1) {
    __syncthreads();
    for (long k = lane; k < nv; k += NL) gv[k] = R.v[k];
    for (long k = lane; k < nr; k += NL) {
      gws[k] = R.ws[k];
      gwy[k] = R.wy[k];
    }
    for (long k = lane; k < ni; k += NL) giv[k] = R.iv[k];
  }
}

}  // namespace

// phase clocks of the next launches (tools/prof_lbfgsb.py), B x PROF_SLOTS, or null.
// The buffer and its capacity change together under one mutex, so a launch on
// another thread reads a consistent pair (never a new capacity with the old,
// smaller buffer).
static std::mutex g_lbfgsb_prof_mu;
static unsigned long long* g_lbfgsb_prof = nullptr;
static int g_lbfgsb_prof_cap = 0;               // restarts the buffer holds
static std::atomic<int> g_lbfgsb_unstaged{0};   // 1: keep the working set in HBM (A/B timing)
extern "C" int bo_lbfgsb_set_profile(unsigned long long* prof, int capacity) {
  BO_CHECK_ARG(capacity >= 0, "bo_lbfgsb_set_profile: capacity %d", capacity);
  std::lock_guard<std::mutex> lk(g_lbfgsb_prof_mu);
  g_lbfgsb_prof = prof;
  g_lbfgsb_prof_cap = prof ? capacity : 0;
  return BO_OK;
}
static unsigned long long* lbfgsb_profile_for(int B) {
  std::lock_guard<std::mutex> lk(g_lbfgsb_prof_mu);
  return B <= g_lbfgsb_prof_cap ? g_lbfgsb_prof : nullptr;
}
extern "C" int bo_lbfgsb_set_staging(int on) {
  g_lbfgsb_unstaged.store(!on);
  return BO_OK;
}

// The grid-wide kernel of a single wide restart (lbfgsb_grid.hip).
bool lbfgsb_grid_fits(int n, int m);
int lbfgsb_grid_launch(const bolb::Problem& P, double* xt, const double* ft, const double* gt,
                       double* v, int* iv, double* ws, double* wy, double* mat, double* ds, int* is,
                       void* stream);
// 0: a single restart of at least GRID_MIN_N variables runs on the grid
// kernel (where it fits); 1: every single restart that fits does; -1: never
static std::atomic<int> g_lbfgsb_grid{0};
constexpr int GRID_MIN_N = 2048;
extern "C" int bo_lbfgsb_set_grid(int mode) {
  BO_CHECK_ARG(mode >= -1 && mode <= 1, "bo_lbfgsb_set_grid: mode %d (-1, 0 or 1)", mode);
  g_lbfgsb_grid.store(mode);
  return BO_OK;
}

extern "C" int bo_lbfgsb_layout(int* out) {
  out[0] = bolb::V_COUNT;
  out[1] = bolb::IV_COUNT;
  out[2] = bolb::NMAT * bolb::MMAX * bolb::MMAX;
  out[3] = bolb::DSLOTS;
  out[4] = bolb::ISLOTS;
  out[5] = bolb::MMAX;
  return BO_OK;
}

extern "C" int bo_lbfgsb_step(int B, int n, int m, int maxls, int maxiter, int maxfun, double ftol,
                              double pgtol, const double* lower, const double* upper, double* xt,
                              const double* ft, const double* gt, double* v, int* iv, double* ws,
                              double* wy, double* mat, double* ds, int* is, void* stream) {
  BO_CHECK_ARG(B >= 0 && n >= 1 && m >= 1 && m <= bolb::MMAX && maxls >= 1,
               "bo_lbfgsb_step: B=%d n=%d m=%d (1..%d) maxls=%d", B, n, m, bolb::MMAX, maxls);
  BO_CHECK_ARG(lower && upper && xt && ft && gt && v && iv && ws && wy && mat && ds && is,
               "bo_lbfgsb_step: null buffer");
  if (B == 0) return BO_OK;
  // profile only launches the buffer can hold (B x PROF_SLOTS clocks)
  unsigned long long* prof = lbfgsb_profile_for(B);
  bolb::Problem P{n, m, maxls, maxiter, maxfun, ftol, pgtol, lower, upper, prof};
  // the joint problem (one restart of b q d variables) over the chip
  const int gmode = g_lbfgsb_grid.load();
  if (B == 1 && gmode >= 0 && (gmode == 1 || n >= GRID_MIN_N) && lbfgsb_grid_fits(n, m))
    return lbfgsb_grid_launch(P, xt, ft, gt, v, iv, ws, wy, mat, ds, is, stream);
  const size_t bytes = staged_bytes(n, m);
  const int staged = bytes <= STAGE_LIMIT && !g_lbfgsb_unstaged.load();
  // one wave per restart; a restart wider than the wave's working set (the
  // joint problem over all restarts, n = b q d) takes an 8-wave workgroup
  if (n <= JOINT_N)
    lbfgsb_kernel<1><<<B, 64, staged ? bytes : 0, as_stream(stream)>>>(P, xt, ft, gt, v, iv, ws, wy,
                                                                       mat, ds, is, staged);
  else {
    // an unstaged wide restart keeps the Cauchy breakpoints in LDS (staged = 2)
    const int mode = staged ? 1 : (n <= JOINT_TB_LDS ? 2 : 0);
    const size_t dyn = mode == 1 ? bytes : (mode == 2 ? sizeof(double) * (size_t)n : 0);
    // the attribute is per device: set it once for each device this process
    // launches the joint kernel on, and report a refusal here, not as a
    // launch failure later
    // 16 waves past n = 8192 (C3's joint problem, n = 12288: 813 -> 695 us per
    // launch, optimize_acqf 76.9 -> 72.8 ms; C2's n = 3072 is faster on 8,
    // 205 against 244 us: its reductions' LDS rounds outweigh the wider
    // vector loops); BO_LBFGSB_JOINT_W=8 / 16 forces either (A/B knob)
    static const int wenv = [] {
      const char* e = getenv("BO_LBFGSB_JOINT_W");
      return e ? atoi(e) : 0;
    }();
    const bool w16 = wenv == 16 || (wenv != 8 && n > 8192);
    const void* fn = w16 ? reinterpret_cast<const void*>(&lbfgsb_kernel<16>)
                         : reinterpret_cast<const void*>(&lbfgsb_kernel<JOINT_W>);
    if (dyn > 64 * 1024) {
      int dev = 0;
      BO_HIP(hipGetDevice(&dev));
      static std::mutex mu;
      static uint64_t set_mask[2] = {0, 0};  // per kernel variant (8 / 16 waves)
      std::lock_guard<std::mutex> lock(mu);
      const uint64_t bit = dev < 64 ? (uint64_t(1) << dev) : 0;
      if (!bit || !(set_mask[w16] & bit)) {
        BO_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)(sizeof(double) * JOINT_TB_LDS)));
        set_mask[w16] |= bit;
      }
    }
    if (w16)
      lbfgsb_kernel<16><<<B, 64 * 16, dyn, as_stream(stream)>>>(P, xt, ft, gt, v, iv, ws, wy, mat, ds,
                                                                 is, mode);
    else
      lbfgsb_kernel<JOINT_W><<<B, 64 * JOINT_W, dyn, as_stream(stream)>>>(P, xt, ft, gt, v, iv, ws,
                                                                           wy, mat, ds, is, mode);
  }
  BO_LAUNCH_CHECK();
  return BO_OK;
}
