// Host (single-lane) build of botorch_amd/csrc/lbfgsb_core.h for the CPU
// tests: the same state machine the gfx950 kernel runs, driven one restart at
// a time from Python and compared with scipy's own setulb trial points
// (tests/test_lbfgsb_cpu.py).  Test infrastructure only; never shipped.
#include <cmath>
#include <cstring>
#define BO_HD
#include "../../botorch_amd/csrc/lbfgsb_core.h"

namespace {
struct HostCtx {
  static constexpr int NL = 1;
  int lane = 0;
  void sync() {}
  unsigned long long clock() { return 0; }
  double sum(double v) { return v; }
  double max(double v) { return v; }
  double min(double v) { return v; }
  void argmin(double&, int&) {}
  int exscan(int v, int& total) {
    total = v;
    return 0;
  }
};
}  // namespace

extern "C" int bo_lbfgsb_host_step(int n, int m, int maxls, int maxiter, int maxfun, double tol,
                                   double pgtol, const double* lower, const double* upper,
                                   double* xt, double ft, const double* gt, double* v, int* iv,
                                   double* ws, double* wy, double* mat, double* ds, int* is) {
  if (n < 1 || m < 1 || m > bolb::MMAX) return -1;
  static bolb::Shared S;
  memset(&S, 0xff, sizeof S);  // LDS holds garbage at a kernel's start: NaN everywhere
  bolb::Problem P{n, m, maxls, maxiter, maxfun, tol, pgtol, lower, upper, nullptr};
  bolb::Restart R{xt, ft, gt, v, iv, ws, wy, mat, ds, is};
  HostCtx c;
  bolb::Step<HostCtx> st(c, P, R, S);
  st.run(nullptr);
  return is[bolb::I_STATUS];
}

extern "C" int bo_lbfgsb_host_layout(int* out) {  // slot counts the Python side allocates
  out[0] = bolb::V_COUNT;
  out[1] = bolb::IV_COUNT;
  out[2] = bolb::NMAT * bolb::MMAX * bolb::MMAX;
  out[3] = bolb::DSLOTS;
  out[4] = bolb::ISLOTS;
  out[5] = bolb::MMAX;
  return 0;
}

// ---- 64-lane emulation: one std::thread per lane, a barrier for sync() and
// the kernel's xor-butterfly reductions, so lane-parallel mistakes of the
// gfx950 build (a missing barrier, a non-uniform value) show on the CPU ----
#include <barrier>
#include <memory>
#include <thread>
#include <vector>
namespace {
// NLANES threads = NLANES / 64 emulated waves: within a wave the kernel's
// xor butterflies and shuffles, across waves the block contexts' LDS steps
// (csrc/lbfgsb.hip WaveCtx for 64 lanes, BlockCtx above)
template <int NLANES>
struct LaneShared {
  std::barrier<> bar{NLANES};
  // per-wave barriers: a wave's butterfly (shuffles on the device) involves
  // only its own lanes, and waves may run different numbers of them
  std::vector<std::unique_ptr<std::barrier<>>> wbar;
  LaneShared() {
    for (int w = 0; w < NLANES / 64; ++w) wbar.emplace_back(new std::barrier<>(64));
  }
  double dv[NLANES];
  int iv[NLANES];
  double wv[NLANES / 64][bolb::M2];
  int wi[NLANES / 64];
};
template <int NLANES>
struct LaneCtx {
  static constexpr int NL = NLANES;
  static constexpr int NW = NLANES / 64;
  int lane;
  LaneShared<NLANES>* sh;
  int wave() const { return lane >> 6; }
  int wlane() const { return lane & 63; }
  void sync() { sh->bar.arrive_and_wait(); }
  unsigned long long clock() { return 0; }
  template <class Op>
  double wave_butterfly(double v, Op op) {  // within each 64-lane wave
    std::barrier<>& wb = *sh->wbar[wave()];
    for (int o = 32; o > 0; o >>= 1) {
      wb.arrive_and_wait();
      sh->dv[lane] = v;
      wb.arrive_and_wait();
      v = op(v, sh->dv[lane ^ o]);
    }
    wb.arrive_and_wait();
    return v;
  }
  template <class Op>
  double all(double v, Op op) {  // waves in order, as BlockCtx::all
    v = wave_butterfly(v, op);
    if (NW == 1) return v;
    sh->bar.arrive_and_wait();
    if (wlane() == 0) sh->wv[wave()][0] = v;
    sh->bar.arrive_and_wait();
    double r = sh->wv[0][0];
    for (int w = 1; w < NW; ++w) r = op(r, sh->wv[w][0]);
    return r;
  }
  double wave_sum(double v) { return wave_butterfly(v, [](double a, double b) { return a + b; }); }
  double sum(double v) { return all(v, [](double a, double b) { return a + b; }); }
  double max(double v) { return all(v, [](double a, double b) { return fmax(a, b); }); }
  double min(double v) { return all(v, [](double a, double b) { return fmin(a, b); }); }
  template <int K>
  void sums(double (&v)[K]) {
    for (int k = 0; k < K; ++k) v[k] = wave_sum(v[k]);
    sh->bar.arrive_and_wait();
    if (wlane() == 0)
      for (int k = 0; k < K; ++k) sh->wv[wave()][k] = v[k];
    sh->bar.arrive_and_wait();
    for (int k = 0; k < K; ++k) {
      double r = sh->wv[0][k];
      for (int w = 1; w < NW; ++w) r += sh->wv[w][k];
      v[k] = r;
    }
    sh->bar.arrive_and_wait();
  }
  void argmin(double& v, int& i) {
    std::barrier<>& wb = *sh->wbar[wave()];
    for (int o = 32; o > 0; o >>= 1) {
      wb.arrive_and_wait();
      sh->dv[lane] = v;
      sh->iv[lane] = i;
      wb.arrive_and_wait();
      const double ov = sh->dv[lane ^ o];
      const int oi = sh->iv[lane ^ o];
      if (ov < v || (ov == v && oi < i)) {
        v = ov;
        i = oi;
      }
    }
    wb.arrive_and_wait();
    if (NW == 1) return;
    sh->bar.arrive_and_wait();
    if (wlane() == 0) {
      sh->wv[wave()][0] = v;
      sh->wi[wave()] = i;
    }
    sh->bar.arrive_and_wait();
    v = sh->wv[0][0];
    i = sh->wi[0];
    for (int w = 1; w < NW; ++w)
      if (sh->wv[w][0] < v || (sh->wv[w][0] == v && sh->wi[w] < i)) {
        v = sh->wv[w][0];
        i = sh->wi[w];
      }
  }
  int exscan(int v, int& total) {  // shuffle-up scan per wave, then the waves in order
    sh->bar.arrive_and_wait();
    sh->iv[lane] = v;
    sh->bar.arrive_and_wait();
    int before = 0;
    total = 0;
    for (int l = 0; l < NL; ++l) {
      if (l < lane) before += sh->iv[l];
      total += sh->iv[l];
    }
    sh->bar.arrive_and_wait();
    return before;
  }
};

template <int NLANES>
int step_lanes(int n, int m, int maxls, int maxiter, int maxfun, double tol, double pgtol,
               const double* lower, const double* upper, double* xt, double ft, const double* gt,
               double* v, int* iv, double* ws, double* wy, double* mat, double* ds, int* is) {
  if (n < 1 || m < 1 || m > bolb::MMAX) return -1;
  static bolb::Shared S;
  memset(&S, 0xff, sizeof S);
  LaneShared<NLANES> sh;
  bolb::Problem P{n, m, maxls, maxiter, maxfun, tol, pgtol, lower, upper, nullptr};
  bolb::Restart R{xt, ft, gt, v, iv, ws, wy, mat, ds, is};
  std::vector<std::thread> th;
  for (int l = 0; l < NLANES; ++l)
    th.emplace_back([&, l] {
      LaneCtx<NLANES> c{l, &sh};
      bolb::Step<LaneCtx<NLANES>> st(c, P, R, S);
      st.run(nullptr);
    });
  for (auto& t : th) t.join();
  return is[bolb::I_STATUS];
}
}  // namespace

extern "C" int bo_lbfgsb_host_step_lanes(int n, int m, int maxls, int maxiter, int maxfun,
                                         double tol, double pgtol, const double* lower,
                                         const double* upper, double* xt, double ft,
                                         const double* gt, double* v, int* iv, double* ws,
                                         double* wy, double* mat, double* ds, int* is) {
  return step_lanes<64>(n, m, maxls, maxiter, maxfun, tol, pgtol, lower, upper, xt, ft, gt, v, iv,
                        ws, wy, mat, ds, is);
}

// two emulated waves: the wide (joint-problem) code paths of the kernel
extern "C" int bo_lbfgsb_host_step_wide(int n, int m, int maxls, int maxiter, int maxfun,
                                        double tol, double pgtol, const double* lower,
                                        const double* upper, double* xt, double ft,
                                        const double* gt, double* v, int* iv, double* ws,
                                        double* wy, double* mat, double* ds, int* is) {
  return step_lanes<128>(n, m, maxls, maxiter, maxfun, tol, pgtol, lower, upper, xt, ft, gt, v, iv,
                         ws, wy, mat, ds, is);
}
