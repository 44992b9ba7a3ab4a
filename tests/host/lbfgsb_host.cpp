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
#include <thread>
#include <vector>

namespace {
struct LaneShared {
  std::barrier<> bar{64};
  double dv[64];
  int iv[64];
};

struct LaneCtx {
  static constexpr int NL = 64;
  int lane;
  LaneShared* sh;
  void sync() { sh->bar.arrive_and_wait(); }
  unsigned long long clock() { return 0; }
  template <class Op>
  double butterfly(double v, Op op) {
    for (int o = 32; o > 0; o >>= 1) {
      sh->bar.arrive_and_wait();
      sh->dv[lane] = v;
      sh->bar.arrive_and_wait();
      v = op(v, sh->dv[lane ^ o]);
    }
    return v;
  }
  double sum(double v) { return butterfly(v, [](double a, double b) { return a + b; }); }
  double max(double v) { return butterfly(v, [](double a, double b) { return fmax(a, b); }); }
  double min(double v) { return butterfly(v, [](double a, double b) { return fmin(a, b); }); }
  void argmin(double& v, int& i) {
    for (int o = 32; o > 0; o >>= 1) {
      sh->bar.arrive_and_wait();
      sh->dv[lane] = v;
      sh->iv[lane] = i;
      sh->bar.arrive_and_wait();
      const double ov = sh->dv[lane ^ o];
      const int oi = sh->iv[lane ^ o];
      if (ov < v || (ov == v && oi < i)) {
        v = ov;
        i = oi;
      }
    }
  }
};
}  // namespace

extern "C" int bo_lbfgsb_host_step_lanes(int n, int m, int maxls, int maxiter, int maxfun,
                                         double tol, double pgtol, const double* lower,
                                         const double* upper, double* xt, double ft,
                                         const double* gt, double* v, int* iv, double* ws,
                                         double* wy, double* mat, double* ds, int* is) {
  if (n < 1 || m < 1 || m > bolb::MMAX) return -1;
  static bolb::Shared S;
  memset(&S, 0xff, sizeof S);
  LaneShared sh;
  bolb::Problem P{n, m, maxls, maxiter, maxfun, tol, pgtol, lower, upper, nullptr};
  bolb::Restart R{xt, ft, gt, v, iv, ws, wy, mat, ds, is};
  std::vector<std::thread> th;
  for (int l = 0; l < 64; ++l)
    th.emplace_back([&, l] {
      LaneCtx c{l, &sh};
      bolb::Step<LaneCtx> st(c, P, R, S);
      st.run(nullptr);
    });
  for (auto& t : th) t.join();
  return is[bolb::I_STATUS];
}
