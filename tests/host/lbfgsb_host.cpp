// Host (single-lane) build of botorch_amd/csrc/lbfgsb_core.h for the CPU
// tests: the same state machine the gfx950 kernel runs, driven one restart at
// a time from Python and compared with scipy's own setulb trial points
// (tests/test_lbfgsb_cpu.py).  Test infrastructure only; never shipped.
#include <cmath>
#define BO_HD
#include "../../botorch_amd/csrc/lbfgsb_core.h"

namespace {
struct HostCtx {
  static constexpr int NL = 1;
  int lane = 0;
  void sync() {}
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
  bolb::Problem P{n, m, maxls, maxiter, maxfun, tol, pgtol, lower, upper};
  bolb::Restart R{xt, ft, gt, v, iv, ws, wy, mat, ds, is};
  HostCtx c;
  bolb::Step<HostCtx> st(c, P, R, S);
  st.run();
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
