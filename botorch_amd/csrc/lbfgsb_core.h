// L-BFGS-B (Byrd, Lu, Nocedal, Zhu; version 3.0 as scipy 1.15 ships it) as a
// reverse-communication state machine, one restart per call.
//
// This is the algorithm behind scipy.optimize.minimize(method="L-BFGS-B"),
// which botorch's gen_candidates_scipy calls (botorch/generation/gen.py:
// 194-267; scipy 1.15.3 optimize/_lbfgsb_py.py _minimize_lbfgsb and its
// setulb driver): generalized Cauchy point along the projected steepest-descent
// path (`cauchy`), free-variable subspace minimisation with the compact L-BFGS
// matrix and the projection step of v3.0 (`formk` / `cmprlb` / `subsm`), the
// MINPACK-2 More-Thuente line search (`dcsrch` / `dcstep`, ftol 1e-3, gtol 0.9,
// xtol 0.1, at most maxls trial steps), the compact-form update (`matupd` /
// `formt`) and the projected-gradient and relative-reduction stopping tests.
//
// Every call consumes f and g at the trial point xt and advances the restart
// until it needs the next evaluation, then writes that point to xt -- the
// scipy driver's task == FG / NEW_X loop, with the maxiter / maxfun checks of
// _minimize_lbfgsb.  The restarts of a batch are independent problems; the
// trial-point sequence of each equals scipy's on the same objective (up to the
// summation order of the dot products), tested against setulb itself.
//
// The code is written once against a lane context C:
//   C::NL lanes; c.lane; c.sync(); c.sum / c.max / c.min (all-lane reduction,
//   identical result on every lane); c.argmin(v, i) (smallest v, ties to the
//   smallest i); c.exscan(v, total) (exclusive prefix sum in lane order).
//   Vector work is strided over lanes; the small dense algebra (2m x 2m) runs
//   on lane 0 in the block-shared record and is published by c.sync().  A
//   context wider than one wave (C::NL > 64: the joint problem over all
//   restarts, n = b q d in the thousands) also provides waves: c.wave(),
//   c.wlane(), c.wave_sum(v) (within the wave) and c.sums(v) (NL-wide sums of
//   a register array); its Step batches the 2m dot products of a pass over
//   the vectors into one pass (wdots) and splits formk's products over the
//   waves (formk_wide).  The including file defines BO_HD.
#pragma once

namespace bolb {

// Strided vector loops: four iterations' loads in flight instead of one memory
// latency per iteration (a joint problem's n = b q d runs ~24 iterations per
// lane); sums keep their per-lane order.
#define BO_UNROLL4 _Pragma("unroll 4")

constexpr int MMAX = 20;  // history limit (scipy default maxcor = 10)
constexpr int M2 = 2 * MMAX;
constexpr double EPSMCH = 2.220446049250313e-16;
constexpr double BIG = 1e10;
// dcsrch parameters of lnsrlb
constexpr double LS_FTOL = 1e-3, LS_GTOL = 0.9, LS_XTOL = 0.1;

enum Phase : int { PH_START = 0, PH_LNSRCH = 1, PH_STOP = 2 };
enum Status : int {
  ST_RUN = 0,
  ST_CONV_PGTOL = 1,    // CONVERGENCE: NORM_OF_PROJECTED_GRADIENT_<=_PGTOL
  ST_CONV_FTOL = 2,     // CONVERGENCE: REL_REDUCTION_OF_F_<=_FACTR*EPSMCH
  ST_ABNORMAL = 3,      // ABNORMAL_TERMINATION_IN_LNSRCH
  ST_MAXITER = 4,       // STOP: TOTAL NO. of ITERATIONS REACHED LIMIT
  ST_MAXFUN = 5,        // STOP: TOTAL NO. of f AND g EVALUATIONS EXCEEDS LIMIT
  ST_ERROR = 6,         // line-search input error / non-finite start
};

// persistent scalar slots (per restart; doubles then ints)
enum D : int {
  D_F, D_FOLD, D_THETA, D_STP, D_STPMX, D_DTD, D_GD, D_GDOLD, D_SBGNRM,
  D_FINIT, D_GINIT, D_GTEST, D_WIDTH, D_WIDTH1, D_STX, D_FX, D_GX, D_STY, D_FY, D_GY,
  D_STMIN, D_STMAX, D_COUNT
};
enum I : int {
  I_PHASE, I_STATUS, I_COL, I_HEAD, I_ITAIL, I_IUPDAT, I_ITER, I_IFUN, I_IBACK, I_NFEV,
  I_NITER, I_BRACKT, I_STAGE, I_NFREE, I_INFO, I_COUNT
};
constexpr int DSLOTS = 24, ISLOTS = 16;
static_assert(D_COUNT <= DSLOTS && I_COUNT <= ISLOTS, "slot layout");

// per-restart n-vectors and int vectors (offsets in units of n)
enum V : int { V_X, V_G, V_T, V_R, V_Z, V_D, V_DC, V_TB, V_RS, V_XP, V_COUNT };
enum IV : int { IV_WHERE, IV_INDEX, IV_COUNT };
constexpr int NMAT = 3;  // SY, SS, WT (MMAX x MMAX, column-major)

struct Problem {
  int n, m, maxls, maxiter, maxfun;
  double tol;    // factr * epsmch (scipy's ftol)
  double pgtol;  // scipy's gtol
  const double* lower;  // n; -inf / +inf for a missing bound
  const double* upper;
  unsigned long long* prof;  // optional per-restart phase clocks (PROF_SLOTS each), or null
};
constexpr int PROF_SLOTS = 8;  // load, cauchy, freev, formk, cmprlb, subsm, line search, store

struct Restart {   // global buffers of one restart
  double* xt;      // trial point (in: where f, g were evaluated; out: next point)
  double f_new;    // f at xt
  const double* g_new;
  double* v;       // V_COUNT x n
  int* iv;         // IV_COUNT x n
  double* ws;      // m x n  (ring slot-major)
  double* wy;
  double* mat;     // NMAT x MMAX*MMAX
  double* ds;      // DSLOTS
  int* is;         // ISLOTS
  // the Cauchy search's breakpoints (n doubles, scratch of one call): the
  // V_TB vector unless the caller gives faster memory (the wide kernel: LDS)
  double* tb_scratch = nullptr;
};

struct Shared {    // block-shared record (LDS on the device)
  double d[DSLOTS];
  int i[ISLOTS];
  double sy[MMAX * MMAX], ss[MMAX * MMAX], wt[MMAX * MMAX];
  double wn[M2 * M2];
  double p[M2], c[M2], v[M2], wbp[M2], wv[M2];
  double t0, t1, t2;  // scalar hand-offs from lane 0
  int k0, k1, flag;
};

BO_HD inline int nbd_of(double l, double u) {  // scipy's bound code
  const bool fl = l > -1e308, fu = u < 1e308;  // finite
  return fl ? (fu ? 2 : 1) : (fu ? 3 : 0);
}

// ---------------------------------------------------------------------------
// small dense algebra (lane 0), column-major, LINPACK semantics
// dpofa: upper Cholesky R (A = R^T R) in place; 0 or the failing column + 1
BO_HD inline int dpofa(double* a, int ld, int n) {
  for (int j = 0; j < n; ++j) {
    double s = 0.0;
    for (int k = 0; k < j; ++k) {
      double t = a[k + j * ld];
      #pragma unroll 4
      for (int i = 0; i < k; ++i) t -= a[i + k * ld] * a[i + j * ld];
      t /= a[k + k * ld];
      a[k + j * ld] = t;
      s += t * t;
    }
    s = a[j + j * ld] - s;
    if (s <= 0.0) return j + 1;
    a[j + j * ld] = sqrt(s);
  }
  return 0;
}
// dtrsl job 11: solve T^T x = b (T upper)
BO_HD inline int dtrsl_t(const double* t, int ld, int n, double* b) {
  for (int j = 0; j < n; ++j)
    if (t[j + j * ld] == 0.0) return j + 1;
  b[0] /= t[0];
  for (int j = 1; j < n; ++j) {
    double s = 0.0;
    #pragma unroll 4
    for (int i = 0; i < j; ++i) s += t[i + j * ld] * b[i];
    b[j] = (b[j] - s) / t[j + j * ld];
  }
  return 0;
}
// dtrsl job 01: solve T x = b (T upper)
BO_HD inline int dtrsl_n(const double* t, int ld, int n, double* b) {
  for (int j = 0; j < n; ++j)
    if (t[j + j * ld] == 0.0) return j + 1;
  b[n - 1] /= t[(n - 1) + (n - 1) * ld];
  for (int j = n - 2; j >= 0; --j) {
    const double temp = -b[j + 1];
    #pragma unroll 4
    for (int i = 0; i <= j; ++i) b[i] += temp * t[i + (j + 1) * ld];
    b[j] /= t[j + j * ld];
  }
  return 0;
}
// bmv: p = M v for the 2col x 2col middle matrix of the compact form
BO_HD inline int bmv(const double* sy, const double* wt, int col, const double* v, double* p) {
  if (col == 0) return 0;
  p[col] = v[col];
  for (int i = 1; i < col; ++i) {
    double sum = 0.0;
    #pragma unroll 4
    for (int k = 0; k < i; ++k) sum += sy[i + k * MMAX] * v[k] / sy[k + k * MMAX];
    p[col + i] = v[col + i] + sum;
  }
  int info = dtrsl_t(wt, MMAX, col, p + col);
  if (info) return info;
  for (int i = 0; i < col; ++i) p[i] = v[i] / sqrt(sy[i + i * MMAX]);
  info = dtrsl_n(wt, MMAX, col, p + col);
  if (info) return info;
  for (int i = 0; i < col; ++i) p[i] = -p[i] / sqrt(sy[i + i * MMAX]);
  for (int i = 0; i < col; ++i) {
    double sum = 0.0;
    #pragma unroll 4
    for (int k = i + 1; k < col; ++k) sum += sy[k + i * MMAX] * p[col + k] / sy[i + i * MMAX];
    p[i] += sum;
  }
  return 0;
}
// formt: WT = chol(theta SS + L D^-1 L^T) (upper)
BO_HD inline int formt(double* wt, const double* sy, const double* ss, int col, double theta) {
  for (int j = 0; j < col; ++j) wt[0 + j * MMAX] = theta * ss[0 + j * MMAX];
  for (int i = 1; i < col; ++i)
    for (int j = i; j < col; ++j) {
      double ddum = 0.0;
      #pragma unroll 4
      for (int k = 0; k < i; ++k) ddum += sy[i + k * MMAX] * sy[j + k * MMAX] / sy[k + k * MMAX];
      wt[i + j * MMAX] = ddum + theta * ss[i + j * MMAX];
    }
  return dpofa(wt, MMAX, col) ? -3 : 0;
}

// MINPACK-2 dcstep: safeguarded step of the More-Thuente search
BO_HD inline void dcstep(double& stx, double& fx, double& dx, double& sty, double& fy, double& dy,
                         double& stp, double fp, double dp, int& brackt, double stpmin,
                         double stpmax) {
  const double sgnd = dp * (dx / fabs(dx));
  double stpf, stpc, stpq, theta, s, gamma, p, q, r;
  if (fp > fx) {
    theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    s = fmax(fmax(fabs(theta), fabs(dx)), fabs(dp));
    gamma = s * sqrt((theta / s) * (theta / s) - (dx / s) * (dp / s));
    if (stp < stx) gamma = -gamma;
    p = (gamma - dx) + theta;
    q = ((gamma - dx) + gamma) + dp;
    r = p / q;
    stpc = stx + r * (stp - stx);
    stpq = stx + ((dx / ((fx - fp) / (stp - stx) + dx)) / 2.0) * (stp - stx);
    stpf = (fabs(stpc - stx) < fabs(stpq - stx)) ? stpc : stpc + (stpq - stpc) / 2.0;
    brackt = 1;
  } else if (sgnd < 0.0) {
    theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    s = fmax(fmax(fabs(theta), fabs(dx)), fabs(dp));
    gamma = s * sqrt((theta / s) * (theta / s) - (dx / s) * (dp / s));
    if (stp > stx) gamma = -gamma;
    p = (gamma - dp) + theta;
    q = ((gamma - dp) + gamma) + dx;
    r = p / q;
    stpc = stp + r * (stx - stp);
    stpq = stp + (dp / (dp - dx)) * (stx - stp);
    stpf = (fabs(stpc - stp) > fabs(stpq - stp)) ? stpc : stpq;
    brackt = 1;
  } else if (fabs(dp) < fabs(dx)) {
    theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    s = fmax(fmax(fabs(theta), fabs(dx)), fabs(dp));
    gamma = s * sqrt(fmax(0.0, (theta / s) * (theta / s) - (dx / s) * (dp / s)));
    if (stp > stx) gamma = -gamma;
    p = (gamma - dp) + theta;
    q = (gamma + (dx - dp)) + gamma;
    r = p / q;
    if (r < 0.0 && gamma != 0.0)
      stpc = stp + r * (stx - stp);
    else if (stp > stx)
      stpc = stpmax;
    else
      stpc = stpmin;
    stpq = stp + (dp / (dp - dx)) * (stx - stp);
    if (brackt) {
      stpf = (fabs(stpc - stp) < fabs(stpq - stp)) ? stpc : stpq;
      if (stp > stx)
        stpf = fmin(stp + 0.66 * (sty - stp), stpf);
      else
        stpf = fmax(stp + 0.66 * (sty - stp), stpf);
    } else {
      stpf = (fabs(stpc - stp) > fabs(stpq - stp)) ? stpc : stpq;
      stpf = fmin(stpmax, stpf);
      stpf = fmax(stpmin, stpf);
    }
  } else {
    if (brackt) {
      theta = 3.0 * (fp - fy) / (sty - stp) + dy + dp;
      s = fmax(fmax(fabs(theta), fabs(dy)), fabs(dp));
      gamma = s * sqrt((theta / s) * (theta / s) - (dy / s) * (dp / s));
      if (stp > sty) gamma = -gamma;
      p = (gamma - dp) + theta;
      q = ((gamma - dp) + gamma) + dy;
      r = p / q;
      stpc = stp + r * (sty - stp);
      stpf = stpc;
    } else if (stp > stx) {
      stpf = stpmax;
    } else {
      stpf = stpmin;
    }
  }
  if (fp > fx) {
    sty = stp;
    fy = fp;
    dy = dp;
  } else {
    if (sgnd < 0.0) {
      sty = stx;
      fy = fx;
      dy = dx;
    }
    stx = stp;
    fx = fp;
    dx = dp;
  }
  stp = stpf;
}

// dcsrch after START: returns 0 = FG (stp holds the next trial step),
// 1 = CONVERGENCE, 2 = WARNING (the search stops either way)
BO_HD inline int dcsrch_cont(double* d, int* iv, double f, double g, double& stp, double stpmin,
                             double stpmax) {
  int brackt = iv[I_BRACKT], stage = iv[I_STAGE];
  double stx = d[D_STX], fx = d[D_FX], gx = d[D_GX], sty = d[D_STY], fy = d[D_FY], gy = d[D_GY];
  double stmin = d[D_STMIN], stmax = d[D_STMAX], width = d[D_WIDTH], width1 = d[D_WIDTH1];
  const double finit = d[D_FINIT], ginit = d[D_GINIT], gtest = d[D_GTEST];
  const double ftest = finit + stp * gtest;
  if (stage == 1 && f <= ftest && g >= 0.0) stage = 2;
  int task = 0;
  if (brackt && (stp <= stmin || stp >= stmax)) task = 2;
  if (brackt && stmax - stmin <= LS_XTOL * stmax) task = 2;
  if (stp == stpmax && f <= ftest && g <= gtest) task = 2;
  if (stp == stpmin && (f > ftest || g >= gtest)) task = 2;
  if (f <= ftest && fabs(g) <= LS_GTOL * (-ginit)) task = 1;
  if (task == 0) {
    if (stage == 1 && f <= fx && f > ftest) {
      const double fm = f - stp * gtest;
      double fxm = fx - stx * gtest, fym = fy - sty * gtest;
      const double gm = g - gtest;
      double gxm = gx - gtest, gym = gy - gtest;
      dcstep(stx, fxm, gxm, sty, fym, gym, stp, fm, gm, brackt, stmin, stmax);
      fx = fxm + stx * gtest;
      fy = fym + sty * gtest;
      gx = gxm + gtest;
      gy = gym + gtest;
    } else {
      dcstep(stx, fx, gx, sty, fy, gy, stp, f, g, brackt, stmin, stmax);
    }
    if (brackt) {
      if (fabs(sty - stx) >= 0.66 * width1) stp = stx + 0.5 * (sty - stx);
      width1 = width;
      width = fabs(sty - stx);
    }
    if (brackt) {
      stmin = fmin(stx, sty);
      stmax = fmax(stx, sty);
    } else {
      stmin = stp + 1.1 * (stp - stx);
      stmax = stp + 4.0 * (stp - stx);
    }
    stp = fmax(stp, stpmin);
    stp = fmin(stp, stpmax);
    if ((brackt && (stp <= stmin || stp >= stmax)) || (brackt && stmax - stmin <= LS_XTOL * stmax))
      stp = stx;
  }
  iv[I_BRACKT] = brackt;
  iv[I_STAGE] = stage;
  d[D_STX] = stx; d[D_FX] = fx; d[D_GX] = gx;
  d[D_STY] = sty; d[D_FY] = fy; d[D_GY] = gy;
  d[D_STMIN] = stmin; d[D_STMAX] = stmax; d[D_WIDTH] = width; d[D_WIDTH1] = width1;
  return task;
}

// dcsrch START (stp, f, g at step 0): 0 = FG, -1 = input error
BO_HD inline int dcsrch_start(double* d, int* iv, double f, double g, double stp, double stpmin,
                              double stpmax) {
  if (stp < stpmin || stp > stpmax || g >= 0.0) return -1;
  iv[I_BRACKT] = 0;
  iv[I_STAGE] = 1;
  d[D_FINIT] = f;
  d[D_GINIT] = g;
  d[D_GTEST] = LS_FTOL * g;
  d[D_WIDTH] = stpmax - stpmin;
  d[D_WIDTH1] = (stpmax - stpmin) / 0.5;
  d[D_STX] = 0.0; d[D_FX] = f; d[D_GX] = g;
  d[D_STY] = 0.0; d[D_FY] = f; d[D_GY] = g;
  d[D_STMIN] = 0.0;
  d[D_STMAX] = stp + 4.0 * stp;
  return 0;
}


// ---------------------------------------------------------------------------
// the per-restart step (mainlb of setulb, resumed at the point it last asked
// for f and g)

template <class C>
struct Step {
  C& c;
  const Problem& P;
  const Restart& R;
  Shared& S;
  int n, m;
  double *x, *g, *t, *r, *z, *dd, *dc, *tb, *rs, *xp;
  int *iwhere, *index;
  bool cnstnd, boxed;

  BO_HD Step(C& c_, const Problem& P_, const Restart& R_, Shared& S_)
      : c(c_), P(P_), R(R_), S(S_), n(P_.n), m(P_.m) {
    x = R.v + (long)V_X * n;   g = R.v + (long)V_G * n;   t = R.v + (long)V_T * n;
    r = R.v + (long)V_R * n;   z = R.v + (long)V_Z * n;   dd = R.v + (long)V_D * n;
    dc = R.v + (long)V_DC * n;
    tb = R.tb_scratch ? R.tb_scratch : R.v + (long)V_TB * n; rs = R.v + (long)V_RS * n;
    xp = R.v + (long)V_XP * n;
    iwhere = R.iv + (long)IV_WHERE * n;
    index = R.iv + (long)IV_INDEX * n;
    cnstnd = boxed = false;
  }

  // a workgroup-wide restart: batched dot products, formk split over waves
  static constexpr bool WIDE = C::NL > 64;

  unsigned long long tprev = 0;
  unsigned long long* prof = nullptr;  // this restart's PROF_SLOTS clocks
  BO_HD void tick(int phase) {  // attribute the time since the last tick to `phase`
    if (!prof) return;
    const unsigned long long now = c.clock();
    if (c.lane == 0) prof[phase] += now - tprev;
    tprev = now;
  }

  BO_HD double lo(int i) const { return P.lower[i]; }
  BO_HD double hi(int i) const { return P.upper[i]; }
  BO_HD int nbd(int i) const { return nbd_of(P.lower[i], P.upper[i]); }
  BO_HD int slot(int j) const { return (S.i[I_HEAD] + j) % m; }  // ordered column -> ring slot
  BO_HD const double* WY(int j) const { return R.wy + (long)slot(j) * n; }
  BO_HD const double* WS(int j) const { return R.ws + (long)slot(j) * n; }

  BO_HD double dot(const double* a, const double* b) {
    double s = 0.0;
#pragma unroll 4  // loads issue ahead; the sum keeps its order
    for (int i = c.lane; i < n; i += C::NL) s += a[i] * b[i];
    return c.sum(s);
  }

  // WIDE: out[j] = WY(j) . b, out[col + j] = WS(j) . b (j < col) over the
  // first cnt entries of b, WY / WS read at index[i] with GATHER -- every
  // product of one pass over the vectors, 2 MMAX partial sums per lane, one
  // NL-wide reduction (lane 0 writes out; the caller syncs).
  template <bool GATHER>
  BO_HD void wdots(const double* b, int cnt, double* out) {
    if constexpr (WIDE) {
      const int col = S.i[I_COL];
      int sl[MMAX];  // ring offsets of the ordered columns
#pragma unroll
      for (int j = 0; j < MMAX; ++j) sl[j] = slot(j < col ? j : 0) * n;
      // the WY products, then the WS ones (MMAX partial sums per lane each)
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const double* W = half ? R.ws : R.wy;
        double acc[MMAX];
#pragma unroll
        for (int j = 0; j < MMAX; ++j) acc[j] = 0.0;
        BO_UNROLL4
        for (int i = c.lane; i < cnt; i += C::NL) {
          const int k = GATHER ? index[i] : i;
          const double bi = b[i];
#pragma unroll
          for (int j = 0; j < MMAX; ++j)
            if (j < col) acc[j] += W[sl[j] + k] * bi;
        }
        c.sums(acc);
        if (c.lane == 0)
          for (int j = 0; j < col; ++j) out[half * col + j] = acc[j];
      }
    }
  }

  BO_HD double projgr() {  // sup-norm of the projected gradient
    double nrm = 0.0;
    BO_UNROLL4
    for (int i = c.lane; i < n; i += C::NL) {
      double gi = g[i];
      const int nb = nbd(i);
      if (nb != 0) {
        if (gi < 0.0) {
          if (nb >= 2) gi = fmax(x[i] - hi(i), gi);
        } else {
          if (nb <= 2) gi = fmin(x[i] - lo(i), gi);
        }
      }
      nrm = fmax(nrm, fabs(gi));
    }
    return c.max(nrm);
  }

  BO_HD void refresh() {  // "refresh the lbfgs memory and restart the iteration"
    c.sync();
    if (c.lane == 0) {
      S.i[I_INFO] = 0;
      S.i[I_COL] = 0;
      S.i[I_HEAD] = 0;
      S.d[D_THETA] = 1.0;
      S.i[I_IUPDAT] = 0;
    }
    c.sync();
  }

  BO_HD void stop(int status) {
    c.sync();
    if (c.lane == 0) {
      S.i[I_STATUS] = status;
      S.i[I_PHASE] = PH_STOP;
    }
    c.sync();
  }

  // ---- cauchy: generalized Cauchy point z; c = W^T (z - x) in S.c ----
  BO_HD int cauchy() {
    const int col = S.i[I_COL];
    const double theta = S.d[D_THETA];
    const double inf = __builtin_inf();
    if (S.d[D_SBGNRM] <= 0.0) {
      BO_UNROLL4
      for (int i = c.lane; i < n; i += C::NL) z[i] = x[i];
      c.sync();
      return 0;
    }
    double f1 = 0.0, nbreak = 0.0, nunb = 0.0, moving = 0.0;
    BO_UNROLL4
    for (int i = c.lane; i < n; i += C::NL) {
      const double neggi = -g[i];
      const int nb = nbd(i);
      int w = iwhere[i];
      double tl = 0.0, tu = 0.0;
      if (w != 3 && w != -1) {
        if (nb <= 2) tl = x[i] - lo(i);
        if (nb >= 2) tu = hi(i) - x[i];
        const bool xlower = nb <= 2 && tl <= 0.0;
        const bool xupper = nb >= 2 && tu <= 0.0;
        w = 0;
        if (xlower) {
          if (neggi <= 0.0) w = 1;
        } else if (xupper) {
          if (neggi >= 0.0) w = 2;
        } else {
          if (fabs(neggi) <= 0.0) w = -3;
        }
        iwhere[i] = w;
      }
      double tbi = inf;
      if (w != 0 && w != -1) {
        dc[i] = 0.0;
      } else {
        dc[i] = neggi;
        f1 -= neggi * neggi;
        if (nb <= 2 && nb != 0 && neggi < 0.0) {
          nbreak += 1.0;
          tbi = tl / (-neggi);
        } else if (nb >= 2 && neggi > 0.0) {
          nbreak += 1.0;
          tbi = tu / neggi;
        } else {
          nunb += 1.0;
          if (fabs(neggi) > 0.0) moving = 1.0;
        }
      }
      tb[i] = tbi;
      z[i] = x[i];
    }
    f1 = c.sum(f1);
    const int nbrk = (int)c.sum(nbreak);
    const int nfr = (int)c.sum(nunb);
    const bool bnded = c.max(moving) == 0.0;
    c.sync();
    if constexpr (WIDE) {  // p = W^T dc
      wdots<false>(dc, n, S.p);
    } else {
      for (int j = 0; j < col; ++j) {
        const double py = dot(WY(j), dc);
        const double ps = dot(WS(j), dc);
        if (c.lane == 0) {
          S.p[j] = py;
          S.p[col + j] = ps;
        }
      }
    }
    if (c.lane == 0 && theta != 1.0)
      for (int j = 0; j < col; ++j) S.p[col + j] *= theta;
    c.sync();
    if (nbrk == 0 && nfr == 0) {  // dc = 0: the GCP is x
      if (c.lane == 0)
        for (int j = 0; j < 2 * col; ++j) S.c[j] = 0.0;
      c.sync();
      return 0;
    }
    if (c.lane == 0) {
      for (int j = 0; j < 2 * col; ++j) S.c[j] = 0.0;
      double f2 = -theta * f1;
      int info = 0;
      if (col > 0) {
        info = bmv(S.sy, S.wt, col, S.p, S.v);
        if (!info)
          for (int j = 0; j < 2 * col; ++j) f2 -= S.v[j] * S.p[j];
      }
      S.t0 = f2;
      S.k0 = info;
    }
    c.sync();
    if (S.k0) return S.k0;
    double f2 = S.t0;
    const double f2_org = -theta * f1;
    double dtm = -f1 / f2;
    double tsum = 0.0;
    if (nbrk > 0) {
      int nleft = nbrk;
      double tj = 0.0;
      while (true) {
        double tmin = inf;
        int ibp = n;
#pragma unroll 4
        for (int i = c.lane; i < n; i += C::NL)
          if (tb[i] < tmin) {
            tmin = tb[i];
            ibp = i;
          }
        c.argmin(tmin, ibp);
        if (ibp >= n) break;  // no breakpoint left (non-finite breakpoints)
        const double tj0 = tj;
        tj = tmin;
        const double dt = tj - tj0;
        if (dtm < dt) break;  // the minimiser lies in this interval
        tsum += dt;
        --nleft;
        const double dibp = dc[ibp];
        const double zibp = dibp > 0.0 ? hi(ibp) - x[ibp] : lo(ibp) - x[ibp];
        c.sync();
        if (c.lane == 0) {
          dc[ibp] = 0.0;
          tb[ibp] = inf;
          z[ibp] = dibp > 0.0 ? hi(ibp) : lo(ibp);
          iwhere[ibp] = dibp > 0.0 ? 2 : 1;
        }
        c.sync();
        if (nleft == 0 && nbrk == n) {  // every variable is fixed: z is the GCP
          if (c.lane == 0 && col > 0)
            for (int j = 0; j < 2 * col; ++j) S.c[j] += dt * S.p[j];
          c.sync();
          return 0;
        }
        const double dibp2 = dibp * dibp;
        f1 = f1 + dt * f2 + dibp2 - theta * dibp * zibp;
        f2 = f2 - theta * dibp2;
        if (col > 0) {
          if (c.lane == 0) {
            for (int j = 0; j < 2 * col; ++j) S.c[j] += dt * S.p[j];
            const double* wyb = R.wy;
            const double* wsb = R.ws;
            for (int j = 0; j < col; ++j) {
              S.wbp[j] = wyb[(long)slot(j) * n + ibp];
              S.wbp[col + j] = theta * wsb[(long)slot(j) * n + ibp];
            }
            const int info = bmv(S.sy, S.wt, col, S.wbp, S.v);
            double wmc = 0.0, wmp = 0.0, wmw = 0.0;
            if (!info) {
              for (int j = 0; j < 2 * col; ++j) wmc += S.c[j] * S.v[j];
              for (int j = 0; j < 2 * col; ++j) wmp += S.p[j] * S.v[j];
              for (int j = 0; j < 2 * col; ++j) wmw += S.wbp[j] * S.v[j];
              for (int j = 0; j < 2 * col; ++j) S.p[j] += -dibp * S.wbp[j];
            }
            S.t0 = wmc;
            S.t1 = wmp;
            S.t2 = wmw;
            S.k0 = info;
          }
          c.sync();
          if (S.k0) return S.k0;
          f1 = f1 + dibp * S.t0;
          f2 = f2 + 2.0 * dibp * S.t1 - dibp2 * S.t2;
          c.sync();
        }
        f2 = fmax(EPSMCH * f2_org, f2);
        if (nleft > 0) {
          dtm = -f1 / f2;
          continue;
        } else if (bnded) {
          f1 = 0.0;
          f2 = 0.0;
          dtm = 0.0;
        } else {
          dtm = -f1 / f2;
        }
        break;
      }
    }
    if (dtm <= 0.0) dtm = 0.0;
    tsum += dtm;
    BO_UNROLL4
    for (int i = c.lane; i < n; i += C::NL) z[i] += tsum * dc[i];
    if (c.lane == 0 && col > 0)
      for (int j = 0; j < 2 * col; ++j) S.c[j] += dtm * S.p[j];
    c.sync();
    return 0;
  }

  // ---- freev: free (iwhere <= 0, ascending) then active (descending from n-1) ----
  // A stream compaction: each lane takes a contiguous chunk, counts its free
  // variables, and the exclusive prefix sums over the lanes place them (the
  // same index array as the serial loop).
  BO_HD void freev() {
    c.sync();
    const int ch = (n + C::NL - 1) / C::NL;
    const int i0 = c.lane * ch < n ? c.lane * ch : n;
    const int i1 = i0 + ch < n ? i0 + ch : n;
    int nf = 0;
    for (int i = i0; i < i1; ++i) nf += iwhere[i] <= 0 ? 1 : 0;
    int tot_f = 0, tot_a = 0;
    int of = c.exscan(nf, tot_f);
    int oa = c.exscan(i1 - i0 - nf, tot_a);
    for (int i = i0; i < i1; ++i) {
      if (iwhere[i] <= 0)
        index[of++] = i;
      else
        index[n - 1 - (oa++)] = i;
    }
    if (c.lane == 0) S.i[I_NFREE] = tot_f;
    c.sync();
  }

  // ---- formk: the LEL^T factorisation of the 2col x 2col K in S.wn ----
  // WIDE: the products of formk are the lower triangle of the Gram matrix of
  // the 2col vectors u < col: WY(u), u >= col: WS(u - col), each over the
  // free set (Y.Y, and S_i.Y_j with i <= j) or the active set (S.S, and
  // S_i.Y_j with i > j).  4 x 4 blocks of it go round-robin to the waves; a
  // wave's lanes stride over the variables in natural order (free: iwhere <=
  // 0, as freev decides), 16 partial sums each, then a wave reduction.
  BO_HD void formk_wide() {
    if constexpr (WIDE) {
      const int col = S.i[I_COL];
      const double theta = S.d[D_THETA];
      const int nv = 2 * col, nb = (nv + 3) / 4;
      const int nblk = nb * (nb + 1) / 2;
      for (int blk = c.wave(); blk < nblk; blk += C::NW) {
        int bu = 0, rem = blk;
        while (rem > bu) {
          rem -= bu + 1;
          ++bu;
        }
        const int bv = rem;  // block (bu, bv), bv <= bu
        const double* pu[4];
        const double* pv[4];
        bool free_e[4][4], ok[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          const int u = 4 * bu + a, v = 4 * bv + a;
          const int uu = u < nv ? u : 0, vv = v < nv ? v : 0;
          pu[a] = uu < col ? WY(uu) : WS(uu - col);
          pv[a] = vv < col ? WY(vv) : WS(vv - col);
        }
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const int u = 4 * bu + a, v = 4 * bv + b;
            ok[a][b] = u < nv && v < nv && v <= u;
            // Y.Y free; S.S active; S_i.Y_j (u = col + i, v = j) free iff i <= j
            free_e[a][b] = v < col && (u < col || u - col <= v);
          }
        double acc[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) acc[a][b] = 0.0;
#pragma unroll 2
        for (int k = c.wlane(); k < n; k += 64) {
          const bool fr = iwhere[k] <= 0;
          double xu[4], xv[4];
#pragma unroll
          for (int a = 0; a < 4; ++a) {
            xu[a] = pu[a][k];
            xv[a] = pv[a][k];
          }
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b)
              if (ok[a][b] && free_e[a][b] == fr) acc[a][b] += xu[a] * xv[b];
        }
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) acc[a][b] = c.wave_sum(acc[a][b]);
        if (c.wlane() == 0) {
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              if (!ok[a][b]) continue;
              const int u = 4 * bu + a, v = 4 * bv + b;
              const double sm = acc[a][b];
              if (u < col) {  // Y_u . Y_v over the free set
                double val = sm / theta;
                if (u == v) val += S.sy[u + u * MMAX];
                S.wn[v + u * M2] = val;
              } else if (v >= col) {  // S_i . S_j over the active set
                S.wn[(v) + (u) * M2] = sm * theta;
              } else {  // S_i . Y_j: -L_a (i > j, active) / R_z (i <= j, free)
                S.wn[v + u * M2] = (u - col > v) ? -sm : sm;
              }
            }
        }
      }
    }
  }

  BO_HD int formk() {
    const int col = S.i[I_COL];
    const int nfree = S.i[I_NFREE];
    const double theta = S.d[D_THETA];
    const int ntri = col * (col + 1) / 2;
    const int npairs = WIDE ? 0 : 2 * ntri + col * col;
    if constexpr (WIDE) formk_wide();
    for (int p = c.lane; p < npairs; p += C::NL) {
      int kind, i, j;
      if (p < 2 * ntri) {
        kind = p < ntri ? 0 : 1;
        int q = p < ntri ? p : p - ntri;
        i = 0;
        while (q > i) {
          q -= i + 1;
          ++i;
        }
        j = q;  // j <= i
      } else {
        kind = 2;
        i = (p - 2 * ntri) / col;  // S index
        j = (p - 2 * ntri) % col;  // Y index
      }
      double s = 0.0;
      if (kind == 0) {  // Y' ZZ' Y
        const double *a = WY(i), *b = WY(j);
        #pragma unroll 8  // loads issue ahead; the sum keeps its order
        for (int k = 0; k < nfree; ++k) s += a[index[k]] * b[index[k]];
        double v = s / theta;
        if (i == j) v += S.sy[i + i * MMAX];
        S.wn[j + i * M2] = v;
      } else if (kind == 1) {  // S' AA' S
        const double *a = WS(i), *b = WS(j);
        #pragma unroll 8  // loads issue ahead; the sum keeps its order
        for (int k = nfree; k < n; ++k) s += a[index[k]] * b[index[k]];
        S.wn[(col + j) + (col + i) * M2] = s * theta;
      } else {  // L_a (i > j, active) / R_z (i <= j, free) of S' . Y
        const double *a = WS(i), *b = WY(j);
        if (i > j) {
          #pragma unroll 8  // loads issue ahead; the sum keeps its order
          for (int k = nfree; k < n; ++k) s += a[index[k]] * b[index[k]];
          S.wn[j + (col + i) * M2] = -s;
        } else {
          #pragma unroll 8  // loads issue ahead; the sum keeps its order
          for (int k = 0; k < nfree; ++k) s += a[index[k]] * b[index[k]];
          S.wn[j + (col + i) * M2] = s;
        }
      }
    }
    c.sync();
    // LEL^T: the upper-left Cholesky, then the col right-hand columns' solves
    // and the lower-right block's col(col+1)/2 products spread over the lanes
    // (each column / entry computed by one lane exactly as the serial loops
    // do: the same values), then the lower-right Cholesky
    if (c.lane == 0) S.k0 = dpofa(S.wn, M2, col) ? -1 : 0;
    c.sync();
    if (S.k0 == 0) {
      for (int js = col + c.lane; js < 2 * col; js += C::NL) dtrsl_t(S.wn, M2, col, S.wn + js * M2);
      c.sync();
      for (int e = c.lane; e < ntri; e += C::NL) {
        int is = 0, q = e;  // e -> (is, js), col <= is <= js < 2 col, row-major over is
        while (q >= col - is) {
          q -= col - is;
          ++is;
        }
        const int js = col + is + q;
        is += col;
        double s = 0.0;
        #pragma unroll 4
        for (int k = 0; k < col; ++k) s += S.wn[k + is * M2] * S.wn[k + js * M2];
        S.wn[is + js * M2] += s;
      }
      c.sync();
      if (c.lane == 0 && dpofa(S.wn + col + col * M2, M2, col)) S.k0 = -2;
    }
    c.sync();
    return S.k0;
  }

  // ---- cmprlb: reduced gradient rs = -Z'(B (z - x) + g) on the free set ----
  BO_HD int cmprlb(bool unconstrained) {
    const int col = S.i[I_COL];
    const int nfree = S.i[I_NFREE];
    const double theta = S.d[D_THETA];
    if (unconstrained) {
      BO_UNROLL4
      for (int i = c.lane; i < n; i += C::NL) rs[i] = -g[i];
      c.sync();
      return 0;
    }
    if (c.lane == 0) S.k0 = bmv(S.sy, S.wt, col, S.c, S.v) ? -8 : 0;
    c.sync();
    if (S.k0) return S.k0;
    BO_UNROLL4
    for (int i = c.lane; i < nfree; i += C::NL) {
      const int k = index[i];
      double acc = -theta * (z[k] - x[k]) - g[k];
      for (int j = 0; j < col; ++j) acc = acc + WY(j)[k] * S.v[j] + WS(j)[k] * (theta * S.v[col + j]);
      rs[i] = acc;
    }
    c.sync();
    return 0;
  }

  // ---- subsm: subspace minimisation over the free set, then the v3.0 projection ----
  BO_HD int subsm() {
    const int col = S.i[I_COL];
    const int nsub = S.i[I_NFREE];
    const double theta = S.d[D_THETA];
    if (nsub <= 0) return 0;
    if constexpr (WIDE) {
      wdots<true>(rs, nsub, S.wv);
      if (c.lane == 0)
        for (int j = 0; j < col; ++j) S.wv[col + j] *= theta;
    } else {
      for (int j = 0; j < col; ++j) {
        const double *wy = WY(j), *ws = WS(j);
        double a = 0.0, b = 0.0;
        BO_UNROLL4
        for (int i = c.lane; i < nsub; i += C::NL) {
          a += wy[index[i]] * rs[i];
          b += ws[index[i]] * rs[i];
        }
        a = c.sum(a);
        b = c.sum(b);
        if (c.lane == 0) {
          S.wv[j] = a;
          S.wv[col + j] = theta * b;
        }
      }
    }
    c.sync();
    if (c.lane == 0) {
      int info = dtrsl_t(S.wn, M2, 2 * col, S.wv);
      if (!info) {
        for (int i = 0; i < col; ++i) S.wv[i] = -S.wv[i];
        info = dtrsl_n(S.wn, M2, 2 * col, S.wv);
      }
      S.k0 = info;
    }
    c.sync();
    if (S.k0) return S.k0;
    const double rtheta = 1.0 / theta;
    double iword = 0.0;
    BO_UNROLL4
    for (int i = c.lane; i < nsub; i += C::NL) {
      const int k = index[i];
      double acc = rs[i];
      for (int jy = 0; jy < col; ++jy) acc = acc + WY(jy)[k] * S.wv[jy] / theta + WS(jy)[k] * S.wv[col + jy];
      rs[i] = acc * rtheta;
    }
    BO_UNROLL4
    for (int i = c.lane; i < n; i += C::NL) xp[i] = z[i];
    c.sync();
    BO_UNROLL4
    for (int i = c.lane; i < nsub; i += C::NL) {  // projected Newton point
      const int k = index[i];
      const double dk = rs[i];
      const double xk = z[k];
      const int nb = nbd(k);
      double v;
      if (nb == 1) {
        v = fmax(lo(k), xk + dk);
        if (v == lo(k)) iword = 1.0;
      } else if (nb == 2) {
        v = fmin(hi(k), fmax(lo(k), xk + dk));
        if (v == lo(k) || v == hi(k)) iword = 1.0;
      } else if (nb == 3) {
        v = fmin(hi(k), xk + dk);
        if (v == hi(k)) iword = 1.0;
      } else {
        v = xk + dk;
      }
      z[k] = v;
    }
    iword = c.max(iword);
    c.sync();
    if (iword == 0.0) return 0;
    double ddp = 0.0;
    BO_UNROLL4
    for (int i = c.lane; i < n; i += C::NL) ddp += (z[i] - x[i]) * g[i];
    ddp = c.sum(ddp);
    if (!(ddp > 0.0)) return 0;
    // positive directional derivative of the projection: the backtracking step
    BO_UNROLL4
    for (int i = c.lane; i < n; i += C::NL) z[i] = xp[i];
    c.sync();
    double cand = __builtin_inf();
    int ibd = nsub;
    BO_UNROLL4
    for (int i = c.lane; i < nsub; i += C::NL) {
      const int k = index[i];
      const double dk = rs[i];
      const int nb = nbd(k);
      double ci = __builtin_inf();
      if (nb != 0) {
        if (dk < 0.0 && nb <= 2) {
          const double temp2 = lo(k) - z[k];
          ci = temp2 >= 0.0 ? 0.0 : temp2 / dk;
        } else if (dk > 0.0 && nb >= 2) {
          const double temp2 = hi(k) - z[k];
          ci = temp2 <= 0.0 ? 0.0 : temp2 / dk;
        }
      }
      if (ci < cand) {
        cand = ci;
        ibd = i;
      }
    }
    c.argmin(cand, ibd);
    const double alpha = fmin(1.0, cand);
    c.sync();
    if (c.lane == 0 && alpha < 1.0) {
      const int k = index[ibd];
      const double dk = rs[ibd];
      if (dk > 0.0) {
        z[k] = hi(k);
        rs[ibd] = 0.0;
      } else if (dk < 0.0) {
        z[k] = lo(k);
        rs[ibd] = 0.0;
      }
    }
    c.sync();
    BO_UNROLL4
    for (int i = c.lane; i < nsub; i += C::NL) z[index[i]] += alpha * rs[i];
    c.sync();
    return 0;
  }

  // trial point of the line search: z at stp = 1, t + stp d otherwise
  BO_HD void write_trial() {
    const double stp = S.d[D_STP];
    BO_UNROLL4
    for (int i = c.lane; i < n; i += C::NL) R.xt[i] = (stp == 1.0) ? z[i] : stp * dd[i] + t[i];
  }

  // line-search failure or ascent direction: restore the iterate; stop
  // without memory, else refresh it and recompute the direction
  BO_HD bool restore_or_refresh() {
    BO_UNROLL4
    for (int i = c.lane; i < n; i += C::NL) {
      x[i] = t[i];
      g[i] = r[i];
    }
    if (c.lane == 0) S.d[D_F] = S.d[D_FOLD];
    c.sync();
    if (S.i[I_COL] == 0) {
      stop(ST_ABNORMAL);
      return false;
    }
    refresh();
    return true;
  }

  // ---- label 222: new search direction and the first trial step ----
  BO_HD void direction() {
    for (int pass = 0; pass < 4; ++pass) {
      const int col = S.i[I_COL];
      const bool unconstrained = !cnstnd && col > 0;
      if (unconstrained) {
        BO_UNROLL4
        for (int i = c.lane; i < n; i += C::NL) {
          z[i] = x[i];
          index[i] = i;
        }
        if (c.lane == 0) S.i[I_NFREE] = n;
        c.sync();
      } else {
        tick(6);
        const int info = cauchy();
        tick(1);
        if (info) {
          refresh();
          continue;
        }
        freev();
        tick(2);
      }
      if (S.i[I_NFREE] != 0 && S.i[I_COL] != 0) {
        int info = formk();
        tick(3);
        if (!info) info = cmprlb(unconstrained);
        tick(4);
        if (!info) info = subsm();
        tick(5);
        if (info) {
          refresh();
          continue;
        }
      }
      // lnsrlb (first entry)
      BO_UNROLL4
      for (int i = c.lane; i < n; i += C::NL) dd[i] = z[i] - x[i];
      c.sync();
      const double dtd = dot(dd, dd);
      const double dnorm = sqrt(dtd);
      double stpmx = BIG;
      if (cnstnd) {
        if (S.i[I_ITER] == 0) {
          stpmx = 1.0;
        } else {
          double sm = BIG;
          BO_UNROLL4
          for (int i = c.lane; i < n; i += C::NL) {
            const double a1 = dd[i];
            const int nb = nbd(i);
            if (nb == 0) continue;
            if (a1 < 0.0 && nb <= 2) {
              const double a2 = lo(i) - x[i];
              sm = fmin(sm, a2 >= 0.0 ? 0.0 : a2 / a1);
            } else if (a1 > 0.0 && nb >= 2) {
              const double a2 = hi(i) - x[i];
              sm = fmin(sm, a2 <= 0.0 ? 0.0 : a2 / a1);
            }
          }
          stpmx = c.min(sm);
        }
      }
      const double stp = (S.i[I_ITER] == 0 && !boxed) ? fmin(1.0 / dnorm, stpmx) : 1.0;
      BO_UNROLL4
      for (int i = c.lane; i < n; i += C::NL) {
        t[i] = x[i];
        r[i] = g[i];
      }
      const double gd = dot(g, dd);
      c.sync();
      if (c.lane == 0) {
        S.d[D_FOLD] = S.d[D_F];
        S.d[D_DTD] = dtd;
        S.d[D_STPMX] = stpmx;
        S.d[D_STP] = stp;
        S.d[D_GD] = gd;
        S.d[D_GDOLD] = gd;
        S.i[I_IFUN] = 0;
        S.i[I_IBACK] = 0;
      }
      c.sync();
      if (gd >= 0.0) {  // ascent direction: the line search is impossible
        if (restore_or_refresh()) continue;
        return;
      }
      if (c.lane == 0) S.k0 = dcsrch_start(S.d, S.i, S.d[D_F], gd, stp, 0.0, stpmx);
      c.sync();
      if (S.k0) {
        stop(ST_ERROR);
        return;
      }
      if (c.lane == 0) {
        S.i[I_IFUN] = 1;
        S.i[I_IBACK] = 0;
        S.i[I_PHASE] = PH_LNSRCH;
      }
      c.sync();
      write_trial();
      return;
    }
    stop(ST_ABNORMAL);  // not reached: a refreshed memory cannot fail again
  }

  // ---- matupd + formt after an accepted step ----
  BO_HD void update() {
    BO_UNROLL4
    for (int i = c.lane; i < n; i += C::NL) r[i] = g[i] - r[i];
    c.sync();
    const double rr = dot(r, r);
    const double stp = S.d[D_STP];
    const double gd = S.d[D_GD], gdold = S.d[D_GDOLD];
    double dr, ddum;
    if (stp == 1.0) {
      dr = gd - gdold;
      ddum = -gdold;
    } else {
      dr = (gd - gdold) * stp;
      BO_UNROLL4
      for (int i = c.lane; i < n; i += C::NL) dd[i] *= stp;
      ddum = -gdold * stp;
    }
    c.sync();
    if (dr <= EPSMCH * ddum) return;  // skip the L-BFGS update
    if (c.lane == 0) {
      const int iupdat = ++S.i[I_IUPDAT];
      if (iupdat <= m) {
        S.i[I_COL] = iupdat;
        S.i[I_ITAIL] = (S.i[I_HEAD] + iupdat - 1) % m;
      } else {
        S.i[I_ITAIL] = (S.i[I_ITAIL] + 1) % m;
        S.i[I_HEAD] = (S.i[I_HEAD] + 1) % m;
      }
    }
    c.sync();
    const int col = S.i[I_COL];
    const int itail = S.i[I_ITAIL];
    BO_UNROLL4
    for (int i = c.lane; i < n; i += C::NL) {
      R.ws[(long)itail * n + i] = dd[i];
      R.wy[(long)itail * n + i] = r[i];
    }
    if (c.lane == 0) {
      S.d[D_THETA] = rr / dr;
      if (S.i[I_IUPDAT] > m) {  // move old information
        for (int j = 0; j < col - 1; ++j) {
          for (int k = 0; k <= j; ++k) S.ss[k + j * MMAX] = S.ss[(k + 1) + (j + 1) * MMAX];
          for (int k = j; k < col - 1; ++k) S.sy[k + j * MMAX] = S.sy[(k + 1) + (j + 1) * MMAX];
        }
      }
    }
    c.sync();
    if constexpr (WIDE) {  // new row of SY, new column of SS
      wdots<false>(dd, n, S.wbp);  // (the Cauchy search's scratch, free here)
      if (c.lane == 0)
        for (int j = 0; j < col - 1; ++j) {
          S.sy[(col - 1) + j * MMAX] = S.wbp[j];
          S.ss[j + (col - 1) * MMAX] = S.wbp[col + j];
        }
    } else {
      for (int j = 0; j < col - 1; ++j) {
        const double a = dot(dd, WY(j));
        const double b = dot(WS(j), dd);
        if (c.lane == 0) {
          S.sy[(col - 1) + j * MMAX] = a;
          S.ss[j + (col - 1) * MMAX] = b;
        }
      }
    }
    if (c.lane == 0) {
      const double dtd = S.d[D_DTD];
      S.ss[(col - 1) + (col - 1) * MMAX] = (stp == 1.0) ? dtd : stp * stp * dtd;
      S.sy[(col - 1) + (col - 1) * MMAX] = dr;
      S.k0 = formt(S.wt, S.sy, S.ss, col, S.d[D_THETA]);
    }
    c.sync();
    if (S.k0) refresh();
  }

  // ---- the call: consume f, g at xt; run to the next evaluation ----
  BO_HD void run(unsigned long long* prof_b) {
    prof = prof_b;
    if (prof) tprev = c.clock();
    // load the persistent record
    for (int k = c.lane; k < DSLOTS; k += C::NL) S.d[k] = R.ds[k];
    for (int k = c.lane; k < ISLOTS; k += C::NL) S.i[k] = R.is[k];
    for (int k = c.lane; k < MMAX * MMAX; k += C::NL) {
      S.sy[k] = R.mat[k];
      S.ss[k] = R.mat[MMAX * MMAX + k];
      S.wt[k] = R.mat[2 * MMAX * MMAX + k];
    }
    double anyb = 0.0, allbox = 1.0;
    BO_UNROLL4
    for (int i = c.lane; i < n; i += C::NL) {
      const int nb = nbd(i);
      if (nb != 0) anyb = 1.0;
      if (nb != 2) allbox = 0.0;
    }
    cnstnd = c.max(anyb) > 0.0;
    boxed = c.min(allbox) > 0.0;
    c.sync();
    const int phase = S.i[I_PHASE];
    if (phase == PH_STOP) {
      BO_UNROLL4
      for (int i = c.lane; i < n; i += C::NL) R.xt[i] = x[i];
      return;
    }
    const double fnew = R.f_new;
    double finite = (fnew - fnew == 0.0) ? 1.0 : 0.0;
    BO_UNROLL4
    for (int i = c.lane; i < n; i += C::NL) {
      const double gi = R.g_new[i];
      if (!(gi - gi == 0.0)) finite = 0.0;
    }
    finite = c.min(finite);
    tick(0);
    if (phase == PH_START) {
      BO_UNROLL4
      for (int i = c.lane; i < n; i += C::NL) {
        x[i] = R.xt[i];
        g[i] = R.g_new[i];
        const int nb = nbd(i);
        iwhere[i] = nb == 0 ? -1 : ((nb == 2 && hi(i) - lo(i) <= 0.0) ? 3 : 0);
      }
      if (c.lane == 0) {
        for (int k = 0; k < DSLOTS; ++k) S.d[k] = 0.0;
        for (int k = 0; k < ISLOTS; ++k) S.i[k] = 0;
        S.d[D_F] = fnew;
        S.d[D_THETA] = 1.0;
        S.i[I_NFEV] = 1;
      }
      c.sync();
      if (finite == 0.0) {
        stop(ST_ERROR);
      } else {
        const double sb = projgr();
        if (c.lane == 0) S.d[D_SBGNRM] = sb;
        c.sync();
        if (sb <= P.pgtol)
          stop(ST_CONV_PGTOL);
        else
          direction();
      }
    } else {  // PH_LNSRCH: x <- the trial point
      BO_UNROLL4
      for (int i = c.lane; i < n; i += C::NL) {
        x[i] = R.xt[i];
        g[i] = R.g_new[i];
      }
      if (c.lane == 0) {
        S.d[D_F] = fnew;
        S.i[I_NFEV] += 1;
      }
      c.sync();
      if (finite == 0.0) {  // a non-finite trial value: keep the last iterate
        BO_UNROLL4
        for (int i = c.lane; i < n; i += C::NL) {
          x[i] = t[i];
          g[i] = r[i];
        }
        if (c.lane == 0) S.d[D_F] = S.d[D_FOLD];
        stop(ST_ERROR);
      } else {
        const double gd = dot(g, dd);
        if (c.lane == 0) {
          double stp = S.d[D_STP];
          S.k0 = dcsrch_cont(S.d, S.i, fnew, gd, stp, 0.0, S.d[D_STPMX]);
          S.d[D_STP] = stp;
          S.d[D_GD] = gd;
          if (S.k0 == 0) {
            S.i[I_IFUN] += 1;
            S.i[I_IBACK] = S.i[I_IFUN] - 1;
          }
        }
        c.sync();
        if (S.k0 == 0) {  // FG: another trial step
          if (S.i[I_IBACK] >= P.maxls) {
            if (restore_or_refresh()) direction();
          } else {
            write_trial();
          }
        } else {  // NEW_X
          const double sb = projgr();
          if (c.lane == 0) {
            S.d[D_SBGNRM] = sb;
            S.i[I_ITER] += 1;
            S.i[I_NITER] += 1;
          }
          c.sync();
          const double fold = S.d[D_FOLD], f = S.d[D_F];
          if (S.i[I_NITER] >= P.maxiter) {
            stop(ST_MAXITER);
          } else if (S.i[I_NFEV] > P.maxfun) {
            stop(ST_MAXFUN);
          } else if (sb <= P.pgtol) {
            stop(ST_CONV_PGTOL);
          } else if (fold - f <= P.tol * fmax(fmax(fabs(fold), fabs(f)), 1.0)) {
            stop(ST_CONV_FTOL);
          } else {
            update();
            direction();
          }
        }
      }
    }
    c.sync();
    tick(6);
    if (S.i[I_PHASE] == PH_STOP)
      BO_UNROLL4
      for (int i = c.lane; i < n; i += C::NL) R.xt[i] = x[i];
    for (int k = c.lane; k < DSLOTS; k += C::NL) R.ds[k] = S.d[k];
    for (int k = c.lane; k < ISLOTS; k += C::NL) R.is[k] = S.i[k];
    for (int k = c.lane; k < MMAX * MMAX; k += C::NL) {
      R.mat[k] = S.sy[k];
      R.mat[MMAX * MMAX + k] = S.ss[k];
      R.mat[2 * MMAX * MMAX + k] = S.wt[k];
    }
    tick(7);
  }
};

}  // namespace bolb
