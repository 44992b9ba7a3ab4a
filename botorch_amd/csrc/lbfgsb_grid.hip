// The joint L-BFGS-B step spread over the chip: ONE restart of n = b q d
// variables -- gen_candidates_device(joint=True), the reference's own problem
// (botorch/generation/gen.py:252-267: one scipy L-BFGS-B over all restarts'
// variables and -sum_b acq) -- on G workgroups of 256 threads, one per CU.
// Workgroup w owns the variables [256 w, 256 w + 256) and their slice of the
// S / Y ring (the 2 m history vectors), all in LDS for the launch.
//
// Why: the one-workgroup kernel (lbfgsb.hip, 16 waves) streams the 2 m n ring
// through ONE CU for every product of an iteration -- formk's Gram matrix,
// W^T dc, W^T rs, the new SY / SS row, cmprlb's and subsm's W v -- about 35 MB
// per iteration at C3 (n = 12 288), which one CU moves at ~150 GB/s: 690 us
// per launch.  Here the ring is read once per launch (2 m n doubles spread over
// G CUs), every product reduces inside its workgroup first, and workgroups
// meet only at the grid exchanges the algorithm needs: the first pass (finite
// check, bounds, g.d, projected gradient), the new memory row, the Cauchy pass
// and its breakpoint rounds, formk's Gram matrix, subsm's W^T rs, projection
// and backtracking, the line-search start.  The 2m x 2m algebra (bmv, formt,
// the LEL^T factor, dcsrch) runs redundantly in every workgroup on values
// that are bit-identical everywhere (every workgroup combines the published
// partials in workgroup order), so all workgroups take the same branches
// without any further exchange.
//
// Exchange (MI355X_MICROARCH.md, inter-workgroup visibility, the hand-off row
// "one lane of each storing workgroup ... agent-scope atomic add"): partials
// stored write-through (sc1), every storing wave drains (vmcnt(0)), workgroup
// barrier, one lane adds to the arrival counter; readers poll the counter with
// sc1 loads and read the partials with sc1 loads only.  Counters count up
// through the launch; the last workgroup to leave resets them, so the next
// launch on the stream starts from zero.  Every wait is bounded (2 s): a
// grid that is not co-resident aborts with status ERROR instead of hanging.
//
// The Cauchy search walks the breakpoints in increasing order (scipy's heap):
// each round every workgroup publishes its KB smallest breakpoints with the
// data the walk needs (d_i, the bound, the ring row), wave 0 of every
// workgroup merges the G sorted lists into the global order -- as far as it is
// known: a workgroup with more breakpoints than it published caps what can be
// taken -- and walks them; the explicit middle matrix M (2col x 2col, column j
// = bmv(e_j)) turns each breakpoint's bmv into 2col-lane products.
//
// Summation order differs from scipy's (and from the one-workgroup kernel's)
// in the dot products, as there: the trial points agree to rounding
// (tests/test_gpu_lbfgsb.py, the grid path forced).
#include "common.h"

#include <atomic>
#include <map>
#include <mutex>
#include <utility>

#pragma clang fp contract(off)  // scipy's rounding (lbfgsb.hip)

#define BO_HD __device__ __attribute__((always_inline))
#include "lbfgsb_core.h"

// BO_GRID_SUBPROF (development builds): the profile slots time sub-phases
// instead -- 0 load + first exchange, 1 Cauchy pass + exchange, 2 bmv + M,
// 3 breakpoint selection + exchange, 4 merge + walk, 5 formk products +
// exchange, 6 LEL^T + cmprlb + subsm, 7 update, line-search start, stores.
#ifdef BO_GRID_SUBPROF
#define SUBTICK(p) tick(p)
#define PHTICK(p)
#else
#define SUBTICK(p)
#define PHTICK(p) tick(p)
#endif

namespace {

using namespace bolb;

constexpr int GT = 256;       // threads per workgroup
constexpr int GWV = GT / 64;  // waves per workgroup
constexpr int SL = GT;        // variables per workgroup (one per thread)
constexpr int WP = SL + 16;   // LDS pitch of a ring column's slice (rows start in other banks)
constexpr int GMAX = 64;      // workgroups (n <= GMAX * SL)
constexpr int PK = 1024;      // published doubles per workgroup per exchange
constexpr int KB = 8;         // Cauchy breakpoints a workgroup publishes per round
constexpr int MPAY = 32;      // breakpoints walked per round at most
constexpr int HW = 1 + 2 * KB;          // header: more, KB breakpoints, KB indices
constexpr int PWMAX = 3 + 2 * MMAX;     // payload of one breakpoint: d, z - x, bound, ring row
// LDS exchange area (doubles): local record | M | headers | payloads
constexpr int R_REC = 0;
constexpr int R_MX = HW + KB * PWMAX;   // 361
constexpr int R_HDR = R_MX + M2 * M2;   // + 1600
constexpr int R_PAY = R_HDR + GMAX * HW;
constexpr int RED = R_PAY + MPAY * PWMAX;
static_assert(HW + KB * PWMAX <= PK, "a workgroup's breakpoint record fits its partial slot");
static_assert(1 + M2 * (M2 + 1) / 2 <= RED && 1 + M2 * (M2 + 1) / 2 <= PK,
              "formk's Gram matrix fits the exchange area and a partial slot");
constexpr long long SPIN_TIMEOUT = 200000000;  // 2 s of the 100 MHz wall clock

enum LV : int { L_X, L_G, L_T, L_R, L_Z, L_D, L_DC, L_TB, L_RS, L_XP, L_LO, L_HI, L_COUNT };
enum Op : int { O_SUM = 0, O_MAX = 1, O_MIN = 2 };

struct GridMem {
  double* part;    // [2][GMAX][PK] published partials (double-buffered by exchange parity)
  unsigned* cnt;   // [0] arrivals, [1] departures, [2] abort word
};

__host__ __device__ constexpr size_t grid_dyn_bytes(int m) {
  return sizeof(double) * ((size_t)L_COUNT * SL + 2 * (size_t)m * WP + RED) + sizeof(int) * SL;
}

BO_HD void st_wt(double* p, double v) {  // write-through (sc1) store
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Exchange reads as buffer loads with the sc1 policy (L1 bypassed, as the
// hand-off needs): unlike atomic loads they issue back to back, eight in
// flight per lane, instead of one cross-XCD latency each.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr int SC1 = 16;
BO_HD rsrc_t make_rsrc(const double* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, (int)bytes, 0x00020000);
}
BO_HD double ldb(rsrc_t r, int idx) {  // element idx (doubles) of the resource
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (unsigned)idx * 8u, 0, SC1));
}
BO_HD unsigned ld_u32(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
BO_HD double opf(int op, double a, double b) {
  return op == O_SUM ? a + b : (op == O_MAX ? fmax(a, b) : fmin(a, b));
}
// (value, index) order of the breakpoint / backtracking searches: smaller
// value first, ties to the smaller index
BO_HD bool before(double v, int i, double w, int j) { return v < w || (v == w && i < j); }

BO_HD double wave_op(double v, int op) {
  for (int o = 32; o > 0; o >>= 1) v = opf(op, v, __shfl_xor(v, o));
  return v;
}
BO_HD double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
BO_HD void wave_argmin(double& v, int& i) {
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(v, o);
    const int oi = __shfl_xor(i, o);
    if (before(ov, oi, v, i)) {
      v = ov;
      i = oi;
    }
  }
}

// ---- the 2m x 2m algebra on one wave (lane = row or column index) -----------
// lbfgsb_core.h runs these on one lane, where every step waits on an LDS
// round trip and many on an fp64 division: ~10 us per bmv, ~5-10 per dpofa
// at col = 10.  Here they are column- / row-parallel over the wave's lanes
// (col <= MMAX, 2 col <= 40 < 64): the same operations on the same values,
// in another summation order (the triangular solves and the Cholesky update
// right-looking); results are uniform or land in LDS.  Wave 0 only; the
// caller's barrier publishes them.
BO_HD double readlane_d(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// upper Cholesky A = R^T R of the n x n leading block (column-major, ld) in
// place, LINPACK dpofa's result: 0 or the failing column + 1 (uniform)
BO_HD int dpofa_w(double* a, int ld, int n, int lane) {
  for (int k = 0; k < n; ++k) {
    const double d = a[k + k * ld];
    if (d <= 0.0) return k + 1;
    const double r = sqrt(d);
    double akj = 0.0;
    if (lane > k && lane < n) akj = a[k + lane * ld] / r;
    __builtin_amdgcn_wave_barrier();
    if (lane == k) a[k + k * ld] = r;
    if (lane > k && lane < n) a[k + lane * ld] = akj;
    __builtin_amdgcn_wave_barrier();
    if (lane > k && lane < n)  // a[i][j] -= R[k][i] R[k][j], k < i <= j (lane j)
      for (int i = k + 1; i <= lane; ++i) a[i + lane * ld] -= a[k + i * ld] * akj;
    __builtin_amdgcn_wave_barrier();
  }
  return 0;
}
// first zero on T's diagonal + 1, or 0 (uniform)
BO_HD int zero_diag_w(const double* t, int ld, int n, int lane) {
  const unsigned long long z = __ballot(lane < n && t[lane + lane * ld] == 0.0);
  return z ? __builtin_ffsll((long long)z) : 0;
}
// T^T x = b (T upper; dtrsl job 11), b in LDS, overwritten by x
BO_HD int dtrsl_t_w(const double* t, int ld, int n, double* b, int lane) {
  const int info = zero_diag_w(t, ld, n, lane);
  if (info) return info;
  double bj = lane < n ? b[lane] : 0.0;
  for (int i = 0; i < n; ++i) {
    const double xi = readlane_d(bj / t[i + i * ld], i);
    if (lane == i) bj = xi;
    if (lane > i && lane < n) bj -= t[i + lane * ld] * xi;
  }
  __builtin_amdgcn_wave_barrier();
  if (lane < n) b[lane] = bj;
  __builtin_amdgcn_wave_barrier();
  return 0;
}
// T x = b (T upper; dtrsl job 01)
BO_HD int dtrsl_n_w(const double* t, int ld, int n, double* b, int lane) {
  const int info = zero_diag_w(t, ld, n, lane);
  if (info) return info;
  double bj = lane < n ? b[lane] : 0.0;
  for (int j = n - 1; j >= 0; --j) {
    const double xj = readlane_d(bj / t[j + j * ld], j);
    if (lane == j) bj = xj;
    if (lane < j) bj -= t[lane + j * ld] * xj;
  }
  __builtin_amdgcn_wave_barrier();
  if (lane < n) b[lane] = bj;
  __builtin_amdgcn_wave_barrier();
  return 0;
}
// bmv: p = M v for the 2col x 2col middle matrix (lbfgsb_core.h bmv; lane i
// does row i's sums in the serial order, the two solves are dtrsl_*_w)
BO_HD int bmv_w(const double* sy, const double* wt, int col, const double* v, double* p, int lane) {
  if (col == 0) return 0;
  if (lane < col) {
    if (lane == 0) {
      p[col] = v[col];
    } else {
      double sum = 0.0;
      for (int k = 0; k < lane; ++k) sum += sy[lane + k * MMAX] * v[k] / sy[k + k * MMAX];
      p[col + lane] = v[col + lane] + sum;
    }
  }
  __builtin_amdgcn_wave_barrier();
  int info = dtrsl_t_w(wt, MMAX, col, p + col, lane);
  if (info) return info;
  if (lane < col) p[lane] = v[lane] / sqrt(sy[lane + lane * MMAX]);
  __builtin_amdgcn_wave_barrier();
  info = dtrsl_n_w(wt, MMAX, col, p + col, lane);
  if (info) return info;
  if (lane < col) {
    const double sii = sy[lane + lane * MMAX];
    double pi = -p[lane] / sqrt(sii);
    double sum = 0.0;
    for (int k = lane + 1; k < col; ++k) sum += sy[k + lane * MMAX] * p[col + k] / sii;
    p[lane] = pi + sum;
  }
  __builtin_amdgcn_wave_barrier();
  return 0;
}
// formt: WT = chol(theta SS + L D^-1 L^T), entries (i, j), i <= j, over the lanes
BO_HD int formt_w(double* wt, const double* sy, const double* ss, int col, double theta, int lane) {
  const int np = col * (col + 1) / 2;
  for (int e = lane; e < np; e += 64) {
    int i = 0, q = e;  // e -> (i, j), i <= j, row-major over i
    while (q >= col - i) {
      q -= col - i;
      ++i;
    }
    const int j = i + q;
    if (i == 0) {
      wt[0 + j * MMAX] = theta * ss[0 + j * MMAX];
    } else {
      double ddum = 0.0;
      for (int k = 0; k < i; ++k) ddum += sy[i + k * MMAX] * sy[j + k * MMAX] / sy[k + k * MMAX];
      wt[i + j * MMAX] = ddum + theta * ss[i + j * MMAX];
    }
  }
  __builtin_amdgcn_wave_barrier();
  return dpofa_w(wt, MMAX, col, lane) ? -3 : 0;
}

struct CauchyState {  // the breakpoint walk's scalars, handed from wave 0 to the workgroup
  double f1, f2, dtm, tsum, tj;
  int nleft, done, all_fixed;
};

struct GStep {
  const Problem& P;
  const Restart& R;
  Shared& S;
  GridMem gm;
  int n, m, G, wg, tid, lane, wave, cnt;
  long base;
  double* L;     // L_COUNT x SL vectors
  double* wyl;   // m x WP ring slices
  double* wsl;
  double* red;   // RED exchange area
  int* iw;       // iwhere slice
  double* tmp;   // GWV x 8
  int* sflag;
  int* ordw;     // MPAY: workgroup of the k-th walked breakpoint
  int* ordh;     // MPAY: its position in that workgroup's list
  CauchyState* cs;
  int seq = 0;
  bool aborted = false;
  bool cnstnd = false, boxed = false;
  int new_slot = -1;  // ring slot written this launch (stored at the end)
  unsigned long long* prof = nullptr;
  unsigned long long tprev = 0;

  BO_HD double* V(int v) const { return L + v * SL; }
  BO_HD bool own() const { return tid < cnt; }
  BO_HD int slot(int j) const { return (S.i[I_HEAD] + j) % m; }
  BO_HD const double* WY(int j) const { return wyl + slot(j) * WP; }
  BO_HD const double* WS(int j) const { return wsl + slot(j) * WP; }
  BO_HD double lo(int k) const { return L[L_LO * SL + k]; }
  BO_HD double hi(int k) const { return L[L_HI * SL + k]; }
  BO_HD int nbd(int k) const { return nbd_of(lo(k), hi(k)); }
  BO_HD bool is_free(int k) const { return iw[k] <= 0; }

  BO_HD void tick(int phase) {
    if (!prof) return;
    const unsigned long long now = wall_clock64();
    if (tid == 0) prof[phase] += now - tprev;
    tprev = now;
  }

  // ---- workgroup reductions --------------------------------------------------
  // red[s0 + i] = op[i] over the workgroup's threads of v[i] (waves in order)
  template <int K>
  BO_HD void wg_reduce(double (&v)[K], const int (&op)[K], int s0) {
#pragma unroll
    for (int i = 0; i < K; ++i) v[i] = wave_op(v[i], op[i]);
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < K; ++i) tmp[wave * 8 + i] = v[i];
    __syncthreads();
    if (tid < K) {
      double r = tmp[tid];
      for (int w = 1; w < GWV; ++w) r = opf(op[tid], r, tmp[w * 8 + tid]);
      red[s0 + tid] = r;
    }
    __syncthreads();
  }

  // red[s0 + e] = sum over this workgroup's variables of a_e[k] b_e[k] (mode 0:
  // all, 1: free, 2: active), e < K; rows(e, a, b, mode).  16 lanes per entry,
  // strided over the slice, then a 16-lane butterfly (every lane of the group
  // ends with the same sum).
  template <class F>
  BO_HD void wg_products(int K, int s0, F rows) {
    const int sub = tid & 15, grp = tid >> 4;
    for (int e0 = 0; e0 < K; e0 += GT / 16) {
      const int e = e0 + grp;
      double s = 0.0;
      if (e < K) {
        const double* a;
        const double* b;
        int mode;
        rows(e, a, b, mode);
#pragma unroll 4
        for (int k = sub; k < cnt; k += 16) {
          const bool fr = is_free(k);
          if (mode == 0 || (mode == 1) == fr) s += a[k] * b[k];
        }
      }
      s += __shfl_xor(s, 8);
      s += __shfl_xor(s, 4);
      s += __shfl_xor(s, 2);
      s += __shfl_xor(s, 1);
      if (sub == 0 && e < K) red[s0 + e] = s;
    }
    __syncthreads();
  }

  // ---- grid exchange -----------------------------------------------------------
  // Publish src[0..K) (this workgroup's record), meet every workgroup.  The
  // records are then readable through parts() until the exchange after next.
  BO_HD bool publish_meet(const double* src, int K) {
    if (aborted) return false;
    double* mine = gm.part + ((size_t)(seq & 1) * GMAX + wg) * PK;
    for (int k = tid; k < K; k += GT) st_wt(mine + k, src[k]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      int ok = 1;
      __hip_atomic_fetch_add(gm.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)(seq + 1) * (unsigned)G;
      if (ld_u32(gm.cnt) < target) {
        const long long t0 = wall_clock64();
        for (;;) {
          __builtin_amdgcn_s_sleep(1);
          if (ld_u32(gm.cnt) >= target) break;
          if (ld_u32(gm.cnt + 2)) {
            ok = 0;
            break;
          }
          if (wall_clock64() - t0 > SPIN_TIMEOUT) {
            __hip_atomic_store(gm.cnt + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = 0;
            break;
          }
        }
      }
      *sflag = ok;
    }
    __syncthreads();
    const int ok = *sflag;
    ++seq;
    if (!ok) aborted = true;
    return ok != 0;
  }
  // the records of the last exchange as one resource: element w * PK + j
  BO_HD rsrc_t parts() const {
    return make_rsrc(gm.part + (size_t)((seq - 1) & 1) * GMAX * PK, (unsigned)(sizeof(double) * GMAX * PK));
  }
  // dst[t] = element (t / cols) * PK + off + t % cols of the last exchange's
  // records (t < G * cols), eight loads in flight per lane; ends with a barrier
  BO_HD void gather(double* dst, int off, int cols) {
    const rsrc_t rp = parts();
    const int tot = G * cols;
    for (int t0 = tid; t0 < tot; t0 += 8 * GT) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int t = t0 + u * GT;
        const int w = t / cols;
        v[u] = t < tot ? ldb(rp, w * PK + off + (t - w * cols)) : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (t0 + u * GT < tot) dst[t0 + u * GT] = v[u];
    }
    __syncthreads();
  }

  // red[0..K) (this workgroup's partials) -> the combination over all
  // workgroups in workgroup order: max for the bits of mx, min for mn, sums
  // otherwise.  Bit-identical in every workgroup.
  BO_HD bool greduce(int K, unsigned mx = 0, unsigned mn = 0) {
    if (!publish_meet(red, K)) return false;
    // the G x K partials gathered into LDS (behind red's first PK entries) in
    // chunks of columns, then each entry combined in workgroup order
    double* gath = red + PK;
    const int chunk = (RED - PK) / G;
    for (int k0 = 0; k0 < K; k0 += chunk) {
      const int kc = min(chunk, K - k0);
      gather(gath, k0, kc);
      for (int j = tid; j < kc; j += GT) {
        const int k = k0 + j;
        const int op = k < 32 ? (((mx >> k) & 1) ? O_MAX : (((mn >> k) & 1) ? O_MIN : O_SUM)) : O_SUM;
        double r = gath[j];
        for (int w = 1; w < G; ++w) r = opf(op, r, gath[w * kc + j]);
        red[k] = r;
      }
      __syncthreads();
    }
    return true;
  }

  // (v, i) -> the grid's smallest (v, i) (ties to the smaller index), on every thread
  BO_HD void gargmin(double& v, int& i) {
    wave_argmin(v, i);
    if (lane == 0) {
      tmp[wave * 8] = v;
      tmp[wave * 8 + 1] = (double)i;
    }
    __syncthreads();
    if (tid == 0) {
      double bv = tmp[0];
      int bi = (int)tmp[1];
      for (int w = 1; w < GWV; ++w)
        if (before(tmp[w * 8], (int)tmp[w * 8 + 1], bv, bi)) {
          bv = tmp[w * 8];
          bi = (int)tmp[w * 8 + 1];
        }
      red[0] = bv;
      red[1] = (double)bi;
    }
    __syncthreads();
    if (!publish_meet(red, 2)) return;
    if (wave == 0) {
      double bv = __builtin_inf();
      int bi = n;
      if (lane < G) {
        const rsrc_t rp = parts();
        bv = ldb(rp, lane * PK);
        bi = (int)ldb(rp, lane * PK + 1);
      }
      wave_argmin(bv, bi);
      if (lane == 0) {
        tmp[0] = bv;
        tmp[1] = (double)bi;
      }
    }
    __syncthreads();
    v = tmp[0];
    i = (int)tmp[1];
    __syncthreads();
  }

  // ---- small steps -------------------------------------------------------------
  BO_HD void refresh() {
    __syncthreads();
    if (tid == 0) {
      S.i[I_INFO] = 0;
      S.i[I_COL] = 0;
      S.i[I_HEAD] = 0;
      S.d[D_THETA] = 1.0;
      S.i[I_IUPDAT] = 0;
    }
    __syncthreads();
  }
  BO_HD void stop(int status) {
    __syncthreads();
    if (tid == 0) {
      S.i[I_STATUS] = status;
      S.i[I_PHASE] = PH_STOP;
    }
    __syncthreads();
  }
  BO_HD double projg(int k) const {  // |projected gradient| of variable k
    const double* x = V(L_X);
    double gi = V(L_G)[k];
    const int nb = nbd(k);
    if (nb != 0) {
      if (gi < 0.0) {
        if (nb >= 2) gi = fmax(x[k] - hi(k), gi);
      } else {
        if (nb <= 2) gi = fmin(x[k] - lo(k), gi);
      }
    }
    return fabs(gi);
  }
  BO_HD void write_trial() {
    const double stp = S.d[D_STP];
    if (own()) {
      const int k = tid;
      R.xt[base + k] = (stp == 1.0) ? V(L_Z)[k] : stp * V(L_D)[k] + V(L_T)[k];
    }
  }
  BO_HD bool restore_or_refresh() {
    if (own()) {
      V(L_X)[tid] = V(L_T)[tid];
      V(L_G)[tid] = V(L_R)[tid];
    }
    if (tid == 0) S.d[D_F] = S.d[D_FOLD];
    __syncthreads();
    if (S.i[I_COL] == 0) {
      stop(ST_ABNORMAL);
      return false;
    }
    refresh();
    return true;
  }

  // ---- cauchy: generalized Cauchy point z; c = W^T (z - x) in S.c --------------
  BO_HD int cauchy() {
    const int col = S.i[I_COL];
    const double theta = S.d[D_THETA];
    const double inf = __builtin_inf();
    double* x = V(L_X);
    double* z = V(L_Z);
    double* dc = V(L_DC);
    double* tb = V(L_TB);
    if (S.d[D_SBGNRM] <= 0.0) {
      if (own()) z[tid] = x[tid];
      __syncthreads();
      return 0;
    }
    double f1 = 0.0, nbreak = 0.0, nunb = 0.0, moving = 0.0;
    if (own()) {
      const int k = tid;
      const double neggi = -V(L_G)[k];
      const int nb = nbd(k);
      int w = iw[k];
      double tl = 0.0, tu = 0.0;
      if (w != 3 && w != -1) {
        if (nb <= 2) tl = x[k] - lo(k);
        if (nb >= 2) tu = hi(k) - x[k];
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
        iw[k] = w;
      }
      double tbi = inf;
      if (w != 0 && w != -1) {
        dc[k] = 0.0;
      } else {
        dc[k] = neggi;
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
      tb[k] = tbi;
      z[k] = x[k];
    }
    {
      double vals[4] = {f1, nbreak, nunb, moving};
      const int ops[4] = {O_SUM, O_SUM, O_SUM, O_MAX};
      wg_reduce(vals, ops, 0);
    }
    if (col > 0)  // p = W^T dc
      wg_products(2 * col, 4, [&](int e, const double*& a, const double*& b, int& mode) {
        a = e < col ? WY(e) : WS(e - col);
        b = dc;
        mode = 0;
      });
    if (!greduce(4 + 2 * col, 1u << 3)) return 0;
    SUBTICK(1);
    f1 = red[0];
    const int nbrk = (int)red[1];
    const int nfr = (int)red[2];
    const bool bnded = red[3] == 0.0;
    if (tid == 0) {
      for (int j = 0; j < 2 * col; ++j) S.p[j] = red[4 + j];
      if (theta != 1.0)
        for (int j = 0; j < col; ++j) S.p[col + j] *= theta;
    }
    __syncthreads();
    if (nbrk == 0 && nfr == 0) {  // dc = 0: the GCP is x
      if (tid == 0)
        for (int j = 0; j < 2 * col; ++j) S.c[j] = 0.0;
      __syncthreads();
      return 0;
    }
    if (wave == 0) {
      if (lane < 2 * col) S.c[lane] = 0.0;
      const int info = col > 0 ? bmv_w(S.sy, S.wt, col, S.p, S.v, lane) : 0;
      if (lane == 0) {
        double f2 = -theta * f1;
        if (col > 0 && !info)
          for (int j = 0; j < 2 * col; ++j) f2 -= S.v[j] * S.p[j];
        S.t0 = f2;
        S.k0 = info;
      }
    }
    __syncthreads();
    if (S.k0) return S.k0;
    const double f2_org = -theta * f1;
    if (tid == 0) {
      cs->f1 = f1;
      cs->f2 = S.t0;
      cs->dtm = -f1 / S.t0;
      cs->tsum = 0.0;
      cs->tj = 0.0;
      cs->nleft = nbrk;
      cs->done = 0;
      cs->all_fixed = 0;
    }
    __syncthreads();
    if (nbrk > 0) {
      double* Mx = red + R_MX;
      // the middle matrix explicitly: column j = bmv(e_j) (wn is free until formk)
      if (col > 0 && wave == 0 && lane < 2 * col) {
        double* e = S.wn + lane * M2;
        for (int i = 0; i < 2 * col; ++i) e[i] = (i == lane) ? 1.0 : 0.0;
        bmv(S.sy, S.wt, col, e, Mx + lane * M2);
      }
      __syncthreads();
      SUBTICK(2);
      const int PW = 3 + 2 * col;
      while (!cs->done) {
        if (!breakpoint_round(col, theta, nbrk, bnded, f2_org, PW, Mx)) return 0;
      }
      if (cs->all_fixed) return 0;
    }
    double dtm = cs->dtm;
    if (dtm <= 0.0) dtm = 0.0;
    const double tsum = cs->tsum + dtm;
    if (own()) z[tid] += tsum * dc[tid];
    if (tid == 0 && col > 0)
      for (int j = 0; j < 2 * col; ++j) S.c[j] += dtm * S.p[j];
    __syncthreads();
    return 0;
  }

  // One round of the breakpoint walk (false: the grid aborted).
  BO_HD bool breakpoint_round(int col, double theta, int nbrk, bool bnded, double f2_org, int PW,
                              const double* Mx) {
    const double inf = __builtin_inf();
    double* tb = V(L_TB);
    double* rec = red + R_REC;
    // (1) this workgroup's KB smallest breakpoints, ascending: KB rounds of a
    // wave argmin per wave, then the four sorted wave lists merged
    {
      const double myv = own() ? tb[tid] : inf;
      const int myi = (own() && myv < inf) ? (int)(base + tid) : n;
      bool taken = false;
      for (int r = 0; r < KB; ++r) {
        double v = taken ? inf : myv;
        int i = taken ? n : myi;
        wave_argmin(v, i);
        if (i < n && i == myi) taken = true;
        if (lane == 0) {
          red[R_HDR + wave * 2 * KB + r] = v;  // (scratch: the headers are read later)
          red[R_HDR + wave * 2 * KB + KB + r] = (double)i;
        }
      }
      const int nfin = __syncthreads_count(own() && myv < inf);
      if (tid == 0) {
        int h[GWV] = {0, 0, 0, 0};
        for (int r = 0; r < KB; ++r) {
          int bw = 0;
          for (int w = 1; w < GWV; ++w) {
            const double* a = red + R_HDR + w * 2 * KB;
            const double* b = red + R_HDR + bw * 2 * KB;
            if (before(a[h[w]], (int)a[KB + h[w]], b[h[bw]], (int)b[KB + h[bw]])) bw = w;
          }
          const double* b = red + R_HDR + bw * 2 * KB;
          rec[1 + r] = b[h[bw]];
          rec[1 + KB + r] = b[KB + h[bw]];
          if (h[bw] < KB - 1) {
            ++h[bw];
          } else {  // this wave's list is spent: park it
            red[R_HDR + bw * 2 * KB + h[bw]] = inf;
            red[R_HDR + bw * 2 * KB + KB + h[bw]] = (double)n;
          }
        }
        rec[0] = nfin > KB ? 1.0 : 0.0;
      }
      __syncthreads();
      // payloads: d_i, bound - x_i, the bound, the ring row (raw WY, WS)
      for (int t = tid; t < KB * PW; t += GT) {
        const int e = t / PW, j = t - e * PW;
        const int gi = (int)rec[1 + KB + e];
        double val = 0.0;
        if (gi < n) {
          const int k = gi - (int)base;
          const double d = V(L_DC)[k];
          const double bnd = d > 0.0 ? hi(k) : lo(k);
          if (j == 0) val = d;
          else if (j == 1) val = bnd - V(L_X)[k];
          else if (j == 2) val = bnd;
          else if (j - 3 < col) val = WY(j - 3)[k];
          else val = WS(j - 3 - col)[k];
        }
        rec[HW + t] = val;
      }
      __syncthreads();
    }
    if (!publish_meet(rec, HW + KB * PW)) return false;
    SUBTICK(3);
    // (2) the headers of all workgroups
    double* hdr = red + R_HDR;
    gather(hdr, 0, HW);
    // (3) wave 0 merges the G sorted lists: the walk order as far as it is
    // known (a workgroup with unpublished breakpoints caps it at its last
    // published one), at most MPAY
    if (wave == 0) {
      const double* hl = hdr + lane * HW;
      const bool live = lane < G;
      // the cap: the smallest last-published entry of a workgroup with more
      double capv = inf;
      int capi = n + 1;
      if (live && hl[0] > 0.0) {
        capv = hl[KB];
        capi = (int)hl[2 * KB];
      }
      wave_argmin(capv, capi);
      int h = 0;
      double kv = live ? hl[1] : inf;
      int ki = live ? (int)hl[1 + KB] : n;
      if (kv == inf) ki = n;
      int M = 0, final_list = 0;
      while (M < MPAY) {
        double bv = kv;
        int bi = ki;
        wave_argmin(bv, bi);
        if (bi >= n) {  // nothing finite left in the published lists
          final_list = capi > n;  // and nothing unpublished
          break;
        }
        if (before(capv, capi, bv, bi)) break;  // past the cap: another round
        if (bi == ki) {  // this lane's head is taken
          ordw[M] = lane;
          ordh[M] = h;
          ++h;
          kv = h < KB ? hl[1 + h] : inf;
          ki = (h < KB && kv < inf) ? (int)hl[1 + KB + h] : n;
        }
        ++M;
      }
      // stage the walked breakpoints' payloads (wave 0 only: the other waves
      // wait at the barrier below)
      {
        const rsrc_t rp = parts();
        for (int t0 = lane; t0 < M * PW; t0 += 4 * 64) {
          double v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int t = t0 + 64 * u;
            const int e = t / PW, j = t - e * PW;
            v[u] = t < M * PW ? ldb(rp, ordw[e] * PK + HW + ordh[e] * PW + j) : 0.0;
          }
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (t0 + 64 * u < M * PW) red[R_PAY + t0 + 64 * u] = v[u];
        }
      }
      // (4) the walk (scipy's cauchy loop body per breakpoint); lane i < 2 col
      // holds p_i and c_i, the breakpoint's products are wave sums
      double f1 = cs->f1, f2 = cs->f2, dtm = cs->dtm, tsum = cs->tsum, tj = cs->tj;
      int nleft = cs->nleft, done = 0, all_fixed = 0;
      const bool li = lane < 2 * col;
      double p = li ? S.p[lane] : 0.0;
      double c = li ? S.c[lane] : 0.0;
      for (int e = 0; e < M; ++e) {
        const double* pay = red + R_PAY + e * PW;
        const double tmin = hdr[ordw[e] * HW + 1 + ordh[e]];
        const int ibp = (int)hdr[ordw[e] * HW + 1 + KB + ordh[e]];
        const double tj0 = tj;
        tj = tmin;
        const double dt = tj - tj0;
        if (dtm < dt) {  // the minimiser lies in this interval
          done = 1;
          break;
        }
        tsum += dt;
        --nleft;
        const double dibp = pay[0], zibp = pay[1];
        if (lane == 0 && ibp >= base && ibp < base + cnt) {  // the owner fixes the variable
          const int k = ibp - (int)base;
          V(L_DC)[k] = 0.0;
          tb[k] = inf;
          V(L_Z)[k] = pay[2];
          iw[k] = dibp > 0.0 ? 2 : 1;
        }
        if (nleft == 0 && nbrk == n) {  // every variable is fixed: z is the GCP
          if (li) c += dt * p;
          done = 1;
          all_fixed = 1;
          break;
        }
        const double dibp2 = dibp * dibp;
        f1 = f1 + dt * f2 + dibp2 - theta * dibp * zibp;
        f2 = f2 - theta * dibp2;
        if (col > 0) {
          double vv = 0.0, wb = 0.0;
          if (li) {
            c += dt * p;
            wb = lane < col ? pay[3 + lane] : theta * pay[3 + lane];
            for (int j = 0; j < 2 * col; ++j) {
              const double wj = j < col ? pay[3 + j] : theta * pay[3 + j];
              vv += Mx[j * M2 + lane] * wj;
            }
          }
          const double wmc = wave_sum(c * vv);
          const double wmp = wave_sum(p * vv);
          const double wmw = wave_sum(wb * vv);
          if (li) p += -dibp * wb;
          f1 = f1 + dibp * wmc;
          f2 = f2 + 2.0 * dibp * wmp - dibp2 * wmw;
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
        done = 1;
        break;
      }
      if (!done && final_list) done = 1;  // no breakpoint left
      // profiling launches (tools/prof_lbfgsb_joint.py): the freev slot, idle
      // on this route, counts the breakpoints walked (x 100 ticks), the store
      // slot the rounds
#ifndef BO_GRID_SUBPROF
      if (prof && lane == 0) {
        prof[2] += 100ull * (unsigned long long)M;
        prof[7] += 100ull;
      }
#endif
      if (li) {
        S.p[lane] = p;
        S.c[lane] = c;
      }
      if (lane == 0) {
        cs->f1 = f1;
        cs->f2 = f2;
        cs->dtm = dtm;
        cs->tsum = tsum;
        cs->tj = tj;
        cs->nleft = nleft;
        cs->done = done;
        cs->all_fixed = all_fixed;
      }
    }
    __syncthreads();
    SUBTICK(4);
    return true;
  }

  // ---- formk over the grid: the Gram products of the 2 col ring vectors over
  // the free set (Y.Y, S_i.Y_j with i <= j) or the active set (S.S, S_i.Y_j
  // with i > j), and the free count; then the LEL^T factorisation in LDS.
  // skip: no free variable (formk / cmprlb / subsm are not run).
  BO_HD int formk(bool& skip) {
    const int col = S.i[I_COL];
    const double theta = S.d[D_THETA];
    const int nv = 2 * col, nb = (nv + 3) / 4, nblk = nb * (nb + 1) / 2;
    const int ntri = nv * (nv + 1) / 2;
    skip = false;
    // 4 x 4 blocks of the lower triangle, 16 lanes per block over the slice
    const int kg = tid & 15, bl = tid >> 4;
    for (int b0 = 0; b0 < nblk; b0 += GT / 16) {
      const int blk = b0 + bl;
      double acc[4][4];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = 0.0;
      int bu = 0, bv = 0;
      if (blk < nblk) {
        int rem = blk;
        while (rem > bu) {
          rem -= bu + 1;
          ++bu;
        }
        bv = rem;
        const double* pu[4];
        const double* pv[4];
        bool ok[4][4], fe[4][4];
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
            fe[a][b] = v < col && (u < col || u - col <= v);
          }
        for (int k = kg; k < cnt; k += 16) {
          const bool fr = is_free(k);
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
              if (ok[a][b] && fe[a][b] == fr) acc[a][b] += xu[a] * xv[b];
        }
      }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          double s = acc[a][b];
          s += __shfl_xor(s, 8);
          s += __shfl_xor(s, 4);
          s += __shfl_xor(s, 2);
          s += __shfl_xor(s, 1);
          acc[a][b] = s;
        }
      if (kg == 0 && blk < nblk)
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const int u = 4 * bu + a, v = 4 * bv + b;
            if (u < nv && v < nv && v <= u) red[1 + u * (u + 1) / 2 + v] = acc[a][b];
          }
    }
    const int nfl = __syncthreads_count(own() && is_free(tid));
    if (tid == 0) red[0] = (double)nfl;
    __syncthreads();
    if (!greduce(1 + ntri)) return 0;
    SUBTICK(5);
    const int nfree = (int)red[0];
    if (tid == 0) S.i[I_NFREE] = nfree;
    if (nfree == 0) {
      __syncthreads();
      skip = true;
      return 0;
    }
    for (int e = tid; e < ntri; e += GT) {  // entry e = (u, v), v <= u
      int u = 0, q = e;
      while (q > u) {
        q -= u + 1;
        ++u;
      }
      const int v = q;
      const double sm = red[1 + e];
      if (u < col) {  // Y_u . Y_v over the free set
        double val = sm / theta;
        if (u == v) val += S.sy[u + u * MMAX];
        S.wn[v + u * M2] = val;
      } else if (v >= col) {  // S_i . S_j over the active set
        S.wn[v + u * M2] = sm * theta;
      } else {  // S_i . Y_j: -L_a (i > j, active) / R_z (i <= j, free)
        S.wn[v + u * M2] = (u - col > v) ? -sm : sm;
      }
    }
    __syncthreads();
    // LEL^T (lbfgsb_core.h formk): the upper-left Cholesky, the col right-hand
    // columns' solves and the lower-right block's products over the threads,
    // then the lower-right Cholesky
    if (wave == 0) {
      const int f = dpofa_w(S.wn, M2, col, lane);
      if (lane == 0) S.k0 = f ? -1 : 0;
    }
    __syncthreads();
    if (S.k0 == 0) {
      for (int js = col + tid; js < 2 * col; js += GT) dtrsl_t(S.wn, M2, col, S.wn + js * M2);
      __syncthreads();
      const int nt = col * (col + 1) / 2;
      for (int e = tid; e < nt; e += GT) {
        int is = 0, q = e;
        while (q >= col - is) {
          q -= col - is;
          ++is;
        }
        const int js = col + is + q;
        is += col;
        double s = 0.0;
        for (int k = 0; k < col; ++k) s += S.wn[k + is * M2] * S.wn[k + js * M2];
        S.wn[is + js * M2] += s;
      }
      __syncthreads();
      if (wave == 0) {
        const int f = dpofa_w(S.wn + col + col * M2, M2, col, lane);
        if (lane == 0 && f) S.k0 = -2;
      }
    }
    __syncthreads();
    return S.k0;
  }

  // ---- cmprlb: rs = -(B (z - x) + g) on the free set ----
  BO_HD int cmprlb(bool unconstrained) {
    const int col = S.i[I_COL];
    const double theta = S.d[D_THETA];
    double* rs = V(L_RS);
    if (unconstrained) {
      if (own()) rs[tid] = -V(L_G)[tid];
      __syncthreads();
      return 0;
    }
    if (wave == 0) {
      const int f = bmv_w(S.sy, S.wt, col, S.c, S.v, lane);
      if (lane == 0) S.k0 = f ? -8 : 0;
    }
    __syncthreads();
    if (S.k0) return S.k0;
    if (own() && is_free(tid)) {
      const int k = tid;
      double acc = -theta * (V(L_Z)[k] - V(L_X)[k]) - V(L_G)[k];
      for (int j = 0; j < col; ++j) acc = acc + WY(j)[k] * S.v[j] + WS(j)[k] * (theta * S.v[col + j]);
      rs[k] = acc;
    }
    __syncthreads();
    return 0;
  }

  // ---- subsm: subspace minimisation over the free set, then the v3.0 projection ----
  BO_HD int subsm() {
    const int col = S.i[I_COL];
    const int nsub = S.i[I_NFREE];
    const double theta = S.d[D_THETA];
    double* rs = V(L_RS);
    double* z = V(L_Z);
    if (nsub <= 0) return 0;
    wg_products(2 * col, 0, [&](int e, const double*& a, const double*& b, int& mode) {
      a = e < col ? WY(e) : WS(e - col);
      b = rs;
      mode = 1;
    });
    if (!greduce(2 * col)) return 0;
    if (wave == 0) {
      if (lane < col) {
        S.wv[lane] = red[lane];
        S.wv[col + lane] = theta * red[col + lane];
      }
      __builtin_amdgcn_wave_barrier();
      int info = dtrsl_t_w(S.wn, M2, 2 * col, S.wv, lane);
      if (!info) {
        if (lane < col) S.wv[lane] = -S.wv[lane];
        __builtin_amdgcn_wave_barrier();
        info = dtrsl_n_w(S.wn, M2, 2 * col, S.wv, lane);
      }
      if (lane == 0) S.k0 = info;
    }
    __syncthreads();
    if (S.k0) return S.k0;
    const double rtheta = 1.0 / theta;
    const bool mine = own() && is_free(tid);
    const int k = tid;
    if (mine) {
      double acc = rs[k];
      for (int jy = 0; jy < col; ++jy)
        acc = acc + WY(jy)[k] * S.wv[jy] / theta + WS(jy)[k] * S.wv[col + jy];
      rs[k] = acc * rtheta;
    }
    if (own()) V(L_XP)[k] = z[k];
    double iword = 0.0;
    if (mine) {  // projected Newton point
      const double dk = rs[k];
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
    {
      double vals[2] = {iword, own() ? (z[k] - V(L_X)[k]) * V(L_G)[k] : 0.0};
      const int ops[2] = {O_MAX, O_SUM};
      wg_reduce(vals, ops, 0);
    }
    if (!greduce(2, 1u)) return 0;
    if (red[0] == 0.0) return 0;
    const double ddp = red[1];
    if (!(ddp > 0.0)) return 0;
    // positive directional derivative of the projection: the backtracking step
    if (own()) z[k] = V(L_XP)[k];
    double cand = __builtin_inf();
    int ibd = n;
    if (mine) {
      const double dk = rs[k];
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
        ibd = (int)(base + k);
      }
    }
    gargmin(cand, ibd);
    if (aborted) return 0;
    const double alpha = fmin(1.0, cand);
    if (alpha < 1.0 && ibd == (int)(base + k) && own()) {
      const double dk = rs[k];
      if (dk > 0.0) {
        z[k] = hi(k);
        rs[k] = 0.0;
      } else if (dk < 0.0) {
        z[k] = lo(k);
        rs[k] = 0.0;
      }
    }
    if (mine) z[k] += alpha * rs[k];
    __syncthreads();
    return 0;
  }

  // ---- label 222: new search direction and the first trial step ----
  BO_HD void direction() {
    double* x = V(L_X);
    double* z = V(L_Z);
    double* dd = V(L_D);
    for (int pass = 0; pass < 4; ++pass) {
      const int col = S.i[I_COL];
      const bool unconstrained = !cnstnd && col > 0;
      if (unconstrained) {  // every variable free (iwhere -1 throughout)
        if (own()) z[tid] = x[tid];
        if (tid == 0) S.i[I_NFREE] = n;
        __syncthreads();
      } else {
        PHTICK(6);
        const int info = cauchy();
        PHTICK(1);
        if (aborted) return;
        if (info) {
          refresh();
          continue;
        }
        PHTICK(2);
      }
      if (S.i[I_COL] != 0) {
        bool skip = false;
        int info = formk(skip);
        PHTICK(3);
        if (aborted) return;
        if (!info && !skip) {
          info = cmprlb(unconstrained);
          PHTICK(4);
          if (!info) info = subsm();
          PHTICK(5);
          if (aborted) return;
        }
        if (info) {
          refresh();
          continue;
        }
      }
      SUBTICK(6);
      // lnsrlb (first entry): |d|^2, the largest feasible step, g.d in one exchange
      const int k = tid;
      double sm = BIG, dtdp = 0.0, gdp = 0.0;
      if (own()) {
        dd[k] = z[k] - x[k];
        const double a1 = dd[k];
        dtdp = a1 * a1;
        gdp = V(L_G)[k] * a1;
        const int nb = nbd(k);
        if (cnstnd && S.i[I_ITER] != 0 && nb != 0) {
          if (a1 < 0.0 && nb <= 2) {
            const double a2 = lo(k) - x[k];
            sm = fmin(sm, a2 >= 0.0 ? 0.0 : a2 / a1);
          } else if (a1 > 0.0 && nb >= 2) {
            const double a2 = hi(k) - x[k];
            sm = fmin(sm, a2 <= 0.0 ? 0.0 : a2 / a1);
          }
        }
      }
      {
        double vals[3] = {dtdp, sm, gdp};
        const int ops[3] = {O_SUM, O_MIN, O_SUM};
        wg_reduce(vals, ops, 0);
      }
      if (!greduce(3, 0u, 1u << 1)) return;
      const double dtd = red[0];
      const double dnorm = sqrt(dtd);
      double stpmx = BIG;
      if (cnstnd) stpmx = S.i[I_ITER] == 0 ? 1.0 : red[1];
      const double stp = (S.i[I_ITER] == 0 && !boxed) ? fmin(1.0 / dnorm, stpmx) : 1.0;
      const double gd = red[2];
      if (own()) {
        V(L_T)[k] = x[k];
        V(L_R)[k] = V(L_G)[k];
      }
      __syncthreads();
      if (tid == 0) {
        S.d[D_FOLD] = S.d[D_F];
        S.d[D_DTD] = dtd;
        S.d[D_STPMX] = stpmx;
        S.d[D_STP] = stp;
        S.d[D_GD] = gd;
        S.d[D_GDOLD] = gd;
        S.i[I_IFUN] = 0;
        S.i[I_IBACK] = 0;
      }
      __syncthreads();
      if (gd >= 0.0) {  // ascent direction: the line search is impossible
        if (restore_or_refresh()) continue;
        return;
      }
      if (tid == 0) S.k0 = dcsrch_start(S.d, S.i, S.d[D_F], gd, stp, 0.0, stpmx);
      __syncthreads();
      if (S.k0) {
        stop(ST_ERROR);
        return;
      }
      if (tid == 0) {
        S.i[I_IFUN] = 1;
        S.i[I_IBACK] = 0;
        S.i[I_PHASE] = PH_LNSRCH;
      }
      __syncthreads();
      write_trial();
      SUBTICK(7);
      return;
    }
    stop(ST_ABNORMAL);  // not reached: a refreshed memory cannot fail again
  }

  // ---- matupd + formt after an accepted step ----
  BO_HD void update() {
    SUBTICK(7);
    double* r = V(L_R);
    double* dd = V(L_D);
    const int k = tid;
    if (own()) r[k] = V(L_G)[k] - r[k];
    const double stp = S.d[D_STP];
    const double gd = S.d[D_GD], gdold = S.d[D_GDOLD];
    double dr, ddum;
    if (stp == 1.0) {
      dr = gd - gdold;
      ddum = -gdold;
    } else {
      dr = (gd - gdold) * stp;
      if (own()) dd[k] *= stp;
      ddum = -gdold * stp;
    }
    __syncthreads();
    if (dr <= EPSMCH * ddum) return;  // skip the L-BFGS update
    if (tid == 0) {
      const int iupdat = ++S.i[I_IUPDAT];
      if (iupdat <= m) {
        S.i[I_COL] = iupdat;
        S.i[I_ITAIL] = (S.i[I_HEAD] + iupdat - 1) % m;
      } else {
        S.i[I_ITAIL] = (S.i[I_ITAIL] + 1) % m;
        S.i[I_HEAD] = (S.i[I_HEAD] + 1) % m;
      }
    }
    __syncthreads();
    const int col = S.i[I_COL];
    const int itail = S.i[I_ITAIL];
    if (own()) {
      wsl[itail * WP + k] = dd[k];
      wyl[itail * WP + k] = r[k];
    }
    new_slot = itail;
    if (tid == 0 && S.i[I_IUPDAT] > m) {  // move old information
      for (int j = 0; j < col - 1; ++j) {
        for (int kk = 0; kk <= j; ++kk) S.ss[kk + j * MMAX] = S.ss[(kk + 1) + (j + 1) * MMAX];
        for (int kk = j; kk < col - 1; ++kk) S.sy[kk + j * MMAX] = S.sy[(kk + 1) + (j + 1) * MMAX];
      }
    }
    __syncthreads();
    // r.r, and the new row of SY / column of SS: WY(j).d, WS(j).d (j < col - 1)
    wg_products(1 + 2 * (col - 1), 0, [&](int e, const double*& a, const double*& b, int& mode) {
      mode = 0;
      if (e == 0) {
        a = r;
        b = r;
      } else if (e < col) {
        a = WY(e - 1);
        b = dd;
      } else {
        a = WS(e - col);
        b = dd;
      }
    });
    if (!greduce(1 + 2 * (col - 1))) return;
    if (wave == 0) {
      const double theta = red[0] / dr;
      if (lane < col - 1) {
        S.sy[(col - 1) + lane * MMAX] = red[1 + lane];
        S.ss[lane + (col - 1) * MMAX] = red[col + lane];
      }
      if (lane == 0) {
        S.d[D_THETA] = theta;
        const double dtd = S.d[D_DTD];
        S.ss[(col - 1) + (col - 1) * MMAX] = (stp == 1.0) ? dtd : stp * stp * dtd;
        S.sy[(col - 1) + (col - 1) * MMAX] = dr;
      }
      __builtin_amdgcn_wave_barrier();
      const int f = formt_w(S.wt, S.sy, S.ss, col, theta, lane);
      if (lane == 0) S.k0 = f;
    }
    __syncthreads();
    SUBTICK(7);
    if (S.k0) refresh();
  }

  // ---- the call: consume f, g at xt; run to the next evaluation ----
  BO_HD void run() {
    if (prof) tprev = wall_clock64();
    for (int k = tid; k < DSLOTS; k += GT) S.d[k] = R.ds[k];
    for (int k = tid; k < ISLOTS; k += GT) S.i[k] = R.is[k];
    for (int k = tid; k < MMAX * MMAX; k += GT) {
      S.sy[k] = R.mat[k];
      S.ss[k] = R.mat[MMAX * MMAX + k];
      S.wt[k] = R.mat[2 * MMAX * MMAX + k];
    }
    const long gi = base + tid;
    const int k = tid;
    double* x = V(L_X);
    double* g = V(L_G);
    if (own()) {
      L[L_LO * SL + k] = P.lower[gi];
      L[L_HI * SL + k] = P.upper[gi];
    }
    __syncthreads();
    const int phase = S.i[I_PHASE];
    if (phase == PH_STOP) {
      if (own()) R.xt[gi] = R.v[(long)V_X * n + gi];
      return;
    }
    if (own()) {
      V(L_T)[k] = R.v[(long)V_T * n + gi];
      V(L_R)[k] = R.v[(long)V_R * n + gi];
      V(L_D)[k] = R.v[(long)V_D * n + gi];
      V(L_Z)[k] = R.v[(long)V_Z * n + gi];
      iw[k] = R.iv[(long)IV_WHERE * n + gi];
      x[k] = R.xt[gi];
      g[k] = R.g_new[gi];
      for (int s = 0; s < m; ++s) {
        wyl[s * WP + k] = R.wy[(long)s * n + gi];
        wsl[s * WP + k] = R.ws[(long)s * n + gi];
      }
    }
    const double fnew = R.f_new;
    // the first exchange: finite f / g, bounds present / all boxed, g.d (the
    // line search's), the projected gradient's norm (the accepted point's)
    double fin = (fnew - fnew == 0.0) ? 1.0 : 0.0, anyb = 0.0, allbox = 1.0, gdp = 0.0, sb = 0.0;
    if (own()) {
      const double gk = g[k];
      if (!(gk - gk == 0.0)) fin = 0.0;
      const int nb = nbd(k);
      anyb = nb != 0 ? 1.0 : 0.0;
      allbox = nb == 2 ? 1.0 : 0.0;
      if (phase == PH_START) iw[k] = nb == 0 ? -1 : ((nb == 2 && hi(k) - lo(k) <= 0.0) ? 3 : 0);
      gdp = gk * V(L_D)[k];
      sb = projg(k);
    }
    {
      double vals[5] = {fin, anyb, allbox, gdp, sb};
      const int ops[5] = {O_MIN, O_MAX, O_MIN, O_SUM, O_MAX};
      wg_reduce(vals, ops, 0);
    }
    if (greduce(5, (1u << 1) | (1u << 4), (1u << 0) | (1u << 2))) {
      const bool finite = red[0] > 0.0;
      cnstnd = red[1] > 0.0;
      boxed = red[2] > 0.0;
      const double gdv = red[3], sbv = red[4];
      PHTICK(0);
      SUBTICK(0);
      if (phase == PH_START) {
        if (tid == 0) {
          for (int j = 0; j < DSLOTS; ++j) S.d[j] = 0.0;
          for (int j = 0; j < ISLOTS; ++j) S.i[j] = 0;
          S.d[D_F] = fnew;
          S.d[D_THETA] = 1.0;
          S.i[I_NFEV] = 1;
        }
        __syncthreads();
        if (!finite) {
          stop(ST_ERROR);
        } else {
          if (tid == 0) S.d[D_SBGNRM] = sbv;
          __syncthreads();
          if (sbv <= P.pgtol)
            stop(ST_CONV_PGTOL);
          else
            direction();
        }
      } else {  // PH_LNSRCH: x <- the trial point
        if (tid == 0) {
          S.d[D_F] = fnew;
          S.i[I_NFEV] += 1;
        }
        __syncthreads();
        if (!finite) {  // a non-finite trial value: keep the last iterate
          if (own()) {
            x[k] = V(L_T)[k];
            g[k] = V(L_R)[k];
          }
          if (tid == 0) S.d[D_F] = S.d[D_FOLD];
          stop(ST_ERROR);
        } else {
          if (tid == 0) {
            double stp = S.d[D_STP];
            S.k0 = dcsrch_cont(S.d, S.i, fnew, gdv, stp, 0.0, S.d[D_STPMX]);
            S.d[D_STP] = stp;
            S.d[D_GD] = gdv;
            if (S.k0 == 0) {
              S.i[I_IFUN] += 1;
              S.i[I_IBACK] = S.i[I_IFUN] - 1;
            }
          }
          __syncthreads();
          if (S.k0 == 0) {  // FG: another trial step
            if (S.i[I_IBACK] >= P.maxls) {
              if (restore_or_refresh()) direction();
            } else {
              write_trial();
            }
          } else {  // NEW_X
            if (tid == 0) {
              S.d[D_SBGNRM] = sbv;
              S.i[I_ITER] += 1;
              S.i[I_NITER] += 1;
            }
            __syncthreads();
            const double fold = S.d[D_FOLD], f = S.d[D_F];
            if (S.i[I_NITER] >= P.maxiter) {
              stop(ST_MAXITER);
            } else if (S.i[I_NFEV] > P.maxfun) {
              stop(ST_MAXFUN);
            } else if (sbv <= P.pgtol) {
              stop(ST_CONV_PGTOL);
            } else if (fold - f <= P.tol * fmax(fmax(fabs(fold), fabs(f)), 1.0)) {
              stop(ST_CONV_FTOL);
            } else {
              update();
              if (!aborted) direction();
            }
          }
        }
      }
    }
    __syncthreads();
    PHTICK(6);
    if (tid == 0) *sflag = (aborted || ld_u32(gm.cnt + 2)) ? 1 : 0;
    __syncthreads();
    if (*sflag) {  // the grid did not meet: keep the iterate, report an error
      if (own()) R.xt[gi] = R.v[(long)V_X * n + gi];
      if (wg == 0 && tid == 0) {
        R.is[I_STATUS] = ST_ERROR;
        R.is[I_PHASE] = PH_STOP;
      }
      return;
    }
    if (own()) {
      if (S.i[I_PHASE] == PH_STOP) R.xt[gi] = x[k];
      R.v[(long)V_X * n + gi] = x[k];
      R.v[(long)V_G * n + gi] = g[k];
      R.v[(long)V_T * n + gi] = V(L_T)[k];
      R.v[(long)V_R * n + gi] = V(L_R)[k];
      R.v[(long)V_D * n + gi] = V(L_D)[k];
      R.v[(long)V_Z * n + gi] = V(L_Z)[k];
      R.iv[(long)IV_WHERE * n + gi] = iw[k];
      if (new_slot >= 0) {
        R.ws[(long)new_slot * n + gi] = wsl[new_slot * WP + k];
        R.wy[(long)new_slot * n + gi] = wyl[new_slot * WP + k];
      }
    }
    if (wg == 0) {
      for (int j = tid; j < DSLOTS; j += GT) R.ds[j] = S.d[j];
      for (int j = tid; j < ISLOTS; j += GT) R.is[j] = S.i[j];
      for (int j = tid; j < MMAX * MMAX; j += GT) {
        R.mat[j] = S.sy[j];
        R.mat[MMAX * MMAX + j] = S.ss[j];
        R.mat[2 * MMAX * MMAX + j] = S.wt[j];
      }
    }
    PHTICK(7);
    SUBTICK(7);
  }
};

__global__ __launch_bounds__(GT) void lbfgsb_grid_kernel(Problem P, double* __restrict__ xt,
                                                         const double* __restrict__ ft,
                                                         const double* __restrict__ gt,
                                                         double* __restrict__ v, int* __restrict__ iv,
                                                         double* __restrict__ ws,
                                                         double* __restrict__ wy,
                                                         double* __restrict__ mat,
                                                         double* __restrict__ ds,
                                                         int* __restrict__ is, GridMem gm) {
  __shared__ Shared S;
  __shared__ double tmp[GWV * 8];
  __shared__ int sflag;
  __shared__ int ordw[MPAY], ordh[MPAY];
  __shared__ CauchyState cs;
  extern __shared__ double lds_dyn[];
  const int G = gridDim.x;
  const int wg = blockIdx.x;
  Restart R{xt, ft[0], gt, v, iv, ws, wy, mat, ds, is};
  GStep st{P, R, S, gm};
  st.n = P.n;
  st.m = P.m;
  st.G = G;
  st.wg = wg;
  st.tid = threadIdx.x;
  st.lane = threadIdx.x & 63;
  st.wave = threadIdx.x >> 6;
  st.base = (long)wg * SL;
  st.cnt = (int)min((long)SL, (long)P.n - st.base);
  st.L = lds_dyn;
  st.wyl = lds_dyn + L_COUNT * SL;
  st.wsl = st.wyl + P.m * WP;
  st.red = st.wsl + P.m * WP;
  st.iw = reinterpret_cast<int*>(st.red + RED);
  st.tmp = tmp;
  st.sflag = &sflag;
  st.ordw = ordw;
  st.ordh = ordh;
  st.cs = &cs;
  st.prof = (P.prof && wg == 0) ? P.prof : nullptr;
  st.run();
  // leave: the last workgroup out resets the counters for the next launch
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(gm.cnt + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (unsigned)G - 1) {
      __hip_atomic_store(gm.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gm.cnt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gm.cnt + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Exchange memory per (device, stream): launches on one stream are ordered,
// so they share it; launches on different streams never do.
struct GridScratch {
  double* part = nullptr;
  unsigned* cnt = nullptr;
};
std::mutex g_grid_mu;
std::map<std::pair<int, void*>, GridScratch> g_grid_scratch;
uint64_t g_grid_attr_set = 0;  // devices whose kernel attribute is set
std::atomic<long long> g_grid_launches{0};

}  // namespace

extern "C" int64_t bo_lbfgsb_grid_launches(void) { return g_grid_launches.load(); }

// Whether the grid kernel takes a single restart of n variables with maxcor m.
bool lbfgsb_grid_fits(int n, int m) {
  if (n < 1 || n > GMAX * SL || m < 1 || m > MMAX) return false;
  return grid_dyn_bytes(m) + sizeof(Shared) + 2048 <= 160 * 1024;
}

int lbfgsb_grid_launch(const bolb::Problem& P, double* xt, const double* ft, const double* gt,
                       double* v, int* iv, double* ws, double* wy, double* mat, double* ds, int* is,
                       void* stream) {
  int dev = 0;
  BO_HIP(hipGetDevice(&dev));
  GridScratch sc;
  {
    std::lock_guard<std::mutex> lock(g_grid_mu);
    const uint64_t bit = dev < 64 ? (uint64_t(1) << dev) : 0;
    if (!bit || !(g_grid_attr_set & bit)) {
      BO_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&lbfgsb_grid_kernel),
                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)(160 * 1024 - sizeof(Shared) - 1024)));
      g_grid_attr_set |= bit;
    }
    GridScratch& s = g_grid_scratch[{dev, stream}];
    if (!s.part) {
      const size_t pb = sizeof(double) * 2 * (size_t)GMAX * PK;
      void* p = nullptr;
      BO_HIP(hipMalloc(&p, pb + 256));
      BO_HIP(hipMemsetAsync(static_cast<char*>(p) + pb, 0, 256, as_stream(stream)));
      s.part = static_cast<double*>(p);
      s.cnt = reinterpret_cast<unsigned*>(static_cast<char*>(p) + pb);
    }
    sc = s;
  }
  const int G = (int)ceil_div(P.n, SL);
  // at least 96 KB of LDS per workgroup: one workgroup per CU
  size_t dyn = grid_dyn_bytes(P.m);
  if (dyn < 96 * 1024) dyn = 96 * 1024;
  GridMem gm{sc.part, sc.cnt};
  lbfgsb_grid_kernel<<<G, GT, dyn, as_stream(stream)>>>(P, xt, ft, gt, v, iv, ws, wy, mat, ds, is, gm);
  BO_LAUNCH_CHECK();
  g_grid_launches.fetch_add(1);
  return BO_OK;
}
