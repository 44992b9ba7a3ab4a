// Exact non-dominated box decompositions of many point sets on the host
// (native replacement of the per-sample FastNondominatedPartitioning loop of
// qNEHVI, botorch/utils/multi_objective/hypervolume.py:680-700, which the
// reference runs on the CPU for m > 2).
//
// Per point set (maximisation, reference point r):
//   1. Pareto filter: non-dominated, first of duplicates kept, and > r in every
//      objective (box_decompositions/non_dominated.py:353-380, pareto.py:16-64);
//   2. m = 2: the sorted-front staircase (utils.py:222-288);
//      m > 2: Lacour et al. 2017 Alg. 1 twice (utils.py:103-162) -- local upper
//      bounds of -front under -r, then of -U under +inf -- and the cells of
//      Eq. 2 (utils.py:165-195), empty cells dropped;
//   3. every set padded with empty (all-zero) cells to the common maximum, as
//      BoxDecompositionList.get_hypercell_bounds (box_decomposition_list.py:62-94).
// The point sets are independent: they are partitioned on worker threads.
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <limits>
#include <thread>
#include <vector>

#include "../../include/botorch_amd.h"

void bo_set_error(const char* fmt, ...);

namespace {

constexpr double INF = std::numeric_limits<double>::infinity();

struct Cells {
  std::vector<double> lo, hi;  // k x m
  int64_t k = 0;
};

// Pareto-optimal points above the reference (original order kept).
std::vector<double> pareto_above_ref(const double* Y, int64_t n, int m, const double* ref) {
  std::vector<double> out;
  for (int64_t i = 0; i < n; ++i) {
    const double* yi = Y + i * m;
    bool above = true;
    for (int t = 0; t < m; ++t) above = above && (yi[t] > ref[t]);
    if (!above) continue;
    bool keep = true;
    for (int64_t k = 0; k < n && keep; ++k) {
      if (k == i) continue;
      const double* yk = Y + k * m;
      bool ge = true, gt = false, eq = true;
      for (int t = 0; t < m; ++t) {
        ge = ge && (yk[t] >= yi[t]);
        gt = gt || (yk[t] > yi[t]);
        eq = eq && (yk[t] == yi[t]);
      }
      if (ge && gt) keep = false;          // dominated
      else if (eq && k < i) keep = false;  // a duplicate already kept
    }
    if (keep) out.insert(out.end(), yi, yi + m);
  }
  return out;
}

// Lacour17 Alg. 1 (minimisation): update the local upper bounds U (k x m) and
// their defining points Z (k x m x m) with the point z.
void local_upper_bounds(std::vector<double>& U, std::vector<double>& Z, const double* z, int m) {
  const int64_t k = (int64_t)U.size() / m;
  const int64_t mm = (int64_t)m * m;
  std::vector<char> dom(k);
  bool any = false;
  for (int64_t i = 0; i < k; ++i) {
    bool d = true;
    for (int t = 0; t < m; ++t) d = d && (U[i * m + t] > z[t]);
    dom[i] = d;
    any = any || d;
  }
  if (!any) return;
  std::vector<double> nU, nZ;
  nU.reserve(U.size());
  nZ.reserve(Z.size());
  for (int64_t i = 0; i < k; ++i) {
    if (dom[i]) continue;
    nU.insert(nU.end(), U.begin() + i * m, U.begin() + (i + 1) * m);
    nZ.insert(nZ.end(), Z.begin() + i * mm, Z.begin() + (i + 1) * mm);
  }
  for (int j = 0; j < m; ++j) {
    for (int64_t i = 0; i < k; ++i) {
      if (!dom[i]) continue;
      const double* Zi = &Z[i * mm];  // Zi[a * m + b]: defining point a, coordinate b
      double zmax = -INF;
      for (int a = 0; a < m; ++a)
        if (a != j) zmax = std::max(zmax, Zi[a * m + j]);
      if (!(z[j] >= zmax)) continue;
      for (int t = 0; t < m; ++t) nU.push_back(t == j ? z[j] : U[i * m + t]);
      for (int a = 0; a < m; ++a)
        for (int b = 0; b < m; ++b) nZ.push_back(a == j ? z[b] : Zi[a * m + b]);
    }
  }
  U.swap(nU);
  Z.swap(nZ);
}

Cells partition(const double* Y, int64_t n, int m, const double* ref) {
  Cells c;
  std::vector<double> P = pareto_above_ref(Y, n, m, ref);
  const int64_t np = (int64_t)P.size() / m;
  if (np == 0) {  // a single cell [ref, inf)
    c.k = 1;
    c.lo.assign(ref, ref + m);
    c.hi.assign(m, INF);
    return c;
  }
  if (m == 2) {
    std::vector<int64_t> idx(np);
    for (int64_t i = 0; i < np; ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(),
                     [&](int64_t a, int64_t b) { return P[a * 2] < P[b * 2]; });
    // front = [(ref0, p0_1), p_0 .. p_{np-1}, (p_last_0, ref1)]
    std::vector<double> f;
    f.push_back(ref[0]);
    f.push_back(P[idx[0] * 2 + 1]);
    for (int64_t i = 0; i < np; ++i) {
      f.push_back(P[idx[i] * 2]);
      f.push_back(P[idx[i] * 2 + 1]);
    }
    f.push_back(P[idx[np - 1] * 2]);
    f.push_back(ref[1]);
    const int64_t nf = (int64_t)f.size() / 2;
    c.k = nf - 1;
    for (int64_t i = 0; i + 1 < nf; ++i) {
      c.lo.push_back(f[i * 2]);
      c.lo.push_back(f[(i + 1) * 2 + 1]);
      c.hi.push_back(i + 1 < nf - 1 ? f[(i + 1) * 2] : INF);
      c.hi.push_back(INF);
    }
    return c;
  }
  // first pass: -front under -ref (minimisation)
  std::vector<double> U(m), Z((size_t)m * m, -INF);
  for (int t = 0; t < m; ++t) U[t] = -ref[t];
  for (int j = 0; j < m; ++j) Z[j * m + j] = U[j];
  std::vector<double> z(m);
  for (int64_t i = 0; i < np; ++i) {
    for (int t = 0; t < m; ++t) z[t] = -P[i * m + t];
    local_upper_bounds(U, Z, z.data(), m);
  }
  // second pass: -U as a new front for minimisation with reference +inf
  std::vector<double> U2(m, INF), Z2((size_t)m * m);
  for (int a = 0; a < m; ++a)
    for (int b = 0; b < m; ++b) Z2[a * m + b] = (a == b) ? INF : ref[b];
  const int64_t k1 = (int64_t)U.size() / m;
  for (int64_t i = 0; i < k1; ++i) {
    for (int t = 0; t < m; ++t) z[t] = -U[i * m + t];
    local_upper_bounds(U2, Z2, z.data(), m);
  }
  // Eq. 2 cells (reference point +inf), empty ones dropped
  const int64_t k2 = (int64_t)U2.size() / m;
  const int64_t mm = (int64_t)m * m;
  std::vector<double> lo(m), hi(m);
  for (int64_t i = 0; i < k2; ++i) {
    const double* Zi = &Z2[i * mm];
    lo[0] = Zi[0];
    hi[0] = INF;
    for (int j = 1; j < m; ++j) {
      double mx = -INF;
      for (int a = 0; a < j; ++a) mx = std::max(mx, Zi[a * m + j]);
      lo[j] = mx;
      hi[j] = U2[i * m + j];
    }
    bool empty = false;
    for (int t = 0; t < m; ++t) empty = empty || (hi[t] <= lo[t]);
    if (empty) continue;
    c.lo.insert(c.lo.end(), lo.begin(), lo.end());
    c.hi.insert(c.hi.end(), hi.begin(), hi.end());
    ++c.k;
  }
  return c;
}

// NondominatedPartitioning's binary partitioning (box_decompositions/
// non_dominated.py:81-192, Couckuyt et al. 2012), the decomposition qNEHVI uses
// with alpha > 0 for m > 2 (utils/multi_objective/hypervolume.py:606-612).
// Under minimisation of -Y: cells are pairs of index vectors into the Pareto
// points sorted per outcome, augmented with an ideal row 0 and an anti-ideal
// row np + 1.  A cell popped from the stack whose upper corner no Pareto point
// dominates is kept; one whose lower corner no point dominates straddles the
// front and is halved along its longest index range -- unless every range is
// down to adjacent indices or its volume is at most alpha of the whole box,
// in which case it is dropped (the approximation); any other cell is dominated.
Cells binary_partition(const double* Y, int64_t n, int m, const double* ref, double alpha) {
  Cells c;
  std::vector<double> P = pareto_above_ref(Y, n, m, ref);
  const int64_t np = (int64_t)P.size() / m;
  if (np == 0) {
    c.k = 1;
    c.lo.assign(ref, ref + m);
    c.hi.assign(m, INF);
    return c;
  }
  // the minimisation front -P, ordered by its first outcome (sort=True)
  std::vector<int64_t> ord(np);
  for (int64_t i = 0; i < np; ++i) ord[i] = i;
  std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return -P[a * m] < -P[b * m]; });
  std::vector<double> N((size_t)np * m);
  for (int64_t i = 0; i < np; ++i)
    for (int t = 0; t < m; ++t) N[i * m + t] = -P[ord[i] * m + t];
  // aug_idx[r][t]: row r of the per-outcome order (0: ideal, 1..np: points, np+1: anti-ideal)
  std::vector<int64_t> aug_idx((size_t)(np + 2) * m);
  for (int t = 0; t < m; ++t) {
    std::vector<int64_t> o(np);
    for (int64_t i = 0; i < np; ++i) o[i] = i;
    std::stable_sort(o.begin(), o.end(), [&](int64_t a, int64_t b) { return N[a * m + t] < N[b * m + t]; });
    aug_idx[t] = 0;
    for (int64_t i = 0; i < np; ++i) aug_idx[(i + 1) * m + t] = o[i] + 1;
    aug_idx[(np + 1) * m + t] = np + 1;
  }
  // aug values for the tests: ideal - 1, the points, anti-ideal + 1
  std::vector<double> aug((size_t)(np + 2) * m);
  for (int t = 0; t < m; ++t) {
    double lo = INF, hi = -INF;
    for (int64_t i = 0; i < np; ++i) {
      lo = std::min(lo, N[i * m + t]);
      hi = std::max(hi, N[i * m + t]);
    }
    aug[t] = lo - 1.0;
    for (int64_t i = 0; i < np; ++i) aug[(i + 1) * m + t] = N[i * m + t];
    aug[(np + 1) * m + t] = hi + 1.0;
  }
  double total = 1.0;
  for (int t = 0; t < m; ++t) total *= aug[(np + 1) * m + t] - aug[t];
  // final bounds (maximisation): lower from the cell's upper index, upper from
  // its lower index; row 0 -> +inf, row np + 1 -> ref, point rows -> P
  auto bound = [&](int64_t row, int t, bool upper) {
    if (row == 0) return INF;
    if (row == np + 1) return ref[t];
    (void)upper;
    return -N[(row - 1) * m + t];
  };
  std::vector<int64_t> stack;  // cells: 2 m index entries each (lower row, upper row per outcome)
  stack.reserve(64 * m);
  for (int t = 0; t < m; ++t) stack.push_back(0);
  for (int t = 0; t < m; ++t) stack.push_back(np + 1);
  std::vector<int64_t> cell(2 * m), bidx(2 * m);
  std::vector<double> bval(2 * m);
  while (!stack.empty()) {
    std::copy(stack.end() - 2 * m, stack.end(), cell.begin());
    stack.resize(stack.size() - 2 * m);
    for (int b = 0; b < 2; ++b)
      for (int t = 0; t < m; ++t) {
        bidx[b * m + t] = aug_idx[cell[b * m + t] * m + t];
        bval[b * m + t] = aug[bidx[b * m + t] * m + t];
      }
    // for every point some outcome where the corner is no worse
    auto corner_free = [&](int b) {
      for (int64_t i = 0; i < np; ++i) {
        bool any = false;
        for (int t = 0; t < m && !any; ++t) any = bval[b * m + t] <= N[i * m + t];
        if (!any) return false;
      }
      return true;
    };
    if (corner_free(1)) {
      for (int t = 0; t < m; ++t) c.lo.push_back(bound(bidx[m + t], t, false));
      for (int t = 0; t < m; ++t) c.hi.push_back(bound(bidx[t], t, true));
      ++c.k;
    } else if (corner_free(0)) {
      bool not_adjacent = false;
      int64_t length = -1;
      int longest = 0;
      double vol = 1.0;
      for (int t = 0; t < m; ++t) {
        const int64_t dist = cell[m + t] - cell[t];
        not_adjacent = not_adjacent || dist > 1;
        if (dist > length) {  // first maximum, as torch.max
          length = dist;
          longest = t;
        }
        vol *= bval[m + t] - bval[t];
      }
      if (not_adjacent && vol / total > alpha) {
        const int64_t h1 = (int64_t)std::nearbyint((double)length / 2.0);  // round half to even
        const int64_t h2 = length - h1;
        std::vector<int64_t> a(cell), b(cell);
        a[m + longest] -= h1;  // the upper half's bound
        b[longest] += h2;      // the lower half's bound
        stack.insert(stack.end(), a.begin(), a.end());
        stack.insert(stack.end(), b.begin(), b.end());
      }
    }
  }
  return c;
}

template <class F>
int partition_all(const double* Y, int64_t S, int64_t n, int m, int64_t K_cap, int64_t* K_out,
                  double* cell_lo, double* cell_hi, int nthreads, F&& one) {
  std::vector<Cells> cells((size_t)S);
  std::atomic<int64_t> next(0);
  auto work = [&]() {
    for (int64_t s = next++; s < S; s = next++) cells[s] = one(Y + s * n * m);
  };
  const int nt = std::max(1, std::min<int>(nthreads, (int)std::max<int64_t>(S, 1)));
  std::vector<std::thread> pool;
  for (int i = 1; i < nt; ++i) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  int64_t K = 0;
  for (const auto& c : cells) K = std::max(K, c.k);
  *K_out = K;
  if (!cell_lo || !cell_hi) return BO_OK;  // size query
  if (K > K_cap) {
    bo_set_error("box decomposition: %lld cells needed, capacity %lld", (long long)K,
                 (long long)K_cap);
    return BO_ERR_ARG;
  }
  for (int64_t s = 0; s < S; ++s) {
    double* lo = cell_lo + s * K_cap * m;
    double* hi = cell_hi + s * K_cap * m;
    std::fill(lo, lo + K_cap * m, 0.0);
    std::fill(hi, hi + K_cap * m, 0.0);
    std::copy(cells[s].lo.begin(), cells[s].lo.end(), lo);
    std::copy(cells[s].hi.begin(), cells[s].hi.end(), hi);
  }
  return BO_OK;
}

}  // namespace

extern "C" int bo_nd_partition_alpha_host(const double* Y, int64_t S, int64_t n, int m,
                                          const double* ref, double alpha, int64_t K_cap,
                                          int64_t* K_out, double* cell_lo, double* cell_hi,
                                          int nthreads) {
  if (S < 0 || n < 0 || m < 2 || (!Y && S * n > 0) || !ref || !K_out || !(alpha >= 0.0)) {
    bo_set_error("bo_nd_partition_alpha_host: bad arguments (S %lld, n %lld, m %d, alpha %g)",
                 (long long)S, (long long)n, m, alpha);
    return BO_ERR_ARG;
  }
  return partition_all(Y, S, n, m, K_cap, K_out, cell_lo, cell_hi, nthreads,
                       [&](const double* Ys) { return binary_partition(Ys, n, m, ref, alpha); });
}

extern "C" int bo_nd_partition_host(const double* Y, int64_t S, int64_t n, int m,
                                    const double* ref, int64_t K_cap, int64_t* K_out,
                                    double* cell_lo, double* cell_hi, int nthreads) {
  if (S < 0 || n < 0 || m < 2 || (!Y && S * n > 0) || !ref || !K_out) {
    bo_set_error("bo_nd_partition_host: bad arguments (S %lld, n %lld, m %d)", (long long)S,
                 (long long)n, m);
    return BO_ERR_ARG;
  }
  return partition_all(Y, S, n, m, K_cap, K_out, cell_lo, cell_hi, nthreads,
                       [&](const double* Ys) { return partition(Ys, n, m, ref); });
}
