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

}  // namespace

extern "C" int bo_nd_partition_host(const double* Y, int64_t S, int64_t n, int m,
                                    const double* ref, int64_t K_cap, int64_t* K_out,
                                    double* cell_lo, double* cell_hi, int nthreads) {
  if (S < 0 || n < 0 || m < 2 || (!Y && S * n > 0) || !ref || !K_out) {
    bo_set_error("bo_nd_partition_host: bad arguments (S %lld, n %lld, m %d)", (long long)S,
                 (long long)n, m);
    return BO_ERR_ARG;
  }
  std::vector<Cells> cells((size_t)S);
  std::atomic<int64_t> next(0);
  auto work = [&]() {
    for (int64_t s = next++; s < S; s = next++) cells[s] = partition(Y + s * n * m, n, m, ref);
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
    bo_set_error("bo_nd_partition_host: %lld cells needed, capacity %lld", (long long)K,
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
