// Blocked Cholesky + triangular inverse of one n x n SPD matrix as ONE
// persistent launch over a task DAG of 64 x 64 tiles (gfx950).
//
// Replaces, for the GP caches and the MLL closure (botorch/models/gpytorch.py:446
// -> [G] DefaultPredictionStrategy; optim/closures/model_closures.py:171-184):
//   L = cholesky(A) and X = L^{-1}  ([G] root_inv_decomposition's L^{-T},
//   botorch/__init__.py:44).
//
// Why one launch: the factorisation is a chain of n/64 diagonal-tile steps.
// Launched step by step (chol.hip's look-ahead path) every step pays kernel
// launch gaps and cross-stream event waits on the critical path, and the
// diagonal factor runs while most CUs idle.  Here every workgroup (one per CU)
// pulls tasks from one queue in a fixed order in which every dependency of a
// task precedes it; a task waits (bounded spin) on per-tile counters.  A task
// is only ever claimed by a running workgroup, and every task it waits on was
// claimed earlier, so the queue cannot deadlock (no co-residency assumption).
//
// Tasks (T = np / 64 tile rows; tile (i, j), i >= j; A holds the lower
// triangle and is overwritten by L; Linv receives X):
//   CRIT(k)            L_{k,k-1} = A_{k,k-1} D_{k-1}^T,  A_kk -= L_{k,k-1} L_{k,k-1}^T,
//                      then L_kk = chol(A_kk) and D_k = L_kk^{-1} (one workgroup, LDS)
//   TRSM(k, rows)      L_ik = A_ik D_k^T                 (i >= k + 2)
//   COLUPD(j, k, rows) A_ij -= L_ik L_jk^T               (step k update of column j)
//   XSTEP(j, k, rows)  X_kj = -D_k acc_kj (k > j; X_jj = D_j), then
//                      acc_ij += L_ik X_kj for the rows i > k  (right-looking trtri)
//   AINV(kb, j, rows)  (optional, round 5: A^{-1} = X^T X for the MLL gradient)
//                      Ainv_ij += sum_{K in [kb, kb + 3), K >= i} X_Ki^T X_Kj, i >= j,
//                      in increasing K per tile (version flags), as soon as the
//                      X rows K are final -- in the idle CUs of the chain-bound tail
// Task order (host-built table): CRIT(0), CRIT(1), then per step k: TRSM(k,.),
// the two COLUPD chunks CRIT(k+2) needs, CRIT(k+2), XSTEP(., k), the other
// COLUPD chunks; finally the X_{T-1,j} finalisations.
//
// Cross-workgroup hand-off (MI355X_MICROARCH.md, inter-workgroup visibility; the
// per-XCD L2s are not coherent): every tile byte another workgroup reads is
// stored write-through (sc1 buffer stores), every storing wave drains
// (s_waitcnt vmcnt(0)), a workgroup barrier, then ONE lane publishes the tile's
// counter with an agent-scope atomic store; consumers poll that word with an
// agent-scope (sc1) load and read the tiles with sc1 loads only (L1 bypassed),
// one workgroup per CU.
#include <algorithm>
#include <cmath>
#include <map>
#include <utility>
#include <mutex>
#include <vector>

#include "common.h"

#include <cstdlib>

namespace {

constexpr int TB = 64;  // tile
constexpr int LP = 68;  // LDS pitch in doubles (rows 16-B aligned)
constexpr int CH = 8;   // tile rows per chunked task of a multi-matrix launch (one matrix: 2)
constexpr int NFLAG0 = 16;  // head counter, abort word, padding
constexpr int GB = 3;       // steps per batched column update (LDS: X0 + GB operand tiles)
constexpr int CHB = 8;      // tile rows per batched task of a multi-matrix launch (one matrix: 4, build_tasks)
constexpr long long SPIN_TIMEOUT = 200000000;  // wall-clock ticks (100 MHz): 2 s

enum : int { T_CRIT = 0, T_TRSM = 1, T_COLUPD = 2, T_XSTEP = 3, T_AINV = 4 };
constexpr int GA = 3;  // steps K per A^{-1} task (LDS: X0 + GA operand tiles)

typedef unsigned int u32;
typedef u32 v2u __attribute__((ext_vector_type(2)));
typedef u32 v4u __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
// the diagonal block's column counter: an explicit LDS pointer, so polls and
// updates are ds_read / ds_write (a generic volatile pointer becomes a flat
// access with a full vmcnt drain per column)
typedef volatile __attribute__((address_space(3))) int lds_cnt_t;

constexpr int SC1 = 16;  // cache-policy bit: write-through store / L1-bypassing load

__device__ __forceinline__ rsrc_t make_rsrc(const double* p, u32 bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ double2 ld16(rsrc_t r, u32 off) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, SC1));
}
__device__ __forceinline__ void st16(rsrc_t r, u32 off, double2 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), r, off, 0, SC1);
}
__device__ __forceinline__ double ld8(rsrc_t r, u32 off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, SC1));
}
__device__ __forceinline__ void st8(rsrc_t r, u32 off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, v), r, off, 0, SC1);
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double rsq_nr(double v) {
  double r = __builtin_amdgcn_rsq(v);
  r = r * fma(-0.5 * v * r, r, 1.5);
  r = r * fma(-0.5 * v * r, r, 1.5);
  return r;
}

struct Ctx {
  rsrc_t rA, rI;
  int np;
  int tid, lane, wave, wm, wn;
};

// byte offset of element (r, c) of tile (ti, tj)
__device__ __forceinline__ u32 toff(const Ctx& c, int ti, int tj, int r, int col) {
  return (u32)((((u32)(ti * TB + r)) * (u32)c.np + (u32)(tj * TB + col)) * 8u);
}

// 64 x 64 tile -> LDS (pitch LP), 16-B sc1 loads, 8 per thread in flight.
__device__ __forceinline__ void tile_to_lds(const Ctx& c, rsrc_t r, int ti, int tj, double* S) {
  double2 v[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int e = c.tid + 256 * p;
    v[p] = ld16(r, toff(c, ti, tj, e >> 5, (e & 31) * 2));
  }
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int e = c.tid + 256 * p;
    *reinterpret_cast<double2*>(S + (e >> 5) * LP + (e & 31) * 2) = v[p];
  }
}

__device__ __forceinline__ void lds_to_tile(const Ctx& c, const double* S, rsrc_t r, int ti, int tj) {
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int e = c.tid + 256 * p;
    st16(r, toff(c, ti, tj, e >> 5, (e & 31) * 2),
         *reinterpret_cast<const double2*>(S + (e >> 5) * LP + (e & 31) * 2));
  }
}

// Accumulator: each wave owns a 32 x 32 quadrant (2 x 2 MFMA tiles).
struct Acc {
  v4d t[2][2];
};

__device__ __forceinline__ void acc_zero(Acc& a) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) a.t[i][j] = v4d_zero();
}

__device__ __forceinline__ void acc_load(const Ctx& c, Acc& a, rsrc_t r, int ti, int tj) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        a.t[i][j][q] = ld8(r, toff(c, ti, tj, c.wm + 16 * i + mfma_row(c.lane, q),
                                   c.wn + 16 * j + mfma_col(c.lane)));
}

// (8-B accesses in the MFMA layout: 16-B ones after a lane-pair exchange
// measured slower, 2.38 -> 2.47 ms at n = 4096)
__device__ __forceinline__ void acc_store(const Ctx& c, const Acc& a, rsrc_t r, int ti, int tj) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        st8(r, toff(c, ti, tj, c.wm + 16 * i + mfma_row(c.lane, q), c.wn + 16 * j + mfma_col(c.lane)),
            a.t[i][j][q]);
}

__device__ __forceinline__ void acc_to_lds(const Ctx& c, const Acc& a, double* S) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        S[(c.wm + 16 * i + mfma_row(c.lane, q)) * LP + c.wn + 16 * j + mfma_col(c.lane)] = a.t[i][j][q];
}

// acc += sgn * SA * op(SB), 64-deep; BT: op(SB) = SB^T, else SB.
template <bool BT>
__device__ __forceinline__ void acc_mma(const Ctx& c, Acc& a, const double* SA, const double* SB,
                                        double sgn) {
  const int r16 = c.lane & 15, kq = c.lane >> 4;
#pragma unroll 4
  for (int ks = 0; ks < 16; ++ks) {
    const int k = 4 * ks + kq;
    const double a0 = sgn * SA[(c.wm + r16) * LP + k];
    const double a1 = sgn * SA[(c.wm + 16 + r16) * LP + k];
    double b0, b1;
    if (BT) {
      b0 = SB[(c.wn + r16) * LP + k];
      b1 = SB[(c.wn + 16 + r16) * LP + k];
    } else {
      b0 = SB[k * LP + c.wn + r16];
      b1 = SB[k * LP + c.wn + 16 + r16];
    }
    a.t[0][0] = mfma_f64(a0, b0, a.t[0][0]);
    a.t[0][1] = mfma_f64(a0, b1, a.t[0][1]);
    a.t[1][0] = mfma_f64(a1, b0, a.t[1][0]);
    a.t[1][1] = mfma_f64(a1, b1, a.t[1][1]);
  }
}

// acc += sgn * SA * SB^T, 64-deep, operands read 16 B at a time: lane group kq
// takes k = 8 s + 2 kq (first MFMA) and 8 s + 2 kq + 1 (second) -- the same k
// permutation on both operands, so the sum is the same set of products.
__device__ __forceinline__ void acc_mma_nt(const Ctx& c, Acc& a, const double* SA, const double* SB,
                                           double sgn) {
  const int r16 = c.lane & 15, kq = c.lane >> 4;
  const double* pa0 = SA + (c.wm + r16) * LP + 2 * kq;
  const double* pa1 = pa0 + 16 * LP;
  const double* pb0 = SB + (c.wn + r16) * LP + 2 * kq;
  const double* pb1 = pb0 + 16 * LP;
  double2 a0 = *reinterpret_cast<const double2*>(pa0), a1 = *reinterpret_cast<const double2*>(pa1);
  double2 b0 = *reinterpret_cast<const double2*>(pb0), b1 = *reinterpret_cast<const double2*>(pb1);
#pragma unroll
  for (int st = 0; st < 8; ++st) {
    double2 na0, na1, nb0, nb1;
    if (st < 7) {  // next k-pair in flight under this pair's MFMAs
      na0 = *reinterpret_cast<const double2*>(pa0 + 8 * (st + 1));
      na1 = *reinterpret_cast<const double2*>(pa1 + 8 * (st + 1));
      nb0 = *reinterpret_cast<const double2*>(pb0 + 8 * (st + 1));
      nb1 = *reinterpret_cast<const double2*>(pb1 + 8 * (st + 1));
    }
    a.t[0][0] = mfma_f64(sgn * a0.x, b0.x, a.t[0][0]);
    a.t[0][1] = mfma_f64(sgn * a0.x, b1.x, a.t[0][1]);
    a.t[1][0] = mfma_f64(sgn * a1.x, b0.x, a.t[1][0]);
    a.t[1][1] = mfma_f64(sgn * a1.x, b1.x, a.t[1][1]);
    a.t[0][0] = mfma_f64(sgn * a0.y, b0.y, a.t[0][0]);
    a.t[0][1] = mfma_f64(sgn * a0.y, b1.y, a.t[0][1]);
    a.t[1][0] = mfma_f64(sgn * a1.y, b0.y, a.t[1][0]);
    a.t[1][1] = mfma_f64(sgn * a1.y, b1.y, a.t[1][1]);
    if (st < 7) { a0 = na0; a1 = na1; b0 = nb0; b1 = nb1; }
  }
}

// 64 x 64 tile -> LDS transposed (S[col][row]): the B operand of acc += L X
// read in the 16-B pattern of acc_mma_nt.
__device__ __forceinline__ void tile_to_lds_t(const Ctx& c, rsrc_t r, int ti, int tj, double* S) {
  double2 v[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int e = c.tid + 256 * p;
    v[p] = ld16(r, toff(c, ti, tj, e >> 5, (e & 31) * 2));
  }
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int e = c.tid + 256 * p;
    const int row = e >> 5, col = (e & 31) * 2;
    S[col * LP + row] = v[p].x;
    S[(col + 1) * LP + row] = v[p].y;
  }
}

__device__ __forceinline__ void acc_to_lds_t(const Ctx& c, const Acc& a, double* S) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        S[(c.wn + 16 * j + mfma_col(c.lane)) * LP + c.wm + 16 * i + mfma_row(c.lane, q)] = a.t[i][j][q];
}

// ---- hand-off ---------------------------------------------------------------
__device__ __forceinline__ u32 flag_load(const u32* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Every storing wave drains its sc1 stores, the workgroup meets, one lane
// publishes the counter value.
__device__ __forceinline__ void publish(const Ctx& c, u32* f, u32 val) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (c.tid == 0) __hip_atomic_store(f, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The same, but waiting only for the stores issued BEFORE the wave's `younger`
// most recent vector-memory instructions (loads, stores and atomics count
// together, in issue order): the prefetch loads issued after a tile's stores
// stay in flight.  `younger` must not exceed the instructions really issued
// after those stores (fewer is safe, only slower); wave-uniform.
__device__ __forceinline__ void publish_after(const Ctx& c, u32* f, u32 val, int younger) {
  younger = __builtin_amdgcn_readfirstlane(younger);  // (uniform: scalar branches)
  if (younger >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if (younger >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (younger >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (c.tid == 0) __hip_atomic_store(f, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Thread 0 polls until f1 >= t1 and f2 >= t2 (bounded: timeout -> abort word);
// the workgroup then proceeds together.  Returns false when aborted.
__device__ __forceinline__ bool wait2(const Ctx& c, const u32* f1, u32 t1, const u32* f2, u32 t2,
                                      u32* abortw, int* s_ok, long long* wacc = nullptr) {
  if (c.tid == 0) {
    int ok = 1;
    if (flag_load(f1) < t1 || flag_load(f2) < t2) {
      const long long t0 = wall_clock64();
      for (;;) {
        __builtin_amdgcn_s_sleep(1);
        if (flag_load(f1) >= t1 && flag_load(f2) >= t2) break;
        if (flag_load(abortw)) { ok = 0; break; }
        if (wall_clock64() - t0 > SPIN_TIMEOUT) {
          __hip_atomic_store(abortw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
      }
      if (wacc) *wacc += wall_clock64() - t0;
    }
    *s_ok = ok;
  }
  __syncthreads();
  const int ok = *s_ok;
  __syncthreads();
  return ok != 0;
}

// ---- the diagonal tile ------------------------------------------------------------
// (row_bcast<K>: lane K of each 16-lane row to the whole row, common.h)

#ifdef BO_TOOLS  // the round-2 four-panel diagonal tile: timing reference of tools/probe_potrf64.py
template <int JJ, int M>
__device__ __forceinline__ void col_update(double (&v)[16], double l) {
  if constexpr (M > JJ) v[M] = fma(-l, row_bcast<M>(l), v[M]);
}
template <int JJ, int... M>
__device__ __forceinline__ void col_updates(std::integer_sequence<int, M...>, double (&v)[16], double l) {
  (col_update<JJ, M>(v, l), ...);
}

template <int JJ, int M>
__device__ __forceinline__ void col_update_lds(double (&v)[16], double l, const double* Lj) {
  if constexpr (M > JJ + 1) v[M] = fma(-l, Lj[M], v[M]);
}
template <int JJ, int... M>
__device__ __forceinline__ void col_updates_lds(std::integer_sequence<int, M...>, double (&v)[16],
                                                double l, const double* Lj) {
  (col_update_lds<JJ, M>(v, l, Lj), ...);
}

// Column JJ of the 16 x 16 diagonal-block factorisation (wave 0; lane = (group
// g, row r), every group holds the whole block): pivot broadcast inside the
// 16-lane row (DPP).  Group 0 publishes the column L[., JJ] and 1 / L_JJ,JJ to
// LDS, then the column counter, for the inverse built concurrently on wave 1
// (diag_inv_step).  The next pivot's column takes its factor through DPP (the
// chain); the other columns read L[M, JJ] back from that LDS copy -- one
// uniform-address read per value instead of two DPP moves: the step is bound
// by the wave's instruction issue, not by the chain.
template <int JJ>
__device__ __forceinline__ void diag_step(double (&v)[16], int r, int g, bool lane0, int& fail,
                                          double* rinv, double* Lc, lds_cnt_t* cnt, int cbase) {
  const double piv = row_bcast<JJ>(v[JJ]);
  if (!(piv > 0.0) && fail == 0) fail = JJ + 1;
  const double rr = rsq_nr(piv);
  const double l = (r >= JJ) ? v[JJ] * rr : 0.0;  // L_{r,JJ} (r == JJ: sqrt(piv))
  v[JJ] = l;
  if (g == 0) Lc[JJ * 16 + r] = l;
  if (lane0) {
    rinv[JJ] = rr;
    *cnt = cbase + JJ + 1;  // LDS writes of one wave land in order
  }
  if constexpr (JJ + 1 < 16) v[JJ + 1] = fma(-l, row_bcast<JJ + 1>(l), v[JJ + 1]);
  col_updates_lds<JJ>(std::make_integer_sequence<int, 16>{}, v, l, Lc + JJ * 16);
}

template <int... JJ>
__device__ __forceinline__ void diag_steps(std::integer_sequence<int, JJ...>, double (&v)[16],
                                           int r, int g, bool lane0, int& fail, double* rinv,
                                           double* Lc, lds_cnt_t* cnt, int cbase) {
  (diag_step<JJ>(v, r, g, lane0, fail, rinv, Lc, cnt, cbase), ...);
}

// Column JJ of the inverse of the diagonal block (wave 1, one column behind wave
// 0): group g owns inverse columns 4 g .. 4 g + 3; row JJ is scaled by 1 / L_JJ,JJ
// and eliminated from the rows below (forward substitution).
template <int JJ>
__device__ __forceinline__ void diag_inv_step(double (&x)[4], int r, const double* rinv,
                                              const double* Lc, lds_cnt_t* cnt, int cbase) {
  while (*cnt < cbase + JJ + 1) __builtin_amdgcn_s_sleep(0);
  const double rr = rinv[JJ];
  const double l = Lc[JJ * 16 + r];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const double xs = (r == JJ) ? x[q] * rr : x[q];
    const double sv = row_bcast<JJ>(xs);
    x[q] = (r > JJ) ? fma(-l, sv, xs) : xs;
  }
}

template <int... JJ>
__device__ __forceinline__ void diag_inv_steps(std::integer_sequence<int, JJ...>, double (&x)[4],
                                               int r, const double* rinv, const double* Lc,
                                               lds_cnt_t* cnt, int cbase) {
  (diag_inv_step<JJ>(x, r, rinv, Lc, cnt, cbase), ...);
}

// ---- timing probe of the 16 x 16 diagonal step (tools/probe_diag16.py) ----------
// Variant 1 broadcasts the L column through v_readlane (every lane group holds
// the same block, so lane M of any group has the pivot column's row M) and
// uses the SGPR in the FMA; variant 0 is diag_steps (DPP row broadcast);
// variant 2 is variant 0 without the inverse.
template <int JJ, int M>
__device__ __forceinline__ void col_update_s(double (&v)[16], double l) {
  if constexpr (M > JJ) v[M] = fma(-l, readlane_d(l, M), v[M]);
}
template <int JJ, int... M>
__device__ __forceinline__ void col_updates_s(std::integer_sequence<int, M...>, double (&v)[16], double l) {
  (col_update_s<JJ, M>(v, l), ...);
}
template <int JJ, int VAR>
__device__ __forceinline__ void diag_step_probe(double (&v)[16], double (&x)[4], int r) {
  const double piv = VAR == 1 ? readlane_d(v[JJ], JJ) : row_bcast<JJ>(v[JJ]);
  const double rr = rsq_nr(piv);
  const double l = (r >= JJ) ? v[JJ] * rr : 0.0;
  v[JJ] = l;
  if (VAR == 1) col_updates_s<JJ>(std::make_integer_sequence<int, 16>{}, v, l);
  else col_updates<JJ>(std::make_integer_sequence<int, 16>{}, v, l);
  if (VAR != 2) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const double xs = (r == JJ) ? x[q] * rr : x[q];
      const double sv = row_bcast<JJ>(xs);
      x[q] = (r > JJ) ? fma(-l, sv, xs) : xs;
    }
  }
}
template <int VAR, int... JJ>
__device__ __forceinline__ void diag_steps_probe(std::integer_sequence<int, JJ...>, double (&v)[16],
                                                 double (&x)[4], int r) {
  (diag_step_probe<JJ, VAR>(v, x, r), ...);
}
template <int VAR>
__global__ void diag16_probe_kernel(int iters, long long* out, double* sink) {
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  double v0[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) v0[m] = (m == r ? 16.0 : 0.0) + 1.0 / (1.0 + (m > r ? m - r : r - m));
  double chk = 0.0;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    double v[16], x[4];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = v0[m] + 1e-9 * it;
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = (r == 4 * g + q) ? 1.0 : 0.0;
    diag_steps_probe<VAR>(std::make_integer_sequence<int, 16>{}, v, x, r);
    chk += v[15] + x[3];
  }
  const long long t1 = clock64();
  if (threadIdx.x == 0) out[VAR] = (t1 - t0) / iters;
  if (chk == 12345.0) sink[0] = chk;
}

#endif  // BO_TOOLS

// 16 x 16 MFMA tile: acc = sum_k A[k] op(B) over K = 16 * nk columns/rows from LDS.
// A(m, k) = SA[m * LP + k]; BT: B(k, n) = SB[n * LP + k], else SB[k * LP + n].
template <bool BT>
__device__ __forceinline__ v4d mma16(const double* SA, const double* SB, int nk, int lane) {
  v4d a = v4d_zero();
  const int r16 = lane & 15, kq = lane >> 4;
  for (int ks = 0; ks < 4 * nk; ++ks) {
    const int k = 4 * ks + kq;
    const double av = SA[r16 * LP + k];
    const double bv = BT ? SB[r16 * LP + k] : SB[k * LP + r16];
    a = mfma_f64(av, bv, a);
  }
  return a;
}

__device__ __forceinline__ void put16(double* D, v4d a, int lane, double scale) {
#pragma unroll
  for (int q = 0; q < 4; ++q) D[mfma_row(lane, q) * LP + mfma_col(lane)] = scale * a[q];
}

#ifdef BO_TOOLS
// S (64 x 64, lower part meaningful) -> L (lower, upper zeroed) in place, and
// D = L^{-1} (lower, upper zero).  Four 16-column panels: wave 0 factors the
// 16 x 16 diagonal block AND inverts it (pivots and columns broadcast inside
// 16-lane rows by DPP), the panel below is solved against that inverse on the
// MFMA, the trailing lower triangle takes the rank-16 update on the MFMA (wave
// 0 updates the next diagonal block and goes on factoring it while the other
// waves update the rest).  The inverse is then merged from the four block
// inverses by recursive doubling, X21 = -X22 L21 X11 (16 -> 32 -> 64), on the
// MFMA; the strictly-upper blocks of S serve as scratch for the products.
__device__ void potrf_trtri64(const Ctx& c, double* S, double* D, double* rinv, int* info, int row0,
                              double* Lc, lds_cnt_t* cnt, long long* ct = nullptr) {
  for (int e = c.tid; e < TB * TB; e += 256) D[(e >> 6) * LP + (e & 63)] = 0.0;
  __syncthreads();
  const int r = c.lane & 15, g = c.lane >> 4;
  if (c.tid == 0) *cnt = 0;
  // diagonal block p (rows/cols 16 p ..): wave 0 factors it in place, wave 1
  // builds its inverse into D
  auto diag_block = [&](int p) {
    const int c0 = 16 * p;
    double* T = S + c0 * LP + c0;
    if (c.wave == 0) {
      double v[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) v[m] = T[r * LP + m];
      int fail = 0;  // first non-positive pivot of the block (1-based), uniform
      diag_steps(std::make_integer_sequence<int, 16>{}, v, r, g, c.lane == 0, fail, rinv + c0,
                 Lc + 256 * (p & 1), cnt, 16 * p);
      if (fail && c.lane == 0) atomicCAS(info, 0, row0 + c0 + fail);
      if (g == 0) {
#pragma unroll
        for (int m = 0; m < 16; ++m) T[r * LP + m] = (m <= r) ? v[m] : 0.0;
      }
    } else {  // wave 1
      double x[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) x[q] = (r == 4 * g + q) ? 1.0 : 0.0;
      diag_inv_steps(std::make_integer_sequence<int, 16>{}, x, r, rinv + c0, Lc + 256 * (p & 1), cnt,
                     16 * p);
#pragma unroll
      for (int q = 0; q < 4; ++q) D[(c0 + r) * LP + c0 + 4 * g + q] = x[q];
    }
  };
  if (c.wave < 2) diag_block(0);
  __syncthreads();
  if (ct && c.tid == 0) ct[4] = wall_clock64();
#pragma unroll 1
  for (int p = 0; p < 3; ++p) {
    const int c0 = 16 * p;
    // panel below: L_{ib,p} = A_{ib,p} D_pp^T, one 16 x 16 tile per wave
    for (int ib = p + 1 + c.wave; ib < 4; ib += 4) {
      double* T = S + 16 * ib * LP + c0;
      const v4d a = mma16<true>(T, D + c0 * LP + c0, 1, c.lane);
      put16(T, a, c.lane, 1.0);
    }
    __syncthreads();
    // trailing update: tiles (ib, jb), p < jb <= ib; wave 0 takes (p+1, p+1)
    // and factors it right away while wave 1 inverts it, waves 2, 3 update the
    // rest
    const int nt = 3 - p;
    const int ntile = nt * (nt + 1) / 2;
    if (c.wave == 0) {
      const int c1 = c0 + 16;
      double* T = S + c1 * LP + c1;
      const v4d a = mma16<true>(S + c1 * LP + c0, S + c1 * LP + c0, 1, c.lane);
#pragma unroll
      for (int q = 0; q < 4; ++q) T[mfma_row(c.lane, q) * LP + mfma_col(c.lane)] -= a[q];
      diag_block(p + 1);
    } else if (c.wave == 1) {
      diag_block(p + 1);
    } else {
      for (int t = c.wave - 1; t < ntile; t += 2) {  // tiles 1.. (tile 0 = (p+1, p+1))
        int tr = 0;
        while ((tr + 1) * (tr + 2) / 2 <= t) ++tr;
        const int tc = t - tr * (tr + 1) / 2;
        const int r0 = c0 + 16 + 16 * tr, q0 = c0 + 16 + 16 * tc;
        const v4d a = mma16<true>(S + r0 * LP + c0, S + q0 * LP + c0, 1, c.lane);
#pragma unroll
        for (int q = 0; q < 4; ++q) S[(r0 + mfma_row(c.lane, q)) * LP + q0 + mfma_col(c.lane)] -= a[q];
      }
    }
    __syncthreads();
  }
  if (ct && c.tid == 0) ct[5] = wall_clock64();
  // 16 -> 32: pairs (0, 1) and (2, 3) (waves 0, 1): X21 = -X22 (L21 X11)
  if (c.wave < 2) {
    const int b1 = 32 * c.wave, b2 = b1 + 16;
    double* Tb = S + b1 * LP + b2;  // strictly-upper scratch
    v4d a = mma16<false>(S + b2 * LP + b1, D + b1 * LP + b1, 1, c.lane);
    put16(Tb, a, c.lane, 1.0);
    a = mma16<false>(D + b2 * LP + b2, Tb, 1, c.lane);
    put16(D + b2 * LP + b1, a, c.lane, -1.0);
  }
  __syncthreads();
  // 32 -> 64: X21 (rows 32.., cols 0..31) = -X22 (L21 X11); one 16 x 16 tile per wave
  {
    const int ti = c.wave >> 1, tj = c.wave & 1;
    double* Tb = S + 32;  // rows 0..31, cols 32..63: strictly upper
    const v4d a = mma16<false>(S + (32 + 16 * ti) * LP, D + 16 * tj, 2, c.lane);
    __syncthreads();  // the (masked-free) reads above precede the scratch writes of other waves
    put16(Tb + 16 * ti * LP + 16 * tj, a, c.lane, 1.0);
    __syncthreads();
    const v4d b = mma16<false>(D + (32 + 16 * ti) * LP + 32, Tb + 16 * tj, 2, c.lane);
    put16(D + (32 + 16 * ti) * LP + 16 * tj, b, c.lane, -1.0);
  }
  __syncthreads();
  for (int e = c.tid; e < TB * TB; e += 256) {
    const int rr = e >> 6, col = e & 63;
    if (col > rr) S[rr * LP + col] = 0.0;
  }
  __syncthreads();
}

#endif  // BO_TOOLS

// ---- the diagonal tile, column-owner form (round 3) ---------------------------------
// Lane r of every wave holds row r of the 64 x 64 block; wave w holds its
// columns 16 w .. 16 w + 15 (v[m] = A[r][16 w + m]).  Column J is factored by
// its owner wave J / 16 with no workgroup barrier: the pivot comes by
// v_readlane, L[J+1][J] too (the chain: pivot -> rsq -> scale -> the next
// pivot's update), the column goes to the column buffer Lc (column-major,
// stride 64) and a column counter in LDS; the later waves apply it to their
// columns as it appears (their row's L[r][J] and the uniform L[16 w + m][J]
// read back from Lc), so wave w + 1 starts factoring one column behind wave w's
// last.  Each wave then inverts its own 16 x 16 diagonal block from Lc while
// the later waves factor, and the inverse is merged by recursive doubling as
// in potrf_trtri64.  Replaces the four-panel scheme's panel solves and
// trailing updates, each behind a workgroup barrier, on the Cholesky's chain.
__device__ __forceinline__ double rcp_nr(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
}

// Column J = c0 + JL on its owner wave; d enters as the pivot d_J and leaves as
// d_{J+1}.  The pivots run on a chain of their own: d_{J+1} = a'_{J+1,J+1} -
// a'_{J+1,J}^2 / d_J (a' = the entries updated through column J - 1, read from
// lane J + 1 before this column's update), so one reciprocal per column is on
// it and 1 / sqrt(d_J) (the column's scale) runs beside it; the entries the
// next two pivots need (columns JL + 1, JL + 2) take L[.][J] by v_readlane,
// the others from the column buffer.
// VAR (timing variants, tools/probe_potrf64.py): 0 pivots from the column
// itself, 1 pivots on their own reciprocal chain, 2 = 0 with one Newton step
// on 1/sqrt, 3 = 0 without the LDS-fed updates (wrong results: the chain alone)
template <int VAR>
__device__ __forceinline__ double rsq_var(double v) {
  double r = __builtin_amdgcn_rsq(v);
  r = r * fma(-0.5 * v * r, r, 1.5);
  if (VAR != 2) r = r * fma(-0.5 * v * r, r, 1.5);
  return r;
}

// Column J = c0 + JL on its owner wave (VAR 1: d enters as the pivot d_J and
// leaves as d_{J+1}, computed as d_{J+1} = a'_{J+1,J+1} - a'_{J+1,J}^2 / d_J
// from lane J + 1's entries before this column's update).  The entries the
// next two pivots need (columns JL + 1, JL + 2) take L[.][J] by v_readlane,
// the others from the column buffer.
template <int JL, int VAR>
__device__ __forceinline__ void lcol_step(double (&v)[16], int r, int c0, int& fail, double* Lc,
                                          double* rinv, lds_cnt_t* cnt, double& d) {
  const int J = c0 + JL;
  if (VAR != 1) d = readlane_d(v[JL], J);
  if (!(d > 0.0) && fail == 0) fail = J + 1;
  const double rr = rsq_var<VAR>(d);
  double dn = 0.0;
  if constexpr (VAR == 1 && JL + 1 < 16) {
    const double inv = rcp_nr(d);
    const double x = readlane_d(v[JL], J + 1), y = readlane_d(v[JL + 1], J + 1);
    dn = fma(-(x * x), inv, y);
  }
  double l;
  if (VAR == 1) l = r > J ? v[JL] * rr : (r == J ? d * rr : 0.0);  // L[r][J] (r == J: sqrt(d_J))
  else l = r >= J ? v[JL] * rr : 0.0;
  v[JL] = l;
  if constexpr (JL + 1 < 16) v[JL + 1] = fma(-l, readlane_d(l, J + 1), v[JL + 1]);
  if constexpr (JL + 2 < 16) v[JL + 2] = fma(-l, readlane_d(l, J + 2), v[JL + 2]);
  // every lane stores the uniform rinv and counter words (no branch: a lane-0
  // branch per column let the compiler sink each column's updates to the next
  // pivot, i.e. onto the chain)
  Lc[J * 64 + r] = l;
  rinv[J] = rr;
  asm volatile("" ::: "memory");  // (compiler order only: LDS writes of one wave land in order)
  *cnt = J + 1;
  if (VAR != 3) {
#pragma unroll
    for (int m = JL + 3; m < 16; ++m) v[m] = fma(-l, Lc[J * 64 + c0 + m], v[m]);
  }
  if (VAR == 1) d = dn;
}

template <int VAR, int... JL>
__device__ __forceinline__ void lcol_steps(std::integer_sequence<int, JL...>, double (&v)[16], int r,
                                           int c0, int& fail, double* Lc, double* rinv, lds_cnt_t* cnt,
                                           double& d) {
  (lcol_step<JL, VAR>(v, r, c0, fail, Lc, rinv, cnt, d), ...);
}

// Column JJ of the inverse of the 16 x 16 diagonal block at c0 (POLL: wait for
// its L column on the counter): group g of the wave owns inverse columns
// 4 g .. 4 g + 3.
template <int JJ, bool POLL>
__device__ __forceinline__ void lcol_inv_step(double (&x)[4], int r, const double* rinv,
                                              const double* Lcb, lds_cnt_t* cnt, int c0) {
  if (POLL) {
    while (*cnt < c0 + JJ + 1) __builtin_amdgcn_s_sleep(0);
    asm volatile("" ::: "memory");
  }
  const double rr = rinv[JJ];
  const double l = Lcb[JJ * 64 + r];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const double xs = (r == JJ) ? x[q] * rr : x[q];
    const double sv = row_bcast<JJ>(xs);
    x[q] = (r > JJ) ? fma(-l, sv, xs) : xs;
  }
}

template <bool POLL, int... JJ>
__device__ __forceinline__ void lcol_inv_steps(std::integer_sequence<int, JJ...>, double (&x)[4], int r,
                                               const double* rinv, const double* Lcb, lds_cnt_t* cnt,
                                               int c0) {
  (lcol_inv_step<JJ, POLL>(x, r, rinv, Lcb, cnt, c0), ...);
}

// The 16 x 16 diagonal block inverse at c0 into D, and the zeros of its D band.
template <bool POLL>
__device__ __forceinline__ void lcol_block_inverse(int lane, int c0, double* D, const double* rinv,
                                                   const double* Lc, lds_cnt_t* cnt) {
  const int rb = lane & 15, g = lane >> 4;
  double x[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) x[q] = (rb == 4 * g + q) ? 1.0 : 0.0;
  for (int e = lane; e < 16 * 64; e += 64) {
    const int rr = e >> 6, col = e & 63;
    if (col < c0 || col >= c0 + 16) D[(c0 + rr) * LP + col] = 0.0;
  }
  lcol_inv_steps<POLL>(std::make_integer_sequence<int, 16>{}, x, rb, rinv + c0, Lc + c0 * 64 + c0, cnt,
                       c0);
#pragma unroll
  for (int q = 0; q < 4; ++q) D[(c0 + rb) * LP + c0 + 4 * g + q] = x[q];
}

// LDS flag handshake between waves of one workgroup (no barrier): the setter's
// LDS writes land in order before the flag; the waiter polls.
__device__ __forceinline__ void lds_flag_set(lds_cnt_t* f) {
  asm volatile("" ::: "memory");
  *f = 1;
}
__device__ __forceinline__ void lds_flag_wait(lds_cnt_t* f) {
  while (*f == 0) __builtin_amdgcn_s_sleep(0);
  asm volatile("" ::: "memory");
}

// S (64 x 64, lower part meaningful) -> L (lower, upper zeroed) in place, and
// D = L^{-1}; Lc, Tsc: 64 x 64 (pitch LP) doubles of LDS scratch (the column
// buffer, the merges' products); sfail, fl: 4 ints of LDS each.  The inverse
// is merged from the four block inverses while the later waves still factor:
//   wave 1:  X10 = -D11 (L10 D00), then T2 = L21 X11 (32 x 32)
//   wave 2:  T' = L32 D22
//   wave 3:  X32 = -D33 T' (D33: wave 0, one column behind wave 3's factor)
// and, after the one barrier, X21 = -X22 T2 (one 16 x 16 tile per wave).
template <int VAR>
__device__ void potrf_trtri64_cols(const Ctx& c, double* S, double* D, double* rinv, int* info, int row0,
                                   double* Lc, double* Tsc, lds_cnt_t* cnt, int* sfail, lds_cnt_t* fl,
                                   long long* ct = nullptr) {
  if (c.tid < 4) fl[c.tid] = 0;
  if (c.tid == 0) *cnt = 0;
  __syncthreads();
  const int w = c.wave, r = c.lane, c0 = 16 * w;
  double v[16];
#pragma unroll
  for (int m = 0; m < 16; m += 2) {
    const double2 a = *reinterpret_cast<const double2*>(S + r * LP + c0 + m);
    v[m] = a.x;
    v[m + 1] = a.y;
  }
  // the earlier waves' columns, applied as they appear
  int avail = 0;
  for (int J = 0; J < c0; ++J) {
    if (J >= avail) {
      while ((avail = *cnt) <= J) __builtin_amdgcn_s_sleep(0);
      asm volatile("" ::: "memory");
    }
    const double lr = Lc[J * 64 + r];
    const double2* col = reinterpret_cast<const double2*>(Lc + J * 64 + c0);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const double2 lm = col[m];
      v[2 * m] = fma(-lr, lm.x, v[2 * m]);
      v[2 * m + 1] = fma(-lr, lm.y, v[2 * m + 1]);
    }
  }
  if (ct && r == 0 && (w == 1 || w == 3)) ct[w == 1 ? 6 : 7] = wall_clock64();
  int fail = 0;  // first non-positive pivot of the wave's columns (1-based), uniform
  double d = readlane_d(v[0], c0);
  lcol_steps<VAR>(std::make_integer_sequence<int, 16>{}, v, r, c0, fail, Lc, rinv, cnt, d);
  if (r == 0) sfail[w] = fail;
  if (ct && c.tid == 192) ct[4] = wall_clock64();
#pragma unroll
  for (int m = 0; m < 16; m += 2) {
    double2 a;
    a.x = c0 + m <= r ? v[m] : 0.0;
    a.y = c0 + m + 1 <= r ? v[m + 1] : 0.0;
    *reinterpret_cast<double2*>(S + r * LP + c0 + m) = a;
  }
  if (w < 3) lcol_block_inverse<false>(r, c0, D, rinv, Lc, cnt);
  if (w == 0) {
    lds_flag_set(fl + 0);                             // D00
    lcol_block_inverse<true>(r, 48, D, rinv, Lc, cnt);  // D33, one column behind wave 3
    lds_flag_set(fl + 1);
  } else if (w == 1) {
    lds_flag_wait(fl + 0);
    put16(Tsc, mma16<false>(S + 16 * LP, D, 1, r), r, 1.0);                         // L10 D00
    put16(D + 16 * LP, mma16<false>(D + 16 * LP + 16, Tsc, 1, r), r, -1.0);          // X10
#pragma unroll 1
    for (int t = 0; t < 4; ++t) {  // T2 = L21 X11
      const int ti = t >> 1, tj = t & 1;
      put16(Tsc + (32 + 16 * ti) * LP + 16 * tj, mma16<false>(S + (32 + 16 * ti) * LP, D + 16 * tj, 2, r),
            r, 1.0);
    }
  } else if (w == 2) {
    put16(Tsc + 16, mma16<false>(S + 48 * LP + 32, D + 32 * LP + 32, 1, r), r, 1.0);  // L32 D22
    lds_flag_set(fl + 2);
  } else {
    lds_flag_wait(fl + 1);
    lds_flag_wait(fl + 2);
    put16(D + 48 * LP + 32, mma16<false>(D + 48 * LP + 48, Tsc + 16, 1, r), r, -1.0);  // X32
  }
  __syncthreads();
  if (c.tid == 0) {
    for (int q = 0; q < 4; ++q)
      if (sfail[q]) {
        atomicCAS(info, 0, row0 + sfail[q]);
        break;
      }
  }
  if (ct && c.tid == 0) ct[5] = wall_clock64();
  {  // X21 = -X22 T2, one 16 x 16 tile per wave
    const int ti = w >> 1, tj = w & 1;
    put16(D + (32 + 16 * ti) * LP + 16 * tj,
          mma16<false>(D + (32 + 16 * ti) * LP + 32, Tsc + 32 * LP + 16 * tj, 2, r), r, -1.0);
  }
  __syncthreads();
}

// ---- the diagonal step's two tile products, triangle-aware (round 5) -----------
// CRIT(k)'s L_{k,k-1} = A_{k,k-1} D_{k-1}^T and A_kk -= L L^T sit on the
// factorisation's chain.  As 32 x 32 quadrants per wave both ran the full
// 64-deep product on every quadrant (64 MFMAs per wave each).  D_{k-1} is lower
// triangular, so column block C of L needs only k < 16 (C + 1): wave w takes
// the 16 rows 16 w .. 16 w + 15 of L, 4 + 8 + 12 + 16 = 40 MFMAs, the same for
// every wave.  Only the 10 lower 16 x 16 blocks of A_kk are updated (the
// column-owner factor never reads above the diagonal), at most 3 per wave:
// 48 MFMAs.  Operands are read 16 B at a time as in acc_mma_nt (lane group kq
// takes k = 8 s + 2 kq and 8 s + 2 kq + 1 on both operands).
__device__ __forceinline__ void crit_trsm(const Ctx& c, v4d (&t)[4], const double* SA,
                                          const double* SD) {
  const int r16 = c.lane & 15, kq = c.lane >> 4;
  const double* pa = SA + (16 * c.wave + r16) * LP + 2 * kq;
#pragma unroll
  for (int C = 0; C < 4; ++C) t[C] = v4d_zero();
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const double2 a = *reinterpret_cast<const double2*>(pa + 8 * s);
#pragma unroll
    for (int C = 0; C < 4; ++C) {
      if (s < 2 * (C + 1)) {
        const double2 b = *reinterpret_cast<const double2*>(SD + (16 * C + r16) * LP + 8 * s + 2 * kq);
        t[C] = mfma_f64(a.x, b.x, t[C]);
        t[C] = mfma_f64(a.y, b.y, t[C]);
      }
    }
  }
}

// The lower blocks (I, J) of A_kk per wave: {(0,0), (3,0), (3,3)}, {(1,0),
// (1,1), (3,1)}, {(2,0), (2,1), (2,2)}, {(3,2)}.
__device__ __forceinline__ int syrk_blocks(int wave, int (&I)[3], int (&J)[3]) {
  if (wave == 0) { I[0] = 0; J[0] = 0; I[1] = 3; J[1] = 0; I[2] = 3; J[2] = 3; return 3; }
  if (wave == 1) { I[0] = 1; J[0] = 0; I[1] = 1; J[1] = 1; I[2] = 3; J[2] = 1; return 3; }
  if (wave == 2) { I[0] = 2; J[0] = 0; I[1] = 2; J[1] = 1; I[2] = 2; J[2] = 2; return 3; }
  I[0] = 3; J[0] = 2; I[1] = 3; J[1] = 2; I[2] = 3; J[2] = 2;
  return 1;
}

// blk -= L_I L_J^T (16 x 16, 64-deep) from the L tile in LDS.
__device__ __forceinline__ v4d syrk_block(const Ctx& c, v4d blk, const double* SL, int I, int J) {
  const int r16 = c.lane & 15, kq = c.lane >> 4;
  const double* pa = SL + (16 * I + r16) * LP + 2 * kq;
  const double* pb = SL + (16 * J + r16) * LP + 2 * kq;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const double2 a = *reinterpret_cast<const double2*>(pa + 8 * s);
    const double2 b = *reinterpret_cast<const double2*>(pb + 8 * s);
    blk = mfma_f64(-a.x, b.x, blk);
    blk = mfma_f64(-a.y, b.y, blk);
  }
  return blk;
}

// ---- the bulk tasks: a chunk of tile rows i in [i0, i1) ----------------------------
// KIND 0 TRSM    X0 <- A_ik,                   acc  = X0 X1^T  -> A_ik = L_ik, fL[i][k] = 1
// KIND 1 COLUPD  X0 <- L_ik (X1 if i == j),    acc  = A_ij - X0 X1^T -> A_ij, fA[i][j] = k + 1
// KIND 2 XSTEP   X0 <- L_ik,                   acc  = acc_ij + X0 X1 -> Linv_ij, fX[i][j] = k - j + 1
// The next tile's operands are loaded into registers while this tile's MFMAs
// run (when its inputs are already published; one poll by thread 0 decides).
struct Flags {
  u32 *fA, *fL, *fX, *fXd, *fAi, *abortw;
  int T;
  __device__ __forceinline__ u32* at(u32* a, int i, int j) const { return a + i * T + j; }
};

template <int KIND>
__device__ __forceinline__ void row_deps(const Flags& f, int i, int j, int k, const u32*& d1, u32& t1,
                                         const u32*& d2, u32& t2) {
  if (KIND == 0) { d1 = f.at(f.fA, i, k); t1 = (u32)k; d2 = d1; t2 = t1; }
  else if (KIND == 1) { d1 = f.at(f.fL, i, k); t1 = 1u; d2 = f.at(f.fA, i, j); t2 = (u32)k; }
  else { d1 = f.at(f.fL, i, k); t1 = 1u; d2 = f.at(f.fX, i, j); t2 = (u32)(k - j); }
}

template <int KIND>
__device__ __forceinline__ void row_issue(const Ctx& c, int i, int j, int k, double2 (&pv)[8],
                                          double (&pa)[16]) {
  if (!(KIND == 1 && i == j)) {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int e = c.tid + 256 * p;
      pv[p] = ld16(c.rA, toff(c, i, k, e >> 5, (e & 31) * 2));
    }
  }
  if (KIND == 1 || (KIND == 2 && k > j)) {
    const rsrc_t r = KIND == 1 ? c.rA : c.rI;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          pa[8 * a + 4 * b + q] = ld8(r, toff(c, i, j, c.wm + 16 * a + mfma_row(c.lane, q),
                                              c.wn + 16 * b + mfma_col(c.lane)));
  }
}

template <int KIND>
__device__ bool row_loop(const Ctx& c, const Flags& f, int k, int j, int i0, int i1, double* X0,
                         const double* X1, int* s_ok, int* s_rdy, long long* wsum,
                         long long* ph = nullptr) {
  long long tA = 0;
  double2 pv[8];
  double pa[16];
  Acc acc;
  bool pre = false;
  u32* pending = nullptr;  // flag of the previous tile, published once its stores drained
  u32 pending_val = 0;
  for (int i = i0; i < i1; ++i) {
    const u32 *d1, *d2;
    u32 t1, t2;
    if (ph && c.tid == 0) ph[4] += pre ? 1 : 0;
    if (!pre) {
      // never block while holding an unpublished row (a waiter could need it)
      if (pending) {
        publish(c, pending, pending_val);
        pending = nullptr;
      }
      row_deps<KIND>(f, i, j, k, d1, t1, d2, t2);
      if (!wait2(c, d1, t1, d2, t2, f.abortw, s_ok, wsum)) return false;
      row_issue<KIND>(c, i, j, k, pv, pa);
      // one round of polls over the rest of the chunk: rows whose inputs are
      // already published get their operands prefetched without a poll
      if (c.tid == 0) {
        int mask = 0;
        for (int ii = i + 1; ii < i1 && ii < i + 31; ++ii) {
          row_deps<KIND>(f, ii, j, k, d1, t1, d2, t2);
          if (flag_load(d1) >= t1 && flag_load(d2) >= t2) mask |= 1 << (ii - i);
          else break;
        }
        s_rdy[i & 1] = mask;
      }
    }
    if (ph && c.tid == 0) {
      tA = wall_clock64();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // traced runs: time the operand arrival
      ph[5] += wall_clock64() - tA;
    }
    const bool own_x0 = !(KIND == 1 && i == j);
    if (own_x0) {
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        const int e = c.tid + 256 * p;
        *reinterpret_cast<double2*>(X0 + (e >> 5) * LP + (e & 31) * 2) = pv[p];
      }
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          acc.t[a][b][q] = (KIND == 1 || (KIND == 2 && k > j)) ? pa[8 * a + 4 * b + q] : 0.0;
    __syncthreads();
    const int mask = s_rdy[i & 1];
    pre = (mask >> 1) & 1;
    if (pre) row_issue<KIND>(c, i + 1, j, k, pv, pa);
    long long tB = 0;
    if (ph && c.tid == 0) { tB = wall_clock64(); ph[0] += tB - tA; }
    if (KIND == 0) acc_mma_nt(c, acc, X0, X1, 1.0);
    else if (KIND == 1) acc_mma_nt(c, acc, own_x0 ? X0 : X1, X1, -1.0);
    else acc_mma_nt(c, acc, X0, X1, 1.0);  // X1 holds X_kj transposed
    long long tC = 0;
    if (ph && c.tid == 0) {
      // MFMAs retire before the timestamp only through a dependent use
      tC = wall_clock64();
      ph[1] += tC - tB;
    }
    // publish the previous tile (its stores were issued one tile ago; the
    // drain also covers the prefetch above, which has had the MFMAs' time)
    // (and the barrier that keeps X0 until every wave's MFMAs have read it)
    if (pending) {
      publish(c, pending, pending_val);
      pending = nullptr;
    } else {
      __syncthreads();
    }
    // next row's readiness in the other slot (its last readers passed this
    // iteration's barrier)
    if (c.tid == 0) s_rdy[(i + 1) & 1] = mask >> 1;
    if (KIND == 2) acc_store(c, acc, c.rI, i, j);
    else acc_store(c, acc, c.rA, i, KIND == 0 ? k : j);
    u32* fl;
    u32 val;
    if (KIND == 0) { fl = f.at(f.fL, i, k); val = 1u; }
    else if (KIND == 1) { fl = f.at(f.fA, i, j); val = (u32)(k + 1); }
    else { fl = f.at(f.fX, i, j); val = (u32)(k - j + 1); }
    if (i == i0) publish(c, fl, val);  // the first row of a chunk may be on the critical path
    else { pending = fl; pending_val = val; }
    if (ph && c.tid == 0) { ph[2] += wall_clock64() - tC; ph[3] += 1; }
  }
  if (pending) publish(c, pending, pending_val);
  return true;
}

// Batched column update: A_ij -= sum_{k in [kb, kb + nk)} L_ik L_jk^T for the
// rows of the chunk, the L_jk of the batch resident in LDS (XB[g]).  A_ij is
// loaded and stored once per batch instead of once per step: per tile update
// the HBM traffic falls from 96 KB (A operand + A_ij in + A_ij out) to
// 32 + 64 / nk KB -- the hand-off traffic, not the MFMAs, bounds the bulk.
// KIND 1: A_ij -= sum_k L_ik L_jk^T (fA[i][j] = kb + nk);
// KIND 2: acc_ij += sum_k L_ik X_kj (X_kj transposed in XB; fX[i][j] = kb + nk - j).
template <int KIND>
__device__ bool batched_update(const Ctx& c, const Flags& f, int kb, int nk, int j, int i0, int i1,
                               double* X0, double* XB0, double* XB1, double* XB2, int* s_ok,
                               int* s_rdy, long long* wsum, long long* ph = nullptr) {
  auto XB = [&](int g) { return g == 0 ? XB0 : (g == 1 ? XB1 : XB2); };
  const rsrc_t rc = KIND == 1 ? c.rA : c.rI;                      // C tile in / out
  u32* const fC = KIND == 1 ? f.fA : f.fX;                        // its version flags
  const u32 v0 = KIND == 1 ? (u32)kb : (u32)(kb - j);             // version before / after
  const u32 v1 = v0 + (u32)nk;
  const double sgn = KIND == 1 ? -1.0 : 1.0;
  double2 pv[8];
  double pa[16];
  Acc acc;
  bool pre = false;
  const int ke = kb + nk;
  auto issue_a = [&](int i, int k) {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int e = c.tid + 256 * p;
      pv[p] = ld16(c.rA, toff(c, i, k, e >> 5, (e & 31) * 2));
    }
  };
  auto issue_c = [&](int i) {
    // X_ij's first contributions (v0 = 0) start from zero: Linv is not
    // cleared ahead of the launch
    const bool zero = KIND == 2 && v0 == 0u;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          pa[8 * a + 4 * b + q] = zero ? 0.0
                                       : ld8(rc, toff(c, i, j, c.wm + 16 * a + mfma_row(c.lane, q),
                                                      c.wn + 16 * b + mfma_col(c.lane)));
  };
  for (int i = i0; i < i1; ++i) {
    long long tA = 0;
    if (ph && c.tid == 0) ph[4] += pre ? 1 : 0;
    if (!pre) {
      if (!wait2(c, f.at(f.fL, i, ke - 1), 1u, f.at(fC, i, j), v0, f.abortw, s_ok, wsum))
        return false;
      issue_c(i);
      if (KIND == 2 || i != j) issue_a(i, kb);
      if (c.tid == 0) {
        int mask = 0;
        for (int ii = i + 1; ii < i1 && ii < i + 31; ++ii) {
          if (flag_load(f.at(f.fL, ii, ke - 1)) >= 1u && flag_load(f.at(fC, ii, j)) >= v0)
            mask |= 1 << (ii - i);
          else
            break;
        }
        s_rdy[i & 1] = mask;
      }
    }
    if (ph && c.tid == 0) tA = wall_clock64();
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc.t[a][b][q] = pa[8 * a + 4 * b + q];
    __syncthreads();  // s_rdy
    const int mask = s_rdy[i & 1];
    const bool next = (mask >> 1) & 1;
    long long tB = 0, tm = 0;
    for (int g = 0; g < nk; ++g) {
      const bool own = KIND == 2 || i != j;  // COLUPD's diagonal tile: the A operand is XB(g)
      if (own) {
#pragma unroll
        for (int p = 0; p < 8; ++p) {
          const int e = c.tid + 256 * p;
          *reinterpret_cast<double2*>(X0 + (e >> 5) * LP + (e & 31) * 2) = pv[p];
        }
        __syncthreads();
      }
      // the next operand tile (this row's next step, or the next row's first
      // step and C) in flight under this step's MFMAs
      if (g + 1 < nk) {
        if (KIND == 2 || i != j) issue_a(i, kb + g + 1);
      } else if (next) {
        issue_c(i + 1);
        if (KIND == 2 || i + 1 != j) issue_a(i + 1, kb);
      }
      if (ph && c.tid == 0) tB = wall_clock64();
      acc_mma_nt(c, acc, own ? X0 : XB(g), XB(g), sgn);
      if (ph && c.tid == 0) tm += wall_clock64() - tB;
      __syncthreads();  // X0 free for the next step's operand
    }
    pre = next;
    if (c.tid == 0) s_rdy[(i + 1) & 1] = mask >> 1;
    long long tC = 0;
    if (ph && c.tid == 0) {
      tC = wall_clock64();
      ph[1] += tm;
      ph[0] += tC - tA - tm;
    }
    acc_store(c, acc, rc, i, j);
    publish(c, f.at(fC, i, j), v1);
    if (ph && c.tid == 0) { ph[2] += wall_clock64() - tC; ph[3] += nk; }
  }
  return true;
}

// The same batched update with the operand tiles prefetched two steps ahead
// (round 4): the chunk's (row, step) pairs form one stream e = (i - i0) nk + g;
// while step e's MFMAs run, the operand of e + 2 is in flight into the
// register slot step e just committed to LDS (two slots, e & 1; the slot is a
// compile-time index: the stream is walked two elements per iteration).  A
// sc1 operand load takes longer than one 64 x 64 x 64 step of MFMAs (round 3
// trace: ~0.9 us of every step waited on it); two steps cover it.  The next
// row's C tile goes with its first operand; rows are only prefetched when
// the poll at the last waited row start found them ready (as batched_update).
template <int KIND>
__device__ bool batched_update2(const Ctx& c, const Flags& f, int kb, int nk, int j, int i0, int i1,
                                double* X0, double* XB0, double* XB1, double* XB2, int* s_ok,
                                int* s_rdy, long long* wsum) {
  auto XB = [&](int g) { return g == 0 ? XB0 : (g == 1 ? XB1 : XB2); };
  const rsrc_t rc = KIND == 1 ? c.rA : c.rI;
  u32* const fC = KIND == 1 ? f.fA : f.fX;
  const u32 v0 = KIND == 1 ? (u32)kb : (u32)(kb - j);
  const u32 v1 = v0 + (u32)nk;
  const double sgn = KIND == 1 ? -1.0 : 1.0;
  const int ke = kb + nk;
  const int E = (i1 - i0) * nk;
  double2 pv0[8], pv1[8];
  double pa[16];
  Acc acc;
  int issued = 0;  // stream elements whose loads are issued (a prefix)
  int mask = 0;    // bit r: row i + r found ready by the last poll
  auto own = [&](int i) { return KIND == 2 || i != j; };
  auto issue_a = [&](double2 (&pv)[8], int i, int k) {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int e = c.tid + 256 * p;
      pv[p] = ld16(c.rA, toff(c, i, k, e >> 5, (e & 31) * 2));
    }
  };
  auto issue_c = [&](int i) {
    // X_ij's first contributions (v0 = 0) start from zero: Linv is not
    // cleared ahead of the launch
    const bool zero = KIND == 2 && v0 == 0u;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          pa[8 * a + 4 * b + q] = zero ? 0.0
                                       : ld8(rc, toff(c, i, j, c.wm + 16 * a + mfma_row(c.lane, q),
                                                      c.wn + 16 * b + mfma_col(c.lane)));
  };
  bool ok = true;
  // Deferred publish (round 6): a row's C tile is stored at its last step and
  // its flag published at the END of the next step, draining only those
  // stores (publish_after: the loads issued after them -- the next operands --
  // stay in flight).  A full vmcnt(0) drain right after the stores waited for
  // the write-through stores and the in-flight prefetch together, every row.
  // The chunk's first row publishes at once (it may be the diagonal tile the
  // chain waits on), and nothing blocks while a row is unpublished.
  u32* pending = nullptr;
  u32 pend_val = 0;
  int pend_younger = 0;  // vector-memory instructions issued after its stores
  // this thread's vector-memory instructions per issue_c / issue_a
  const int n_c = (KIND == 2 && v0 == 0u) ? 0 : 16;
  const int n_a = 8;
  auto flush = [&]() {
    if (pending) {
      publish(c, pending, pend_val);
      pending = nullptr;
    }
  };
  // one stream element in register slot S (the other slot: O)
  auto step = [&](int e, double2 (&pvS)[8], double2 (&pvO)[8]) {
    const int r = e / nk, g = e - r * nk, i = i0 + r;
    if (g == 0) {
      if (issued <= e) {  // not prefetched: wait for the row, then its C and two operands
        flush();  // never block while holding an unpublished row (a waiter could need it)
        if (!wait2(c, f.at(f.fL, i, ke - 1), 1u, f.at(fC, i, j), v0, f.abortw, s_ok, wsum)) {
          ok = false;
          return;
        }
        issue_c(i);
        if (own(i)) issue_a(pvS, i, kb);
        issued = e + 1;
        if (nk > 1) {
          if (own(i)) issue_a(pvO, i, kb + 1);
          issued = e + 2;
        }
        if (c.tid == 0) {
          int m = 0;
          for (int ii = i + 1; ii < i1 && ii < i + 31; ++ii) {
            if (flag_load(f.at(f.fL, ii, ke - 1)) >= 1u && flag_load(f.at(fC, ii, j)) >= v0)
              m |= 1 << (ii - i);
            else
              break;
          }
          s_rdy[i & 1] = m;
        }
        __syncthreads();
        mask = s_rdy[i & 1];
      } else {
        mask >>= 1;  // this row was prefetched: the last poll's word, one row on
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int q = 0; q < 4; ++q) acc.t[a][b][q] = pa[8 * a + 4 * b + q];
    }
    if (own(i)) {
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        const int x = c.tid + 256 * p;
        *reinterpret_cast<double2*>(X0 + (x >> 5) * LP + (x & 31) * 2) = pvS[p];
      }
      __syncthreads();
    }
    // element e + 2 into the slot just committed: this row, or the next one
    // when the poll found it ready (its C tile with its first operand; this
    // row's C was taken at its start)
    const int e2 = e + 2;
    if (e2 < E && issued == e2) {
      const int r2 = e2 / nk, g2 = e2 - r2 * nk, i2 = i0 + r2;
      if (r2 == r || (r2 == r + 1 && (mask & 2))) {
        if (g2 == 0) issue_c(i2);
        if (own(i2)) issue_a(pvS, i2, kb + g2);
        issued = e2 + 1;
        pend_younger += (g2 == 0 ? n_c : 0) + (own(i2) ? n_a : 0);
      }
    }
    acc_mma_nt(c, acc, own(i) ? X0 : XB(g), XB(g), sgn);
    if (pending) {  // the previous row: its stores had this step's MFMAs to land
      publish_after(c, pending, pend_val, pend_younger);
      pending = nullptr;
    } else {
      __syncthreads();  // X0 free for the next element's operand
    }
    if (g == nk - 1) {
      acc_store(c, acc, rc, i, j);
      if (i == i0 || e + 1 >= E) {
        publish(c, f.at(fC, i, j), v1);
      } else {
        // (compiler order: no later load may be hoisted above these stores,
        // or publish_after's count would not cover them)
        asm volatile("" ::: "memory");
        pending = f.at(fC, i, j);
        pend_val = v1;
        pend_younger = 0;
      }
    }
  };
  for (int e = 0; e < E; e += 2) {
    step(e, pv0, pv1);
    if (!ok) return false;
    if (e + 1 < E) {
      step(e + 1, pv1, pv0);
      if (!ok) return false;
    }
  }
  flush();
  return true;
}

// acc += SA^T SB, 64-deep, both operands as stored (row-major [k][col]): lane
// (r16, kq) reads SA[k][wm + r16] and SB[k][wn + r16] -- 16 consecutive
// doubles per k row, no transposed staging (A^{-1}'s X_Ki^T X_Kj).
__device__ __forceinline__ void acc_mma_tn(const Ctx& c, Acc& a, const double* SA, const double* SB) {
  const int r16 = c.lane & 15, kq = c.lane >> 4;
#pragma unroll 4
  for (int ks = 0; ks < 16; ++ks) {
    const int k = 4 * ks + kq;
    const double a0 = SA[k * LP + c.wm + r16], a1 = SA[k * LP + c.wm + 16 + r16];
    const double b0 = SB[k * LP + c.wn + r16], b1 = SB[k * LP + c.wn + 16 + r16];
    a.t[0][0] = mfma_f64(a0, b0, a.t[0][0]);
    a.t[0][1] = mfma_f64(a0, b1, a.t[0][1]);
    a.t[1][0] = mfma_f64(a1, b0, a.t[1][0]);
    a.t[1][1] = mfma_f64(a1, b1, a.t[1][1]);
  }
}

// A^{-1} tiles: Ainv_ij += sum_{K in [kb, ke), K >= i} X_Ki^T X_Kj for the
// rows i of the chunk (i >= j), the X_Kj of the batch resident in LDS (XB[g],
// as stored).  Row i's first contribution (K = i) starts from zero, so A^{-1}
// needs no clearing; fAi[i][j] counts the contributions applied (ke - i after
// this task).  X_Ki is final once X_{ke-1, i} is (each X_Ki is formed from the
// X_mi, m < K), so one flag per operand column: fXd[ke-1][i], or fL[i][i] when
// ke - 1 == i (X_ii = D_i).  The (row, step) pairs form one stream; the
// operand of the next pair is in flight in registers under this pair's MFMAs
// (the next row's only when one poll found its inputs published).
__device__ bool ainv_update(const Ctx& c, const Flags& f, int kb, int nk, int j, int i0, int i1,
                            double* X0, double* XB0, double* XB1, double* XB2, rsrc_t rAi,
                            int* s_ok, int* s_rdy, long long* wsum) {
  auto XB = [&](int g) { return g == 0 ? XB0 : (g == 1 ? XB1 : XB2); };
  const int ke = kb + nk;
  Acc acc;
  double2 pv[8];
  double pa[16];
  auto xd_flag = [&](int i) { return (ke - 1 == i) ? f.at(f.fL, i, i) : f.at(f.fXd, ke - 1, i); };
  auto g_first = [&](int i) { return i > kb ? i - kb : 0; };  // K = kb + g >= i
  auto issue_a = [&](int i, int K) {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int e = c.tid + 256 * p;
      pv[p] = ld16(c.rI, toff(c, K, i, e >> 5, (e & 31) * 2));
    }
  };
  auto issue_c = [&](int i) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          pa[8 * a + 4 * b + q] = ld8(rAi, toff(c, i, j, c.wm + 16 * a + mfma_row(c.lane, q),
                                               c.wn + 16 * b + mfma_col(c.lane)));
  };
  bool pre = false;  // this row's C and first operand already in flight
  for (int i = i0; i < i1; ++i) {
    const int g0 = g_first(i);
    const u32 v0 = (u32)(kb + g0 - i);
    if (!pre) {
      if (!wait2(c, xd_flag(i), 1u, f.at(f.fAi, i, j), v0, f.abortw, s_ok, wsum)) return false;
      if (v0 > 0) issue_c(i);
      if (i != j) issue_a(i, kb + g0);
    }
    // the next row's readiness, polled once
    if (c.tid == 0) {
      int r = 0;
      if (i + 1 < i1) {
        const u32 v1 = (u32)(kb + g_first(i + 1) - (i + 1));
        r = flag_load(xd_flag(i + 1)) >= 1u && flag_load(f.at(f.fAi, i + 1, j)) >= v1;
      }
      s_rdy[i & 1] = r;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc.t[a][b][q] = v0 > 0 ? pa[8 * a + 4 * b + q] : 0.0;
    __syncthreads();
    const bool next = s_rdy[i & 1] != 0;
    for (int g = g0; g < nk; ++g) {
      const bool own = i != j;
      if (own) {
#pragma unroll
        for (int p = 0; p < 8; ++p) {
          const int e = c.tid + 256 * p;
          *reinterpret_cast<double2*>(X0 + (e >> 5) * LP + (e & 31) * 2) = pv[p];
        }
        __syncthreads();
      }
      if (g + 1 < nk) {
        if (own) issue_a(i, kb + g + 1);
      } else if (next) {
        const int gn = g_first(i + 1);
        if (kb + gn - (i + 1) > 0) issue_c(i + 1);
        if (i + 1 != j) issue_a(i + 1, kb + gn);
      }
      acc_mma_tn(c, acc, own ? X0 : XB(g), XB(g));
      __syncthreads();  // X0 free for the next operand
    }
    pre = next;
    acc_store(c, acc, rAi, i, j);
    publish(c, f.at(f.fAi, i, j), (u32)(ke - i));
  }
  return true;
}

// nb > 1: nb independent matrices (A + m * np^2, Linv + m * np^2, info[m], flag
// block m) share the launch; each task names its matrix in bits 9-15 of x, and
// the queue interleaves the matrices' own queues, so one matrix's diagonal
// chain runs while the others' bulk updates fill the CUs.
__global__ __launch_bounds__(256) void chol_dag_kernel(double* __restrict__ A, double* __restrict__ Linv,
                                                       int np, int T, const int4* __restrict__ tasks,
                                                       int ntasks, u32* __restrict__ flags,
                                                       int* __restrict__ info,
                                                       long long* __restrict__ trace, int nb,
                                                       int pf2, double* __restrict__ Ainv,
                                                       int zero_upper) {
  __shared__ __attribute__((aligned(16))) double X0[TB * LP];
  __shared__ __attribute__((aligned(16))) double X1[TB * LP];
  __shared__ __attribute__((aligned(16))) double X2[TB * LP];  // batched update operands
  __shared__ __attribute__((aligned(16))) double X3[TB * LP];
  __shared__ double rinv[TB];
  __shared__ int s_cnt;
  __shared__ int s_fail[4];
  __shared__ int s_fl[4];
  __shared__ int s_ok;
  __shared__ int s_rdy[2];
  __shared__ int s_task;

  Ctx c;
  c.np = np;
  c.tid = threadIdx.x;
  c.lane = c.tid & 63;
  c.wave = c.tid >> 6;
  c.wm = (c.wave >> 1) * 32;
  c.wn = (c.wave & 1) * 32;
  const u32 bytes = (u32)np * (u32)np * 8u;
  c.rA = make_rsrc(A, bytes);
  c.rI = make_rsrc(Linv, bytes);
  u32* head = flags;
  u32* abortw = flags + 1;
  const int fstride = (Ainv ? 5 : 4) * T * T;  // flag words per matrix
  u32* fA = flags + NFLAG0;
  u32* fL = fA + T * T;
  u32* fX = fL + T * T;
  u32* fXd = fX + T * T;
  const rsrc_t rAi = make_rsrc(Ainv ? Ainv : A, bytes);
#define F(arr, i, j) (arr + (i) * T + (j))
  Flags fl;
  fl.fA = fA; fl.fL = fL; fl.fX = fX; fl.fXd = fXd; fl.fAi = fXd + T * T;
  fl.abortw = abortw; fl.T = T;
  int cur = 0;          // matrix of the buffer resources / flags above
  int* minfo = info;

  // The strictly upper tiles of every Linv (zero in the result): stored here
  // by the workgroups past the first 8 before their first claim -- the stores
  // drain while those workgroups wait for the first diagonal steps, where a
  // memset of the whole np x np ahead of the launch cost 17.9 us of the
  // closure at n = 4096.  No task reads an upper tile.
  if (zero_upper && (int)blockIdx.x >= 8) {
    const int nz = (int)gridDim.x - 8, zb = (int)blockIdx.x - 8;
    const int row = c.tid >> 2, col = (c.tid & 3) * 16;
    for (int u = zb; u < nb * T * T; u += nz) {
      const int m = u / (T * T), r = u - m * (T * T), ti = r / T, tj = r - ti * T;
      if (ti >= tj) continue;
      double2* p = reinterpret_cast<double2*>(Linv + (size_t)m * np * np +
                                              (size_t)(ti * TB + row) * np + tj * TB + col);
#pragma unroll
      for (int e = 0; e < 8; ++e) p[e] = make_double2(0.0, 0.0);
    }
  }
  if (c.tid == 0) s_task = (int)__hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  int t = s_task;
  __syncthreads();
  Acc acc;
  while (t < ntasks) {
    const int4 tk = tasks[t];
    const int type = tk.x & 0xff, fin = (tk.x >> 8) & 1, nk = tk.x >> 16;
    const int mid = (tk.x >> 9) & 0x7f;
    if (mid != cur) {  // rebind to matrix mid
      cur = mid;
      const size_t off = (size_t)mid * (size_t)np * (size_t)np;
      c.rA = make_rsrc(A + off, bytes);
      c.rI = make_rsrc(Linv + off, bytes);
      fA = flags + NFLAG0 + (size_t)mid * fstride;
      fL = fA + T * T;
      fX = fL + T * T;
      fXd = fX + T * T;
      fl.fA = fA; fl.fL = fL; fl.fX = fX; fl.fXd = fXd; fl.fAi = fXd + T * T;
      minfo = info + mid;
    }
    long long wsum = 0;
    long long phs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    long long* ph = trace ? phs : nullptr;
    if (trace && c.tid == 0) trace[4 * t] = wall_clock64();
    const int k = tk.y, j = tk.z, i0 = tk.w & 0xffff, i1 = tk.w >> 16;
    bool ok = true;
    if (type == T_CRIT) {
      // roles: the factor's input S = X1 (free once the TRSM has read D_{k-1}),
      // its inverse D = X0 (free once the A_kk update has read L_{k,k-1})
      if (k > 0) {
        // the bulk's inputs (A_{k,k-1}, A_kk at version k-1) are usually ready
        // before D_{k-1}: load them while the previous diagonal step runs, so
        // only D_{k-1}'s load, two tile products and the L_{k,k-1} hand-off
        // stay on the chain
        int bI[3], bJ[3];
        const int nbk = syrk_blocks(c.wave, bI, bJ);
        v4d akk[3];
        ok = wait2(c, F(fA, k, k - 1), (u32)(k - 1), F(fA, k, k), (u32)(k - 1), abortw, &s_ok, &wsum);
        if (ok) {
          tile_to_lds(c, c.rA, k, k - 1, X0);
#pragma unroll
          for (int b = 0; b < 3; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              akk[b][r] = b < nbk ? ld8(c.rA, toff(c, k, k, 16 * bI[b] + mfma_row(c.lane, r),
                                                 16 * bJ[b] + mfma_col(c.lane)))
                                  : 0.0;
          ok = wait2(c, F(fL, k - 1, k - 1), 1u, F(fL, k - 1, k - 1), 1u, abortw, &s_ok, &wsum);
        }
        if (ok) {
          tile_to_lds(c, c.rI, k - 1, k - 1, X1);
          __syncthreads();
          v4d tl[4];
          crit_trsm(c, tl, X0, X1);  // rows 16 w.. of L_{k,k-1} = A_{k,k-1} D_{k-1}^T
          // the wave's own rows: X0 <- L (only this wave read them), and to A
#pragma unroll
          for (int C = 0; C < 4; ++C)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = 16 * c.wave + mfma_row(c.lane, r), col = 16 * C + mfma_col(c.lane);
              X0[row * LP + col] = tl[C][r];
              st8(c.rA, toff(c, k, k - 1, row, col), tl[C][r]);  // in flight under the update
            }
          __syncthreads();  // X0 = L_{k,k-1} complete; every wave's reads of X1 done
#pragma unroll
          for (int b = 0; b < 3; ++b)
            if (b < nbk) akk[b] = syrk_block(c, akk[b], X0, bI[b], bJ[b]);  // A_kk -= L L^T
#pragma unroll
          for (int b = 0; b < 3; ++b)
            if (b < nbk)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                X1[(16 * bI[b] + mfma_row(c.lane, r)) * LP + 16 * bJ[b] + mfma_col(c.lane)] = akk[b][r];
          publish(c, F(fL, k, k - 1), 1u);  // (its barrier also orders the X1 writes)
        }
      } else {
        tile_to_lds(c, c.rA, 0, 0, X1);
      }
      if (ok) {
        __syncthreads();
        long long* ct = trace ? trace + 4 * ntasks + 8 * k : nullptr;
        if (ct && c.tid == 0) ct[0] = wall_clock64();
        potrf_trtri64_cols<0>(c, X1, X0, rinv, minfo, k * TB, X2, X3, (lds_cnt_t*)&s_cnt, s_fail,
                              (lds_cnt_t*)s_fl, ct);
        if (ct && c.tid == 0) ct[1] = wall_clock64();
        if (ct && c.tid == 0) ct[2] = wall_clock64();
        lds_to_tile(c, X1, c.rA, k, k);
        lds_to_tile(c, X0, c.rI, k, k);
        publish(c, F(fL, k, k), 1u);
        if (ct && c.tid == 0) ct[3] = wall_clock64();
      }
    } else if (type == T_TRSM) {
      ok = wait2(c, F(fL, k, k), 1u, F(fL, k, k), 1u, abortw, &s_ok, &wsum);
      if (ok) tile_to_lds(c, c.rI, k, k, X1);  // D_k
      if (ok) ok = row_loop<0>(c, fl, k, j, i0, i1, X0, X1, &s_ok, s_rdy, &wsum, ph);
    } else if (type == T_COLUPD && nk > 1) {
      ok = wait2(c, F(fL, j, k + nk - 1), 1u, F(fL, j, k + nk - 1), 1u, abortw, &s_ok, &wsum);
      if (ok) {
        for (int g = 0; g < nk; ++g)  // L_jk of the batch
          tile_to_lds(c, c.rA, j, k + g, g == 0 ? X1 : (g == 1 ? X2 : X3));
        __syncthreads();
        ok = (pf2 && !ph) ? batched_update2<1>(c, fl, k, nk, j, i0, i1, X0, X1, X2, X3, &s_ok, s_rdy, &wsum)
                          : batched_update<1>(c, fl, k, nk, j, i0, i1, X0, X1, X2, X3, &s_ok, s_rdy, &wsum, ph);
      }
    } else if (type == T_COLUPD) {
      ok = wait2(c, F(fL, j, k), 1u, F(fL, j, k), 1u, abortw, &s_ok, &wsum);
      if (ok) tile_to_lds(c, c.rA, j, k, X1);  // L_jk
      if (ok) ok = row_loop<1>(c, fl, k, j, i0, i1, X0, X1, &s_ok, s_rdy, &wsum, ph);
    } else if (type == T_AINV) {
      const int kl = k + nk - 1;  // X_{k..kl, j} final once X_{kl, j} is
      if (kl == j) ok = wait2(c, F(fL, j, j), 1u, F(fL, j, j), 1u, abortw, &s_ok, &wsum);
      else ok = wait2(c, F(fXd, kl, j), 1u, F(fXd, kl, j), 1u, abortw, &s_ok, &wsum);
      if (ok) {
        for (int g = j > k ? j - k : 0; g < nk; ++g)  // X_Kj as stored (K >= j: the rest is 0)
          tile_to_lds(c, c.rI, k + g, j, g == 0 ? X1 : (g == 1 ? X2 : X3));
        __syncthreads();
        ok = ainv_update(c, fl, k, nk, j, i0, i1, X0, X1, X2, X3, rAi, &s_ok, s_rdy, &wsum);
      }
    } else if (nk > 1) {  // T_XSTEP, batched: the far rows of steps k .. k + nk - 1
      const int kl = k + nk - 1;  // X_{k..kl, j} final once X_{kl, j} is
      if (kl == j) ok = wait2(c, F(fL, j, j), 1u, F(fL, j, j), 1u, abortw, &s_ok, &wsum);
      else ok = wait2(c, F(fXd, kl, j), 1u, F(fXd, kl, j), 1u, abortw, &s_ok, &wsum);
      if (ok) {
        for (int g = 0; g < nk; ++g)  // X_kj transposed (X_jj = D_j)
          tile_to_lds_t(c, c.rI, k + g, j, g == 0 ? X1 : (g == 1 ? X2 : X3));
        __syncthreads();
        ok = (pf2 && !ph) ? batched_update2<2>(c, fl, k, nk, j, i0, i1, X0, X1, X2, X3, &s_ok, s_rdy, &wsum)
                          : batched_update<2>(c, fl, k, nk, j, i0, i1, X0, X1, X2, X3, &s_ok, s_rdy, &wsum, ph);
      }
    } else {  // T_XSTEP: column j of X at step k
      if (k == j) {
        ok = wait2(c, F(fL, k, k), 1u, F(fL, k, k), 1u, abortw, &s_ok, &wsum);
        if (ok) tile_to_lds_t(c, c.rI, k, k, X1);  // X_kk = D_k (transposed)
      } else if (fin) {
        ok = wait2(c, F(fX, k, j), (u32)(k - j), F(fL, k, k), 1u, abortw, &s_ok, &wsum);
        if (ok) {
          tile_to_lds(c, c.rI, k, k, X0);  // D_k
          tile_to_lds(c, c.rI, k, j, X1);  // acc_kj
          __syncthreads();
          acc_zero(acc);
          acc_mma<false>(c, acc, X0, X1, -1.0);  // X_kj = -D_k acc_kj
          __syncthreads();
          acc_to_lds_t(c, acc, X1);
          acc_store(c, acc, c.rI, k, j);
          publish(c, F(fXd, k, j), 1u);
        }
      } else {
        ok = wait2(c, F(fXd, k, j), 1u, F(fXd, k, j), 1u, abortw, &s_ok, &wsum);
        if (ok) tile_to_lds_t(c, c.rI, k, j, X1);
      }
      if (ok && i0 < i1) {
        __syncthreads();  // X1 (X_kj) complete before the row loop reads it
        ok = row_loop<2>(c, fl, k, j, i0, i1, X0, X1, &s_ok, s_rdy, &wsum, ph);
      }
    }
    if (trace && c.tid == 0) {
      trace[4 * t + 1] = wall_clock64();
      trace[4 * t + 3] = wsum;
      long long* pt = trace + 4 * ntasks + 8 * T + 8 * t;
      for (int e = 0; e < 8; ++e) pt[e] = phs[e];
      trace[4 * t + 2] = (long long)blockIdx.x | ((long long)tk.x << 16) | ((long long)k << 24) |
                         ((long long)j << 40);
    }
    // claim the next task only now: a task claimed early would sit behind this
    // one (a critical-path task claimed by a busy workgroup stalls the chain)
    if (c.tid == 0)
      s_task = ok ? (int)__hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                  : ntasks;
    __syncthreads();
    t = s_task;
    __syncthreads();
  }
  if (c.tid == 0 && flag_load(abortw))
    for (int m = 0; m < nb; ++m) atomicExch(info + m, -1);
#undef F
}

// ---- host: task table (cached per device and order) ------------------------------
struct DagTable {
  int4* dev = nullptr;
  int n = 0;
};

void push_rows(std::vector<int4>& v, int type, int k, int j, int lo, int hi, bool first_fin,
               int ch = CH, int first_ch = 0) {
  bool first = true;
  for (int i0 = lo; i0 < hi;) {
    const int c = (first && first_ch > 0) ? first_ch : ch;
    const int i1 = i0 + c < hi ? i0 + c : hi;
    v.push_back(make_int4(type | ((first && first_fin) ? 256 : 0), k, j, i0 | (i1 << 16)));
    first = false;
    i0 = i1;
  }
}

// Rows in the first chunk of a batched column update (the chunk holding the
// diagonal tile A(j, j)): the batched updates of one column are serialised on
// that tile's versions; with a whole chb-row chunk each link took ~45 us for 3
// steps at n = 4096, as slow as the diagonal chain it feeds (round-5 trace:
// every third diagonal step waited 25-35 us on it).  BO_CHOL_DIAG_CH overrides
// the default at the call (0: chb).  A dedicated workgroup per diagonal chain
// (CRIT(k) run in order, never claimed late) was measured too: no gain once
// CRIT waits on its inputs instead, and the restructured loop cost 12% in
// register allocation (1.65 -> 1.84 ms).
static int diag_chunk_rows() {
  static const int r = [] {
    const char* e = getenv("BO_CHOL_DIAG_CH");
    return e ? atoi(e) : -1;
  }();
  return r;
}

// Queue order: the generation order above is a topological order of the task
// DAG; it is re-sorted by bottom level (estimated time from the task's start to
// the end of the run along its longest chain of dependants), which keeps a
// topological order (every dependant has a strictly smaller bottom level) and
// puts the diagonal chain and the tiles it waits on ahead of the bulk updates.
std::vector<int4> priority_order(const std::vector<int4>& v, int T) {
  const int n = (int)v.size();
  auto tix = [T](int i, int j) { return (size_t)i * T + j; };
  std::vector<int> prodL((size_t)T * T, -1), prodXd((size_t)T * T, -1);
  // version-indexed producers: A(i,j) after v updates (v = 1..j), X(i,j) after v
  std::vector<std::vector<int>> prodA((size_t)T * T), prodX((size_t)T * T), prodAi((size_t)T * T);
  for (int t = 0; t < n; ++t) {
    const int type = v[t].x & 0xff, fin = (v[t].x >> 8) & 0xff, k = v[t].y, j = v[t].z;
    const int nk = std::max(1, v[t].x >> 16);
    const int i0 = v[t].w & 0xffff, i1 = v[t].w >> 16;
    if (type == T_CRIT) {
      prodL[tix(k, k)] = t;
      if (k > 0) prodL[tix(k, k - 1)] = t;
    } else if (type == T_TRSM) {
      for (int i = i0; i < i1; ++i) prodL[tix(i, k)] = t;
    } else if (type == T_COLUPD) {
      for (int i = i0; i < i1; ++i) {
        auto& pa = prodA[tix(i, j)];
        if ((int)pa.size() < k + nk + 1) pa.resize(k + nk + 1, -1);
        pa[k + nk] = t;
      }
    } else if (type == T_AINV) {
      for (int i = i0; i < i1; ++i) {  // version = contributions applied = ke - i
        auto& pv = prodAi[tix(i, j)];
        if ((int)pv.size() < k + nk - i + 1) pv.resize(k + nk - i + 1, -1);
        pv[k + nk - i] = t;
      }
    } else {
      if (fin && k > j) prodXd[tix(k, j)] = t;
      for (int i = i0; i < i1; ++i) {
        auto& px = prodX[tix(i, j)];
        if ((int)px.size() < k + nk - j + 1) px.resize(k + nk - j + 1, -1);
        px[k + nk - j] = t;
      }
    }
  }
  auto verA = [&](int i, int j, int ver) {
    const auto& pa = prodA[tix(i, j)];
    return ver >= 1 && ver < (int)pa.size() ? pa[ver] : -1;
  };
  auto verX = [&](int i, int j, int ver) {
    const auto& px = prodX[tix(i, j)];
    return ver >= 1 && ver < (int)px.size() ? px[ver] : -1;
  };
  std::vector<std::vector<int>> deps(n);
  std::vector<double> dur(n);
  // CRIT's weight in the bottom levels (BO_CHOL_CRIT_W): above 1 it lifts the
  // factorisation's tasks (every path to a diagonal step) over the inverse's
  // XSTEP chains, which feed no diagonal step -- measured slower (the inverse's
  // work piles up into the tail: 1.76 -> 1.85-2.35 ms at 2-16); below 1 the
  // 28 us estimate matches round 3's shorter diagonal step: 0.25 measured
  // n = 4096 1.769-1.779 -> 1.760-1.762 ms, 3 x 2048 0.866-0.883 -> 0.855-0.859
  // ms (profiles/r03/cholesky/critw*.log).  Dependants still sort after their
  // inputs (ties keep the generation order), so the queue stays topological.
  // Only finite weights >= 0 are taken: a negative one would give CRIT a
  // negative duration, sort dependants ahead of their inputs and leave the
  // persistent launch spinning until its timeout.
  double crit_w = 0.25;
  if (const char* e = getenv("BO_CHOL_CRIT_W")) {
    char* end = nullptr;
    const double w = strtod(e, &end);
    if (end != e && std::isfinite(w) && w >= 0.0) crit_w = w;
  }
  for (int t = 0; t < n; ++t) {
    const int type = v[t].x & 0xff, fin = (v[t].x >> 8) & 0xff, k = v[t].y, j = v[t].z;
    const int nk = std::max(1, v[t].x >> 16);
    const int i0 = v[t].w & 0xffff, i1 = v[t].w >> 16;
    auto& d = deps[t];
    const int rows = i1 - i0;
    if (type == T_CRIT) {
      if (k > 0) {
        d.push_back(verA(k, k - 1, k - 1));
        d.push_back(prodL[tix(k - 1, k - 1)]);
        d.push_back(verA(k, k, k - 1));
      }
      dur[t] = 28.0 * crit_w;
    } else if (type == T_TRSM) {
      d.push_back(prodL[tix(k, k)]);
      for (int i = i0; i < i1; ++i) d.push_back(verA(i, k, k));
      dur[t] = 1.0 + 3.6 * rows;
    } else if (type == T_COLUPD) {
      d.push_back(prodL[tix(j, k + nk - 1)]);
      for (int i = i0; i < i1; ++i) {
        d.push_back(prodL[tix(i, k + nk - 1)]);
        d.push_back(verA(i, j, k));
      }
      dur[t] = 2.0 + (nk > 1 ? 2.6 * nk + 1.0 : 3.6) * rows;
    } else if (type == T_AINV) {
      const int kl = k + nk - 1;
      d.push_back(kl == j ? prodL[tix(j, j)] : prodXd[tix(kl, j)]);
      double steps = 0.0;
      for (int i = i0; i < i1; ++i) {
        d.push_back(kl == i ? prodL[tix(i, i)] : prodXd[tix(kl, i)]);
        const int v0 = std::max(k, i) - i;
        const auto& pv = prodAi[tix(i, j)];
        if (v0 > 0) d.push_back(v0 < (int)pv.size() ? pv[v0] : -1);
        steps += k + nk - std::max(k, i);
      }
      dur[t] = 2.0 + 2.6 * steps + 1.0 * rows;
    } else if (nk > 1) {
      const int kl = k + nk - 1;
      d.push_back(kl == j ? prodL[tix(j, j)] : prodXd[tix(kl, j)]);
      for (int i = i0; i < i1; ++i) {
        d.push_back(prodL[tix(i, kl)]);
        d.push_back(verX(i, j, k - j));
      }
      dur[t] = 2.0 + (2.6 * nk + 1.0) * rows;
    } else {
      if (k == j) d.push_back(prodL[tix(k, k)]);
      else if (fin) { d.push_back(verX(k, j, k - j)); d.push_back(prodL[tix(k, k)]); }
      else d.push_back(prodXd[tix(k, j)]);
      for (int i = i0; i < i1; ++i) {
        d.push_back(prodL[tix(i, k)]);
        d.push_back(verX(i, j, k - j));
      }
      dur[t] = 2.0 + 3.6 * rows + (fin && k > j ? 3.0 : 0.0);
    }
  }
  // bottom levels, dependants first (reverse generation order is reverse topological)
  std::vector<double> succ(n, 0.0), bl(n, 0.0);
  for (int t = n - 1; t >= 0; --t) {
    bl[t] = dur[t] + succ[t];
    for (int dd : deps[t])
      if (dd >= 0 && bl[t] > succ[dd]) succ[dd] = bl[t];
  }
  // A^{-1} tasks (no factorisation task waits on them): by bottom level they
  // would sort behind nearly every factorisation task, i.e. run after the
  // factorisation, serially (measured 2.27 ms for n = 4096 against 2.09 ms as
  // two launches).  ASAP instead: each goes right behind the last of its
  // inputs in the queue (its key just under the smallest input key), so the
  // idle workgroups of the chain-bound stretches pick them up as the X rows
  // become final.  Keys of inputs are final first (generation order is
  // topological).  Opt-in (BO_CHOL_AINV_ASAP=1): measured 2.28 against 2.25 ms
  // with the bottom levels (profiles/r05/ainv_fold/).
  static const bool asap = [] {
    const char* e = getenv("BO_CHOL_AINV_ASAP");
    return e && e[0] == '1';
  }();
  if (asap)
    for (int t = 0; t < n; ++t) {
      if ((v[t].x & 0xff) != T_AINV) continue;
      double key = 1e300;
      for (int dd : deps[t])
        if (dd >= 0) key = std::min(key, bl[dd]);
      if (key < 1e300) bl[t] = key - 1e-6 * (1 + (t % 1000));
    }
  std::vector<int> idx(n);
  for (int t = 0; t < n; ++t) idx[t] = t;
  std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return bl[a] > bl[b]; });
  // the queue must stay topological (a task waits only on tasks claimed
  // before it): check it, and keep the generation order if it is not
  std::vector<int> pos(n);
  for (int t = 0; t < n; ++t) pos[idx[t]] = t;
  for (int t = 0; t < n; ++t)
    for (int dd : deps[t])
      if (dd >= 0 && pos[dd] > pos[t]) return v;
  std::vector<int4> out(n);
  for (int t = 0; t < n; ++t) out[t] = v[idx[t]];
  return out;
}

// ch / chb: tile rows per single-step / batched task -- 2 / 4 for one matrix,
// CH / CHB (8 / 8) for batches: at n = 4096 one matrix ran 1.727-1.733 ms with
// ch 4 against 1.753-1.771 with 8 and 1.91-1.92 with 16, while 4 x 4096 ran
// 5.42-5.45 against 5.38 ms (profiles/r03/cholesky/ab_ch.log); chb 4 then
// 1.709-1.718 against 1.721-1.744 ms for one matrix, but 3 x 2048 0.90 against
// 0.85 ms (ab_chb.log); ch 2 then 1.650-1.684 against 1.684-1.733 ms with 4
// (1: 1.70-1.72, 3: 1.70-1.72; ab_ch23.log, ab_ch21.log): one matrix takes 2 / 4
std::vector<int4> build_tasks(int T, int ch = 2, int chb = 4, bool ainv = false) {
  std::vector<int4> v;
  auto crit = [&](int k) { v.push_back(make_int4(T_CRIT, k, k, 0)); };
  crit(0);
  if (T > 1) crit(1);
  for (int k = 0; k + 1 < T; ++k) {
    push_rows(v, T_TRSM, k, k, k + 2, T, false, ch);
    // the two chunks CRIT(k + 2) waits on: tiles (k+2, k+1) and (k+2, k+2) at step k
    const int c1 = (k + 2 + ch < T) ? k + 2 + ch : T;
    if (k + 2 < T) {
      v.push_back(make_int4(T_COLUPD, k, k + 1, (k + 2) | (c1 << 16)));
      v.push_back(make_int4(T_COLUPD, k, k + 2, (k + 2) | (c1 << 16)));
      crit(k + 2);
    }
    // column j of X at step k: the near rows (k, ke) of the aligned batch
    // [kb, ke) one step at a time (X_kj's finalisation rides on the first
    // chunk, or is a task of its own); at the batch's last step, one batched
    // update of the far rows [ke, T) over all its steps
    for (int j = 0; j <= k; ++j) {
      const int kb = j + ((k - j) / GB) * GB, ke = std::min(kb + GB, T);
      if (k + 1 < ke) push_rows(v, T_XSTEP, k, j, k + 1, ke, true, ch);
      else if (k > j) v.push_back(make_int4(T_XSTEP | 256, k, j, 0));
      if (k == ke - 1 && ke < T) {
        const size_t first = v.size();
        push_rows(v, T_XSTEP, kb, j, ke, T, false, chb);
        for (size_t t = first; t < v.size(); ++t) v[t].x |= (ke - kb) << 16;
      }
    }
    if (k + 2 < T) {
      push_rows(v, T_COLUPD, k, k + 1, c1, T, false, ch);
      push_rows(v, T_COLUPD, k, k + 2, c1, T, false, ch);
    }
    // columns j >= k + 3 at step k: the steps of an aligned batch [kb, kb + GB)
    // that lies wholly at or below j - 3 go in one batched task at the batch's
    // last step (A_ij loaded / stored once per batch); the rest one per step
    for (int j = k + 3; j < T; ++j) {
      const int kb = (k / GB) * GB;
      if (GB > 1 && kb + GB - 1 <= j - 3) {
        if (k == kb + GB - 1) {
          const size_t first = v.size();
          // 2 rows where chunks are 4 (one matrix, small batches): n = 4096
          // 1.659-1.661 -> 1.621-1.638 ms, 3 x 2048 0.786-0.791 -> 0.766-0.769;
          // not with the 8-row chunks of 4096 batches (4 x 4096 5.33 -> 5.38)
          const int dch = diag_chunk_rows() >= 0 ? diag_chunk_rows() : (chb <= 4 ? 2 : 0);
          push_rows(v, T_COLUPD, kb, j, j, T, false, chb, dch);
          for (size_t t = first; t < v.size(); ++t) v[t].x |= GB << 16;
        }
      } else {
        push_rows(v, T_COLUPD, k, j, j, T, false, ch);
      }
    }
  }
  for (int j = 0; j + 1 < T; ++j) v.push_back(make_int4(T_XSTEP | 256, T - 1, j, 0));
  if (ainv) {
    // A^{-1} = X^T X: per aligned batch [kb, ke) of GA rows K of X (final in
    // K order), the tiles (i, j), j <= i <= ke - 1, take their contributions
    // K >= i of the batch; batches in K order, so every tile's contributions
    // arrive in increasing K (a fixed summation order)
    for (int kb = 0; kb < T; kb += GA) {
      const int ke = std::min(kb + GA, T);
      for (int j = 0; j < ke; ++j) {
        const size_t first = v.size();
        push_rows(v, T_AINV, kb, j, j, ke, false, chb);
        for (size_t t = first; t < v.size(); ++t) v[t].x |= (ke - kb) << 16;
      }
    }
  }
  return priority_order(v, T);
}

// nb matrices: the single queue repeated per matrix (id in bits 9-15 of x),
// interleaved task by task.  Each matrix's tasks keep their order, and a task
// only waits on tasks of its own matrix, so every dependency still precedes
// its task in the merged queue.
// Matrix m's queue is offset by m * stagger * (queue length) / nb positions
// (merge key: own position + offset, ties to the lower matrix), so one
// matrix's chain-bound tail overlaps the next one's update-heavy opening
// instead of all matrices opening together.
std::vector<int4> build_tasks_batched(int T, int nb, bool ainv = false) {
  // one matrix, or batches of small ones (n <= 2048: C4's 3 x 2048 0.855-0.867
  // -> 0.797-0.805 ms), take 2 / 4 rows; batches of n = 4096 keep 8 / 8 (with
  // 2 / 4: 4 x 4096 5.38 -> 5.69 ms; profiles/r03/cholesky/ab_ch_batched_small.log)
  // (BO_CHOL_CH / BO_CHOL_CHB override the one-matrix chunk rows: an A/B knob,
  // read once, 1..16).  Round 5 (with the 2-row diagonal-tile first chunk):
  // batched chunks of 3 rows, n = 4096 1.603-1.616 -> 1.598-1.602 ms, 3 x
  // 2048 0.759-0.764 -> 0.751-0.752 ms; 6 rows 1.655-1.663 / 0.825 ms
  // (tools/sweep_chol.sh)
  static const int ch1 = [] {
    const char* e = getenv("BO_CHOL_CH");
    const int v = e ? atoi(e) : 2;
    return v >= 1 && v <= 16 ? v : 2;
  }();
  static const int chb1 = [] {
    const char* e = getenv("BO_CHOL_CHB");
    const int v = e ? atoi(e) : 3;
    return v >= 1 && v <= 16 ? v : 3;
  }();
  const std::vector<int4> one =
      (nb == 1 || T <= 32) ? build_tasks(T, ch1, chb1, ainv) : build_tasks(T, CH, CHB, ainv);
  if (nb == 1) return one;
  double stagger = 0.0;
  if (const char* e = getenv("BO_CHOL_BATCH_STAGGER")) {  // finite values only (sort keys)
    char* end = nullptr;
    const double v = strtod(e, &end);
    if (end != e && std::isfinite(v)) stagger = v;
  }
  const double shift = stagger * (double)one.size() / nb;
  std::vector<std::pair<double, int4>> keyed;
  keyed.reserve(one.size() * nb);
  for (size_t i = 0; i < one.size(); ++i)
    for (int m = 0; m < nb; ++m) {
      const int4& t = one[i];
      keyed.push_back({(double)i + m * shift, make_int4(t.x | (m << 9), t.y, t.z, t.w)});
    }
  std::stable_sort(keyed.begin(), keyed.end(),
                   [](const std::pair<double, int4>& a, const std::pair<double, int4>& b) {
                     return a.first < b.first;
                   });
  std::vector<int4> v;
  v.reserve(keyed.size());
  for (const auto& kv : keyed) v.push_back(kv.second);
  return v;
}

std::mutex g_tab_mu;
std::map<std::tuple<int, int, int, int>, DagTable> g_tabs;  // (device, T, nb, ainv) -> table

int dag_table(int T, DagTable** out, int nb = 1, bool ainv = false) {
  int dev = 0;
  BO_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_tab_mu);
  DagTable& tb = g_tabs[std::make_tuple(dev, T, nb, ainv ? 1 : 0)];
  if (!tb.dev) {
    const std::vector<int4> v = build_tasks_batched(T, nb, ainv);
    int4* d = nullptr;
    BO_HIP(hipMalloc(&d, sizeof(int4) * v.size()));
    BO_HIP(hipMemcpy(d, v.data(), sizeof(int4) * v.size(), hipMemcpyHostToDevice));
    tb.dev = d;
    tb.n = (int)v.size();
  }
  *out = &tb;
  return BO_OK;
}

}  // namespace

// In-place L = chol(A) (lower) and Linv = L^{-1} as one persistent launch, for
// nb matrices stored back to back (np x np each).  np % 64 == 0; work: >=
// (16 + 4 nb (np/64)^2) * 4 bytes of scratch for the counters; info[m] as in
// bo_cholesky_inverse (-1: the task DAG timed out).
int bo_chol_dag(double* A, double* Linv, int64_t np, int* info, void* work, hipStream_t st,
                long long* trace, int nb, double* Ainv) {
  BO_CHECK_ARG(np > 0 && np % TB == 0 && np <= 16384, "bo_chol_dag: order %lld", (long long)np);
  BO_CHECK_ARG(nb >= 1 && nb <= 128 && (trace == nullptr || nb == 1),
               "bo_chol_dag: batch %d (1..128; traced launches single)", nb);
  BO_CHECK_ARG(Ainv == nullptr || nb == 1, "bo_chol_dag: A^{-1} tasks take one matrix");
  const int T = (int)(np / TB);
  DagTable* tb = nullptr;
  int s = dag_table(T, &tb, nb, Ainv != nullptr);
  if (s) return s;
  int dev = 0, cus = 0;
  BO_HIP(hipGetDevice(&dev));
  BO_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const size_t fbytes =
      ((size_t)(NFLAG0 + (size_t)nb * (Ainv ? 5 : 4) * T * T) * 4 + 15) / 16 * 16;
  BO_HIP(hipMemsetAsync(work, 0, fbytes, st));
  BO_HIP(hipMemsetAsync(info, 0, sizeof(int) * nb, st));
  // BO_CHOL_ZERO_IN_DAG=0: memset Linv ahead of the launch instead (A/B knob)
  static const int zero_in = [] {
    const char* e = getenv("BO_CHOL_ZERO_IN_DAG");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  if (!zero_in) BO_HIP(hipMemsetAsync(Linv, 0, sizeof(double) * np * np * nb, st));
  // one workgroup per CU: two per CU (74 KB of LDS each fits) measured slower,
  // 2.35 -> 2.97 ms at n = 4096 -- the sc1 tile traffic, not latency, is the limit
  const int grid = cus < tb->n ? cus : tb->n;
  if (zero_in && grid <= 8) BO_HIP(hipMemsetAsync(Linv, 0, sizeof(double) * np * np * nb, st));
  // BO_CHOL_PREFETCH2 (default 1): batched updates prefetch two steps ahead
  static const int pf2 = [] {
    const char* e = getenv("BO_CHOL_PREFETCH2");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  chol_dag_kernel<<<grid, 256, 0, st>>>(A, Linv, (int)np, T, tb->dev, tb->n, (u32*)work, info,
                                          trace, nb, pf2, Ainv, zero_in && grid > 8 ? 1 : 0);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

// Timing probe of the task DAG (tools/trace_chol.py): trace receives, per task
// in queue order, [start, end, packed (block, type, k, j)] in wall-clock ticks
// (100 MHz); returns the task count through *ntasks (host int).
#ifdef BO_TOOLS  // development probes (tools/bo_tools.h), not the product ABI
extern "C" int bo_probe_chol_dag(double* A, double* Linv, int64_t np, int* info, void* work,
                                 long long* trace, int* ntasks, void* stream) {
  BO_CHECK_ARG(np > 0 && np % TB == 0, "bo_probe_chol_dag: order");
  DagTable* tb = nullptr;
  int s = dag_table((int)(np / TB), &tb);
  if (s) return s;
  *ntasks = tb->n;
  return bo_chol_dag(A, Linv, np, info, work, as_stream(stream), trace, 1, nullptr);
}

// One workgroup factors + inverts the 64 x 64 SPD matrix A (row-major) reps
// times in LDS with the diagonal-tile routine of the DAG (variant 1: column
// owners, 0: four panels); out = [L | D] (2 x 4096), ct[8] = the phase stamps
// of the last rep, ct[8] = total wall-clock ticks of all reps.
__global__ __launch_bounds__(256) void potrf64_probe_kernel(const double* A, double* out, long long* ct,
                                                            int* info, int variant, int reps) {
  __shared__ __attribute__((aligned(16))) double S[TB * LP];
  __shared__ __attribute__((aligned(16))) double D[TB * LP];
  __shared__ __attribute__((aligned(16))) double Lc[TB * LP];
  __shared__ __attribute__((aligned(16))) double Tsc[TB * LP];
  __shared__ double rinv[TB];
  __shared__ double Lcol[512];
  __shared__ int s_cnt;
  __shared__ int s_fail[4];
  __shared__ int s_fl[4];
  Ctx c;
  c.np = 64; c.tid = threadIdx.x; c.lane = c.tid & 63; c.wave = c.tid >> 6;
  c.wm = (c.wave >> 1) * 32; c.wn = (c.wave & 1) * 32;
  const long long t0 = wall_clock64();
  for (int it = 0; it < reps; ++it) {
    for (int e = c.tid; e < 4096; e += 256) S[(e >> 6) * LP + (e & 63)] = A[e];
    __syncthreads();
    if (c.tid == 0) ct[0] = wall_clock64();
    lds_cnt_t* cn = (lds_cnt_t*)&s_cnt;
    lds_cnt_t* fl = (lds_cnt_t*)s_fl;
    if (variant == 1) potrf_trtri64_cols<0>(c, S, D, rinv, info, 0, Lc, Tsc, cn, s_fail, fl, ct);
    else if (variant == 2) potrf_trtri64_cols<1>(c, S, D, rinv, info, 0, Lc, Tsc, cn, s_fail, fl, ct);
    else if (variant == 3) potrf_trtri64_cols<2>(c, S, D, rinv, info, 0, Lc, Tsc, cn, s_fail, fl, ct);
    else if (variant == 4) potrf_trtri64_cols<3>(c, S, D, rinv, info, 0, Lc, Tsc, cn, s_fail, fl, ct);
    else potrf_trtri64(c, S, D, rinv, info, 0, Lcol, cn, ct);
    if (c.tid == 0) ct[1] = wall_clock64();
    __syncthreads();
  }
  if (c.tid == 0) ct[8] = wall_clock64() - t0;
  for (int e = c.tid; e < 4096; e += 256) {
    out[e] = S[(e >> 6) * LP + (e & 63)];
    out[4096 + e] = D[(e >> 6) * LP + (e & 63)];
  }
}

extern "C" int bo_probe_potrf64(const double* A, double* out, long long* ct, int* info, int variant,
                                int reps, void* stream) {
  potrf64_probe_kernel<<<1, 256, 0, as_stream(stream)>>>(A, out, ct, info, variant, reps);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

// Cycles (s_memtime ticks) per 16 x 16 diagonal factor + inverse on one wave:
// out[0] DPP broadcasts, out[1] readlane broadcasts, out[2] DPP, factor only.
extern "C" int bo_probe_diag16(long long* out, double* sink, void* stream) {
  hipStream_t st = as_stream(stream);
  diag16_probe_kernel<0><<<1, 64, 0, st>>>(256, out, sink);
  diag16_probe_kernel<1><<<1, 64, 0, st>>>(256, out, sink);
  diag16_probe_kernel<2><<<1, 64, 0, st>>>(256, out, sink);
  BO_LAUNCH_CHECK();
  return BO_OK;
}
#endif  // BO_TOOLS

// The queue of the task DAG for T tile rows (host only, no device call): out
// receives 4 ints per task (type | fin << 8 | nk << 16, k, j, i0 | i1 << 16) in queue
// order, up to cap tasks; returns the task count (tests/test_chol_dag_cpu.py
// checks that every dependency precedes its task).
static int dag_tasks_out(const std::vector<int4>& v, int* out, int cap) {
  const int n = (int)v.size();
  for (int t = 0; t < n && t < cap; ++t) {
    out[4 * t] = v[t].x;
    out[4 * t + 1] = v[t].y;
    out[4 * t + 2] = v[t].z;
    out[4 * t + 3] = v[t].w;
  }
  return n;
}

extern "C" int bo_chol_dag_tasks_ainv(int T, int* out, int cap) {
  if (T < 1) return 0;
  return dag_tasks_out(build_tasks(T, 2, 4, true), out, cap);
}

extern "C" int bo_chol_dag_tasks(int T, int* out, int cap) {
  if (T < 1) return 0;
  // the queue one matrix's launch runs (bo_chol_dag: build_tasks_batched)
  const std::vector<int4> v = build_tasks_batched(T, 1);
  const int n = (int)v.size();
  for (int t = 0; t < n && t < cap; ++t) {
    out[4 * t] = v[t].x;
    out[4 * t + 1] = v[t].y;
    out[4 * t + 2] = v[t].z;
    out[4 * t + 3] = v[t].w;
  }
  return n;
}
