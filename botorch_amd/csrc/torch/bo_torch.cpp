// PyTorch-ROCm operators of the fused MC-acquisition forward, in C++.
//
// the hot path is bound as PyTorch custom ops registered with
// TORCH_LIBRARY.  One call of bo::qmc_acq_native issues the whole fused qEI /
// qLogEI / posterior chain of acquisition/monte_carlo.py:253-289 (+ logei.py:
// 137-234) for B t-batches -- rows prepared, K*x^T built, the R = K*x L^-T
// contraction with its R R^T / R beta epilogue, the per-t-batch finalisation
// with the jitter ladder and the MC reduction, and (with need_grad) the
// backward's W^T -- on the caller's current HIP stream, with the buffers from
// torch's caching allocator and no Python between the launches.  The kernels
// are the C ABI of include/botorch_amd.h (libbotorch_amd.so); this library
// adds only the host sequence, so the ctypes binding (botorch_amd/_lib.py)
// and these ops drive the same code.
//
// The jitter-ladder status of a forward-only call is deferred, as [G]
// psd_safe_cholesky's host check would otherwise synchronise every call: the
// status is reduced on the device into pinned host memory behind an event, and
// read once that event has passed (a later call's query, or the driver's own
// sync, bo::ladder_poll) -- a ring of slots per device, so a call waits on an
// older one only when the whole ring is in flight.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <torch/library.h>

#include <algorithm>
#include <array>
#include <deque>
#include <atomic>
#include <mutex>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../../include/botorch_amd.h"

namespace {

void ck(int rc, const char* what) {
  TORCH_CHECK(rc == BO_OK, "botorch_amd ", what, ": ", bo_last_error());
}
void hk(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "botorch_amd ", what, ": ", hipGetErrorString(e));
}
const double* cp(const at::Tensor& t) { return t.defined() && t.numel() ? t.data_ptr<double>() : nullptr; }
double* mp(const at::Tensor& t) { return t.defined() && t.numel() ? t.data_ptr<double>() : nullptr; }

void check_f64(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "bo::qmc_acq_native: ", name, " must be a ROCm device tensor");
  TORCH_CHECK(t.scalar_type() == at::kDouble, "bo::qmc_acq_native: ", name, " must be fp64");
  TORCH_CHECK(t.is_contiguous(), "bo::qmc_acq_native: ", name, " must be contiguous");
}

// ---- deferred ladder status ---------------------------------------------------------
// A ring of NSLOT status slots per device.  A call enqueues its status into a
// free slot behind an event and returns what the FINISHED calls reported
// (event queries, no wait); it waits only when every slot is in flight, so the
// host keeps issuing while the GPU runs (a failed root is reported within
// NSLOT calls, or at bo::ladder_poll, which waits for all of them).
constexpr int NSLOT = 4;
constexpr int SLOT_MEMBERS = 8;       // a ModelListGP's members (qehvi_members_eager)
constexpr int SLOT_WORDS = 2 + 2 * SLOT_MEMBERS;
struct Slot {
  // pinned [info_max, jitter_max], then one such pair per ModelListGP member
  // (bo::qehvi_members_eager folds each member's ladder into its own pair:
  // one pair for all would race between the members' last workgroups)
  double* host = nullptr;
  double* host_dev = nullptr;  // the same pinned words as a device pointer (zero-copy)
  double* dev = nullptr;    // device [info_max, jitter_max]
  int* count = nullptr;     // arrival counters of the fused status (qmc_kernel re-zeroes them)
  hipEvent_t ev = nullptr;
  bool busy = false;
};
struct DeviceLadder {
  std::array<Slot, NSLOT> slot;
  std::deque<int> pending;  // slots in flight, oldest first
};
std::mutex g_ladder_mu;
std::unordered_map<int, DeviceLadder> g_ladder;

DeviceLadder& ladder_for(int dev) {
  auto& L = g_ladder[dev];
  if (!L.slot[0].host) {
    for (auto& s : L.slot) {
      hk(hipHostMalloc(reinterpret_cast<void**>(&s.host), SLOT_WORDS * sizeof(double),
                       hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
      for (int e = 0; e < SLOT_WORDS; ++e) s.host[e] = 0.0;
      hk(hipHostGetDevicePointer(reinterpret_cast<void**>(&s.host_dev), s.host, 0),
         "hipHostGetDevicePointer");
      hk(hipMalloc(reinterpret_cast<void**>(&s.dev), 2 * sizeof(double)), "hipMalloc");
      hk(hipMalloc(reinterpret_cast<void**>(&s.count), (1 + SLOT_MEMBERS) * sizeof(int)), "hipMalloc");
      hk(hipMemset(s.count, 0, (1 + SLOT_MEMBERS) * sizeof(int)), "hipMemset");
      hk(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming), "hipEventCreate");
    }
  }
  return L;
}

// Fold the oldest pending slot into out = [has, info_max, jitter_max] and free it.
void fold_front(DeviceLadder& L, double* o) {
  Slot& s = L.slot[L.pending.front()];
  o[0] = 1.0;
  for (int e = 0; e < SLOT_WORDS; e += 2) {  // the call's own pair and its members'
    o[1] = std::max(o[1], s.host[e]);
    o[2] = std::max(o[2], s.host[e + 1]);
  }
  s.busy = false;
  L.pending.pop_front();
}

// [has_status, info_max, jitter_max] over the finished calls (all pending ones
// with wait_all), freeing their slots.  Caller holds g_ladder_mu.
at::Tensor take_pending(DeviceLadder& L, bool wait_all) {
  auto out = at::zeros({3}, at::TensorOptions().dtype(at::kDouble));
  auto* o = out.data_ptr<double>();
  while (!L.pending.empty()) {
    Slot& s = L.slot[L.pending.front()];
    if (wait_all) {
      hk(hipEventSynchronize(s.ev), "hipEventSynchronize");
    } else {
      const hipError_t q = hipEventQuery(s.ev);
      if (q == hipErrorNotReady) break;
      hk(q, "hipEventQuery");
    }
    fold_front(L, o);
  }
  return out;
}

// The slot this call's status goes to: a free one, after waiting for the
// oldest call when all are in flight (folded into *prev).  Caller holds
// g_ladder_mu until publish_slot.
int free_slot(DeviceLadder& L, at::Tensor& prev) {
  prev = take_pending(L, false);
  if ((int)L.pending.size() == NSLOT) {
    hk(hipEventSynchronize(L.slot[L.pending.front()].ev), "hipEventSynchronize");
    fold_front(L, prev.data_ptr<double>());
  }
  for (int i = 0; i < NSLOT; ++i)
    if (!L.slot[i].busy) {
      // qmc_kernel folds its status into the words it finds (sticky max)
      for (int e = 0; e < SLOT_WORDS; ++e) L.slot[i].host[e] = 0.0;
      return i;
    }
  TORCH_CHECK(false, "botorch_amd: no free ladder-status slot");
}

// Copy the slot's device status to its pinned host words (unless the kernel
// wrote them there itself: zero_copy) behind an event; it joins the pending
// ring.  Caller holds g_ladder_mu.
void publish_slot(DeviceLadder& L, int mine, void* stream, bool zero_copy = false) {
  Slot& s = L.slot[mine];
  if (!zero_copy)
    hk(hipMemcpyAsync(s.host, s.dev, 2 * sizeof(double), hipMemcpyDeviceToHost,
                      static_cast<hipStream_t>(stream)), "hipMemcpyAsync");
  hk(hipEventRecord(s.ev, static_cast<hipStream_t>(stream)), "hipEventRecord");
  s.busy = true;
  L.pending.push_back(mine);
}

// Enqueue this call's status (bo_ladder_status over info / jitter) into a free
// slot; return the finished calls' statuses.
at::Tensor defer_status(const at::Tensor& info, const at::Tensor& jitter, void* stream, int dev) {
  std::lock_guard<std::mutex> lk(g_ladder_mu);
  auto& L = ladder_for(dev);
  at::Tensor prev;
  const int mine = free_slot(L, prev);
  ck(bo_ladder_status(info.data_ptr<int>(), jitter.data_ptr<double>(), info.numel(),
                      L.slot[mine].dev, stream), "ladder_status");
  publish_slot(L, mine, stream);
  return prev;
}

// ---- post_partials launch timing (bench.py: HIP events around the launch) ------------
std::mutex g_time_mu;
bool g_time_on = false;
std::vector<std::pair<hipEvent_t, hipEvent_t>> g_time_ev;

hipEvent_t timing_event(void* stream) {
  hipEvent_t e;
  hk(hipEventCreate(&e), "hipEventCreate");
  hk(hipEventRecord(e, static_cast<hipStream_t>(stream)), "hipEventRecord");
  return e;
}

// ---- the fused forward ------------------------------------------------------------------
// The fused forward.  lean (bo::qmc_acq_eager, forward-only eager calls):
// every intermediate (rows, K*x^T, partials, split-k workspace, ladder
// entries) is carved from ONE allocation and only [acq, previous status] is
// returned -- each at::empty costs host time on the critical path of small
// calls (C2: ~70 us of host issue per call against ~45 us of kernels).
std::vector<at::Tensor> qmc_acq_impl(
    const at::Tensor& X, const at::Tensor& Xt_scaled, const at::Tensor& U, const at::Tensor& Linv,
    const at::Tensor& beta, const at::Tensor& lengthscale, const at::Tensor& Z,
    const c10::optional<at::Tensor>& best_f_s, int64_t kind, int64_t mode, int64_t n,
    double outputscale, double constant, double ymean, double ystd, double best_f, bool fat,
    double tau_relu, double tau_max, bool need_grad, int64_t kxt_cap, bool defer_ladder,
    const c10::optional<at::Tensor>& Ainv, const c10::optional<at::Tensor>& alpha, bool lean,
    const c10::optional<at::Tensor>& cap_status = c10::nullopt,
    const c10::optional<at::Tensor>& cap_count = c10::nullopt) {
  check_f64(X, "X");
  check_f64(Xt_scaled, "Xt_scaled");
  check_f64(U, "U");
  check_f64(beta, "beta");
  check_f64(lengthscale, "lengthscale");
  check_f64(Z, "Z");
  TORCH_CHECK(X.dim() == 3, "bo::qmc_acq_native: X must be B x q x d");
  const int B = static_cast<int>(X.size(0)), q = static_cast<int>(X.size(1)),
            d = static_cast<int>(X.size(2));
  TORCH_CHECK(Xt_scaled.size(0) == n && lengthscale.numel() == d,
              "bo::qmc_acq_native: model and X disagree (n, d)");
  TORCH_CHECK(Z.dim() == 2 && Z.size(1) == q, "bo::qmc_acq_native: Z must be S x q");
  TORCH_CHECK(!(lean && need_grad), "bo::qmc_acq_eager is forward-only");
  if (need_grad) check_f64(Linv, "Linv");
  const int dev = X.device().index();
  void* st = c10::hip::getCurrentHIPStream(dev).stream();
  auto f64 = X.options().dtype(at::kDouble);
  const int64_t np = U.size(0);

  int Qp = 0, nrows = 0, nC = 0;
  ck(bo_post_geometry(B, q, n, &Qp, &nrows, &nC), "post_geometry");
  const bool kxt = np * int64_t(nrows) * 8 <= kxt_cap;
  // forward-only small grids: the quad plan over the cached A^{-1} (quad.hip)
  int npairs = 0;
  const bool quad_operands = !need_grad && kxt && Ainv.has_value() && Ainv->defined() &&
                             alpha.has_value() && alpha->defined();
  if (quad_operands) {
    check_f64(*Ainv, "Ainv");
    check_f64(*alpha, "alpha");
    TORCH_CHECK(Ainv->size(0) == np && Ainv->size(1) == np, "bo::qmc_acq_native: Ainv must be np x np");
    ck(bo_post_quad_plan(B, q, n, &npairs), "post_quad_plan");
  }
  // small grids: equal 32-row units over column-tile pairs (post_small_kernel),
  // no split-k workspace or reduction launch; with need_grad it also stores
  // R^T row-major for the backward's W^T routes
  int nsmall = 0;
  if (kxt && npairs == 0) ck(bo_post_small_plan(B, q, n, &nsmall), "post_small_plan");
  const int nparts = npairs > 0 ? npairs : (nsmall > 0 ? nsmall : nC);
  int kc = 0;
  int64_t we = 0;
  if (npairs == 0 && nsmall == 0) ck(bo_post_split_plan(B, q, n, 0, &kc, &we), "post_split_plan");

  // one workspace for the intermediates (offsets in doubles, 16-B aligned)
  auto al2 = [](int64_t v) { return (v + 1) & ~int64_t(1); };
  const bool own_xq = need_grad;  // the backward keeps Xq
  const int64_t o_spart = 0;
  const int64_t o_mpart = o_spart + al2(int64_t(nparts) * nrows * 16);
  const int64_t o_kt = o_mpart + al2(int64_t(nparts) * nrows);
  const int64_t o_work = o_kt + (kxt ? al2(np * nrows) : 0);
  const int64_t o_xq = o_work + (kc ? al2(std::max<int64_t>(we, 1)) : 0);
  const int64_t o_info = o_xq + (own_xq ? 0 : al2(int64_t(nrows) * 8));
  const int64_t o_jit = o_info + (lean ? al2((B + 1) / 2) : 0);
  const int64_t total = o_jit + (lean ? al2(B) : 0);
  auto ws = at::empty({std::max<int64_t>(total, 2)}, f64);
  double* w = ws.data_ptr<double>();
  double* Spart = w + o_spart;
  double* mpart = w + o_mpart;
  double* Kt = kxt ? w + o_kt : nullptr;
  double* work = kc ? w + o_work : nullptr;
  at::Tensor Xq_t = own_xq ? at::empty({nrows, 8}, f64) : at::Tensor();
  double* Xq = own_xq ? Xq_t.data_ptr<double>() : w + o_xq;
  at::Tensor Rt = need_grad ? at::empty({int64_t(nC) * 128, nrows}, f64) : at::Tensor();
  int rt_layout = BO_RT_ROWMAJOR;

  if (kxt) {  // rows and K*x^T in one launch
    ck(bo_post_kxt_rows(int(kind), X.data_ptr<double>(), B, q, d, lengthscale.data_ptr<double>(),
                        Xt_scaled.data_ptr<double>(), n, outputscale, Xq, Kt, st), "post_kxt_rows");
  } else {
    ck(bo_prepare_rows(X.data_ptr<double>(), B, q, d, lengthscale.data_ptr<double>(), Xq, st),
       "prepare_rows");
  }
  hipEvent_t t0 = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_time_mu);
    if (g_time_on) t0 = timing_event(st);
  }
  if (npairs > 0) {
    ck(bo_post_quad(Kt, Ainv->data_ptr<double>(), np, alpha->data_ptr<double>(), B, q, n, Spart,
                    mpart, st), "post_quad");
  } else if (nsmall > 0) {
    ck(bo_post_small(Kt, B, q, n, U.data_ptr<double>(), np, beta.data_ptr<double>(), Spart, mpart,
                     mp(Rt), st), "post_small");
  } else {
    BoPostPartialsArgs pa{};
    pa.struct_size = sizeof(pa);
    pa.abi_version = BO_ABI_VERSION;
    pa.kind = int(kind);
    pa.B = B;
    pa.q = q;
    pa.d = d;
    pa.Xq = Xq;
    pa.Xt_scaled = Xt_scaled.data_ptr<double>();
    pa.n = n;
    pa.U = U.data_ptr<double>();
    pa.ldu = np;
    pa.beta = beta.data_ptr<double>();
    pa.outputscale = outputscale;
    pa.Spart = Spart;
    pa.mpart = mpart;
    pa.Rt = mp(Rt);
    pa.kc_len = kc;
    pa.work = work;
    pa.Kt = Kt;
    if (need_grad) {
      // the backward reads R^T in the blocked layout where its fused W -> dX
      // pass applies (bo_post_w_dx), row-major everywhere else
      int64_t wdx = 0;
      ck(bo_post_w_dx_work(B, q, n, &wdx), "post_w_dx_work");
      rt_layout = (wdx > 0 && kc == 0) ? BO_RT_BLOCKED : BO_RT_ROWMAJOR;
      pa.rt_layout = rt_layout;
    }
    ck(bo_post_partials_v(&pa, st), "post_partials");
  }
  if (t0) {
    std::lock_guard<std::mutex> lk(g_time_mu);
    g_time_ev.emplace_back(t0, timing_event(st));
  }

  auto acq = at::empty({B}, f64);
  at::Tensor info, jit;
  if (!lean) {
    info = at::empty({B}, X.options().dtype(at::kInt));
    jit = at::empty({B}, f64);
  }
  int* info_p = lean ? reinterpret_cast<int*>(w + o_info) : info.data_ptr<int>();
  double* jit_p = lean ? w + o_jit : jit.data_ptr<double>();
  at::Tensor mean = need_grad ? at::empty({B, q}, f64) : at::Tensor();
  at::Tensor L = need_grad ? at::empty({B, q, q}, f64) : at::Tensor();
  const at::Tensor bfs = best_f_s.has_value() ? best_f_s->contiguous() : at::Tensor();
  BoQmcFinalizeArgs fa{};
  fa.struct_size = sizeof(fa);
  fa.abi_version = BO_ABI_VERSION;
  fa.kind = int(kind);
  fa.mode = int(mode);
  fa.B = B;
  fa.q = q;
  fa.Xq = Xq;
  fa.Spart = Spart;
  fa.mpart = mpart;
  fa.n = n;
  fa.outputscale = outputscale;
  fa.constant = constant;
  fa.ymean = ymean;
  fa.ystd = ystd;
  fa.Z = Z.data_ptr<double>();
  fa.S = static_cast<int32_t>(Z.size(0));
  fa.max_tries = 6;        // botorch/__init__.py:47 (cholesky_max_tries)
  fa.best_f = best_f;
  fa.best_f_s = cp(bfs);
  fa.jitter0 = 1e-8;       // [G] cholesky_jitter, double
  fa.acq = acq.data_ptr<double>();
  fa.mean_out = mp(mean);
  fa.L_out = mp(L);
  fa.info_out = info_p;
  fa.jitter_out = jit_p;
  fa.fat = fat ? 1 : 0;
  fa.tau_relu = tau_relu;
  fa.tau_max = tau_max;
  fa.nparts = npairs > 0 ? npairs : nsmall;
  fa.sym_parts = npairs > 0 ? 1 : 0;

  // (the backward's W = R L^-1 is formed by qmc_acq_backward_native, fused
  // into its dX reduction where the grid allows: nothing of it is stored here)
  at::Tensor prev;
  const bool cap = cap_status.has_value() && cap_status->defined();
  if (cap && B > 0 && mode != BO_QMC_POSTERIOR) {
    // a forward under HIP-graph capture (graphs.GraphedAcquisition): the
    // finalisation folds its ladder status straight into the graph's own
    // pinned words (sticky max over the replays) -- no status kernel, copy
    // or host bookkeeping among the captured nodes
    TORCH_CHECK(cap_count.has_value() && cap_count->defined() && cap_count->is_cuda() &&
                    cap_count->scalar_type() == at::kInt && cap_status->numel() == 2 &&
                    cap_status->scalar_type() == at::kDouble,
                "bo::qmc_acq_eager: cap_status (2 pinned doubles) needs cap_count (1 device int)");
    double* hd = nullptr;
    hk(hipHostGetDevicePointer(reinterpret_cast<void**>(&hd), cap_status->data_ptr<double>(), 0),
       "hipHostGetDevicePointer");
    fa.status_out = hd;
    fa.status_count = cap_count->data_ptr<int>();
    ck(bo_qmc_finalize_v(&fa, st), "qmc_finalize");
    prev = at::zeros({3}, at::TensorOptions().dtype(at::kDouble));
  } else if (defer_ladder && B > 0 && mode != BO_QMC_POSTERIOR) {
    // the ladder status reduced by the finalisation launch itself (its last
    // workgroup) straight into this call's pinned slot (zero-copy: no copy
    // launch), read behind an event one call later
    std::lock_guard<std::mutex> lk(g_ladder_mu);
    auto& Ld = ladder_for(dev);
    const int mine = free_slot(Ld, prev);
    fa.status_out = Ld.slot[mine].host_dev;
    fa.status_count = Ld.slot[mine].count;
    ck(bo_qmc_finalize_v(&fa, st), "qmc_finalize");
    publish_slot(Ld, mine, st, true);
  } else {
    ck(bo_qmc_finalize_v(&fa, st), "qmc_finalize");
    TORCH_CHECK(!(lean && defer_ladder && B > 0), "bo::qmc_acq_eager: posterior mode has no status");
    prev = (defer_ladder && B > 0) ? defer_status(info, jit, st, dev)
                                   : at::zeros({3}, at::TensorOptions().dtype(at::kDouble));
  }
  if (lean) return {acq, prev};
  auto empty = [&]() { return at::empty({0}, f64); };
  return {acq,
          need_grad ? mean : empty(),
          need_grad ? L : empty(),
          need_grad ? Xq_t : empty(),
          // the layout travels with the tensor: a blocked R^T is returned as
          // [column blocks][row blocks][256], a row-major one as [columns][rows]
          need_grad ? (rt_layout == BO_RT_BLOCKED ? Rt.view({int64_t(nC) * 8, nrows / 16, 256}) : Rt)
                    : empty(),
          empty(),
          jit,
          info,
          prev};
}

std::vector<at::Tensor> qmc_acq_native(
    const at::Tensor& X, const at::Tensor& Xt_scaled, const at::Tensor& U, const at::Tensor& Linv,
    const at::Tensor& beta, const at::Tensor& lengthscale, const at::Tensor& Z,
    const c10::optional<at::Tensor>& best_f_s, int64_t kind, int64_t mode, int64_t n,
    double outputscale, double constant, double ymean, double ystd, double best_f, bool fat,
    double tau_relu, double tau_max, bool need_grad, int64_t kxt_cap, bool defer_ladder,
    const c10::optional<at::Tensor>& Ainv, const c10::optional<at::Tensor>& alpha) {
  return qmc_acq_impl(X, Xt_scaled, U, Linv, beta, lengthscale, Z, best_f_s, kind, mode, n,
                      outputscale, constant, ymean, ystd, best_f, fat, tau_relu, tau_max, need_grad,
                      kxt_cap, defer_ladder, Ainv, alpha, false);
}

// Forward-only eager calls: [acq, previous deferred status [has, info_max, jitter_max]].
std::vector<at::Tensor> qmc_acq_eager(
    const at::Tensor& X, const at::Tensor& Xt_scaled, const at::Tensor& U,
    const at::Tensor& beta, const at::Tensor& lengthscale, const at::Tensor& Z,
    const c10::optional<at::Tensor>& best_f_s, int64_t kind, int64_t mode, int64_t n,
    double outputscale, double constant, double ymean, double ystd, double best_f, bool fat,
    double tau_relu, double tau_max, int64_t kxt_cap, const c10::optional<at::Tensor>& Ainv,
    const c10::optional<at::Tensor>& alpha, const c10::optional<at::Tensor>& cap_status,
    const c10::optional<at::Tensor>& cap_count) {
  return qmc_acq_impl(X, Xt_scaled, U, U, beta, lengthscale, Z, best_f_s, kind, mode, n,
                      outputscale, constant, ymean, ystd, best_f, fat, tau_relu, tau_max, false,
                      kxt_cap, true, Ainv, alpha, true, cap_status, cap_count);
}

// Two coherent, device-mapped pinned doubles, zeroed: a captured graph's
// ladder-status words (bo::qmc_acq_eager's cap_status).
at::Tensor pinned_status() {
  double* h = nullptr;
  hk(hipHostMalloc(reinterpret_cast<void**>(&h), 2 * sizeof(double),
                   hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
  h[0] = 0.0;
  h[1] = 0.0;
  return at::from_blob(h, {2}, [](void* p) { (void)hipHostFree(p); },
                       at::TensorOptions().dtype(at::kDouble));
}

// The posterior-backward route the last qmc_acq_backward_native call took
// (bo::last_backward_route; tests assert the config-size gradient goes
// through the fused pass).
enum { BO_ROUTE_NONE = 0, BO_ROUTE_W_DX = 1, BO_ROUTE_W_SPLIT = 2, BO_ROUTE_W_GEMM = 3 };
std::atomic<int> g_last_route{BO_ROUTE_NONE};

int64_t last_backward_route() { return g_last_route.load(); }

// dX of qmc_acq_native (the registered autograd formula of bo::qmc_acq): the
// reduction + sampling + q x q Cholesky backward (bo_qmc_backward), then the
// posterior backward -- W = R L^-1 formed tile by tile and reduced into dX in
// the same launch (bo_post_w_dx) where the one-pass grid applies, else W^T by
// the stream-K / structured-GEMM route and bo_post_backward.
at::Tensor qmc_acq_backward_native(
    const at::Tensor& dacq, const at::Tensor& acq, const at::Tensor& mean, const at::Tensor& L,
    const at::Tensor& Z, const c10::optional<at::Tensor>& best_f_s, const at::Tensor& Xq,
    const at::Tensor& Rt, const at::Tensor& Linv, const at::Tensor& U, const at::Tensor& Xt_scaled,
    const at::Tensor& alpha, const at::Tensor& lengthscale, int64_t kind, int64_t mode, int64_t d,
    int64_t n, double outputscale, double ystd, double best_f, bool fat, double tau_relu,
    double tau_max) {
  for (const auto* t : {&mean, &L, &Z, &Xq, &Rt, &Linv, &U, &Xt_scaled, &alpha, &lengthscale})
    check_f64(*t, "backward operand");
  const int B = static_cast<int>(mean.size(0)), q = static_cast<int>(mean.size(1));
  const int dev = mean.device().index();
  void* st = c10::hip::getCurrentHIPStream(dev).stream();
  auto f64 = mean.options();
  const int64_t np = U.size(0);
  auto dX = at::empty({B, q, d}, f64);
  if (B == 0) return dX;
  auto dmean = at::empty({B, q}, f64);
  auto dcov = at::empty({B, q, q}, f64);
  const at::Tensor da = dacq.to(at::kDouble).contiguous();
  const at::Tensor af = acq.contiguous();
  const at::Tensor bfs = best_f_s.has_value() ? best_f_s->contiguous() : at::Tensor();
  BoQmcBackwardArgs qa{};
  qa.struct_size = sizeof(qa);
  qa.abi_version = BO_ABI_VERSION;
  qa.mode = int(mode);
  qa.B = B;
  qa.q = q;
  qa.S = static_cast<int32_t>(Z.size(0));
  qa.mean = mean.data_ptr<double>();
  qa.Lq = L.data_ptr<double>();
  qa.Z = Z.data_ptr<double>();
  qa.best_f = best_f;
  qa.best_f_s = cp(bfs);
  qa.dacq = da.data_ptr<double>();
  qa.dmean = dmean.data_ptr<double>();
  qa.dcov = dcov.data_ptr<double>();
  qa.acq_fwd = af.data_ptr<double>();
  qa.fat = fat ? 1 : 0;
  qa.tau_relu = tau_relu;
  qa.tau_max = tau_max;
  ck(bo_qmc_backward_v(&qa, st), "qmc_backward");

  // R^T's layout is the forward's decision, carried by its shape: blocked
  // (3-d) R^T is read only by the fused W -> dX pass, row-major (2-d) R^T
  // only by the W^T routes below
  const bool rt_blocked = Rt.dim() == 3;
  TORCH_CHECK(Rt.dim() == 2 || rt_blocked, "bo::qmc_acq_backward_native: R^T must be 2-d or blocked 3-d");
  int64_t wdx = 0;
  ck(bo_post_w_dx_work(B, q, n, &wdx), "post_w_dx_work");
  TORCH_CHECK(!rt_blocked || wdx > 0,
              "bo::qmc_acq_backward_native: blocked R^T but the fused W -> dX grid does not apply "
              "to (B, q, n) = (", B, ", ", q, ", ", n, ")");
  if (rt_blocked) {
    g_last_route.store(BO_ROUTE_W_DX);
    auto work = at::empty({wdx}, f64);
    ck(bo_post_w_dx(int(kind), Linv.data_ptr<double>(), np, Rt.data_ptr<double>(), B, q, int(d), n,
                    Xq.data_ptr<double>(), Xt_scaled.data_ptr<double>(), alpha.data_ptr<double>(),
                    dmean.data_ptr<double>(), dcov.data_ptr<double>(),
                    lengthscale.data_ptr<double>(), outputscale, ystd, work.data_ptr<double>(),
                    dX.data_ptr<double>(), st), "post_w_dx");
    return dX;
  }
  int Qp = 0, nrows = 0, nC = 0;
  ck(bo_post_geometry(B, q, n, &Qp, &nrows, &nC), "post_geometry");
  int wkc = 0;
  int64_t wwe = 0;
  ck(bo_post_w_work(B, q, n, &wkc, &wwe), "post_w_work");
  at::Tensor W;
  bool kmajor = true;
  g_last_route.store(wkc == -1 ? BO_ROUTE_W_SPLIT : BO_ROUTE_W_GEMM);
  if (wkc == -1) {
    W = at::empty({np, nrows}, f64);
    auto ww = at::empty({std::max<int64_t>(wwe, 1)}, f64);
    ck(bo_post_w_split(Linv.data_ptr<double>(), np, Rt.data_ptr<double>(), B, q, n,
                       W.data_ptr<double>(), ww.data_ptr<double>(), st), "post_w_split");
  } else {
    W = at::empty({nrows, np}, f64);
    kmajor = false;
    ck(bo_gemm_f64(1, 1, nrows, int(np), nC * 128, 1.0, Rt.data_ptr<double>(), nrows, 0,
                   U.data_ptr<double>(), np, 0, 0.0, W.data_ptr<double>(), np, 0, 1,
                   BO_GEMM_B_LOWER, st), "w_matrix");
  }
  BoPostBackwardArgs pb{};
  pb.struct_size = sizeof(pb);
  pb.abi_version = BO_ABI_VERSION;
  pb.kind = int(kind);
  pb.B = B;
  pb.q = q;
  pb.d = int(d);
  pb.Xq = Xq.data_ptr<double>();
  pb.Xt_scaled = Xt_scaled.data_ptr<double>();
  pb.n = n;
  pb.W = W.data_ptr<double>();
  pb.ldw = W.size(1);
  pb.alpha = alpha.data_ptr<double>();
  pb.dmean = dmean.data_ptr<double>();
  pb.dcov = dcov.data_ptr<double>();
  pb.lengthscale = lengthscale.data_ptr<double>();
  pb.outputscale = outputscale;
  pb.ystd = ystd;
  pb.accumulate = 0;
  pb.w_kmajor = kmajor ? 1 : 0;
  pb.dX = dX.data_ptr<double>();
  ck(bo_post_backward_v(&pb, st), "post_backward");
  return dX;
}

at::Tensor ladder_defer(const at::Tensor& info, const at::Tensor& jitter) {
  TORCH_CHECK(info.is_cuda() && info.scalar_type() == at::kInt && info.is_contiguous(),
              "bo::ladder_defer: info must be a contiguous int32 device tensor");
  TORCH_CHECK(jitter.is_cuda() && jitter.scalar_type() == at::kDouble && jitter.is_contiguous(),
              "bo::ladder_defer: jitter must be a contiguous fp64 device tensor");
  if (info.numel() == 0) return at::zeros({3}, at::TensorOptions().dtype(at::kDouble));
  const int dev = info.device().index();
  return defer_status(info, jitter, c10::hip::getCurrentHIPStream(dev).stream(), dev);
}

at::Tensor ladder_poll(int64_t device) {
  std::lock_guard<std::mutex> lk(g_ladder_mu);
  auto it = g_ladder.find(static_cast<int>(device));
  if (it == g_ladder.end()) return at::zeros({3}, at::TensorOptions().dtype(at::kDouble));
  return take_pending(it->second, true);
}

void post_timing(bool on) {
  std::lock_guard<std::mutex> lk(g_time_mu);
  g_time_on = on;
}

// Durations (ms) of the timed post_partials launches since the last read;
// waits for the last one.
at::Tensor post_timing_read() {
  std::lock_guard<std::mutex> lk(g_time_mu);
  auto out = at::empty({int64_t(g_time_ev.size())}, at::TensorOptions().dtype(at::kDouble));
  auto* o = out.data_ptr<double>();
  for (size_t i = 0; i < g_time_ev.size(); ++i) {
    float ms = 0.f;
    hk(hipEventSynchronize(g_time_ev[i].second), "hipEventSynchronize");
    hk(hipEventElapsedTime(&ms, g_time_ev[i].first, g_time_ev[i].second), "hipEventElapsedTime");
    o[i] = ms;
    hk(hipEventDestroy(g_time_ev[i].first), "hipEventDestroy");
    hk(hipEventDestroy(g_time_ev[i].second), "hipEventDestroy");
  }
  g_time_ev.clear();
  return out;
}

// ---- qEHVI over a ModelListGP's members, forward only --------------------------------
// Per device: 8 pairs of pinned, device-mapped status words (one per member)
// and their arrival counters; the finalisation launches fold each member's
// ladder outcome into its pair, the caller reads them after a stream sync.
struct MemberStatus {
  double* host = nullptr;
  double* dev = nullptr;
  int* count = nullptr;
};
std::mutex g_member_mu;
std::unordered_map<int, MemberStatus> g_member;

MemberStatus& member_status(int dev) {
  auto& M = g_member[dev];
  if (!M.host) {
    hk(hipHostMalloc(reinterpret_cast<void**>(&M.host), 16 * sizeof(double),
                     hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
    hk(hipHostGetDevicePointer(reinterpret_cast<void**>(&M.dev), M.host, 0), "hipHostGetDevicePointer");
    hk(hipMalloc(reinterpret_cast<void**>(&M.count), 8 * sizeof(int)), "hipMalloc");
    hk(hipMemset(M.count, 0, 8 * sizeof(int)), "hipMemset");
  }
  return M;
}

// The qEHVI forward of acquisition/multi_objective/monte_carlo.py:146-322 over
// a ModelListGP of m <= 8 exact GPs of one shape (models/model_list_gp.py ->
// one posterior per member), in one host call: every member's rows and K*x^T,
// the members' R R^T / R beta partials (one small-grid or member-batched
// stream-K launch where those plans apply, else one launch per member), each
// member's finalisation (mean + jittered q x q root, written into the stacked
// m x B x q (x q) inputs, ladder outcome folded into pinned words), then the
// qEHVI launch.  Returns [acq, status]: status is an m x 2 host view of the
// pinned words ([max info, max jitter] per member), valid once the caller has
// synchronised the stream (the caller raises / warns in member order).
std::vector<at::Tensor> qehvi_members_eager(
    const at::Tensor& X, at::TensorList Xt_scaled, at::TensorList U, at::TensorList beta,
    at::TensorList lengthscale, at::ArrayRef<double> outputscale, at::ArrayRef<double> constant,
    at::ArrayRef<double> ymean, at::ArrayRef<double> ystd, int64_t kind, int64_t n,
    const at::Tensor& Z, const at::Tensor& cell_lo, const at::Tensor& cell_hi, int64_t kxt_cap,
    bool defer_ladder) {
  check_f64(X, "X");
  check_f64(Z, "Z");
  check_f64(cell_lo, "cell_lo");
  check_f64(cell_hi, "cell_hi");
  const int M = static_cast<int>(U.size());
  TORCH_CHECK(M >= 1 && M <= 8 && Xt_scaled.size() == size_t(M) && beta.size() == size_t(M) &&
                  lengthscale.size() == size_t(M) && outputscale.size() == size_t(M) &&
                  constant.size() == size_t(M) && ymean.size() == size_t(M) && ystd.size() == size_t(M),
              "bo::qehvi_members_eager: 1..8 members, one entry per member in every list");
  TORCH_CHECK(X.dim() == 3, "bo::qehvi_members_eager: X must be B x q x d");
  const int B = static_cast<int>(X.size(0)), q = static_cast<int>(X.size(1)),
            d = static_cast<int>(X.size(2));
  TORCH_CHECK(cell_lo.dim() == 2 && cell_lo.size(1) == M && cell_hi.sizes() == cell_lo.sizes(),
              "bo::qehvi_members_eager: shared K x m cells");
  TORCH_CHECK(Z.dim() == 2 && Z.size(1) == int64_t(q) * M, "bo::qehvi_members_eager: Z must be S x (q m)");
  const int64_t np = U[0].size(0);
  for (int m = 0; m < M; ++m) {
    check_f64(Xt_scaled[m], "Xt_scaled");
    check_f64(U[m], "U");
    check_f64(beta[m], "beta");
    check_f64(lengthscale[m], "lengthscale");
    TORCH_CHECK(U[m].size(0) == np && Xt_scaled[m].size(0) == n && lengthscale[m].numel() == d,
                "bo::qehvi_members_eager: members of one shape (n, d) only");
  }
  const int dev = X.device().index();
  void* st = c10::hip::getCurrentHIPStream(dev).stream();
  auto f64 = X.options().dtype(at::kDouble);
  auto acq = at::empty({B}, f64);
  // ladder outcomes: deferred (the ring of pinned slots, as qmc_acq_eager:
  // this call's members fold into one slot's member pairs, the finished
  // calls' statuses come back as [has, info_max, jitter_max]) or, with
  // defer_ladder off, the member pairs of per-device words the caller reads
  // after a stream sync ([M, 2]: per member, in member order)
  std::unique_lock<std::mutex> lk_ring(g_ladder_mu, std::defer_lock);
  std::unique_lock<std::mutex> lk_mem(g_member_mu, std::defer_lock);
  double* words_dev = nullptr;
  int* counts = nullptr;
  at::Tensor status;
  DeviceLadder* Ld = nullptr;
  int mine = -1;
  if (defer_ladder) {
    lk_ring.lock();
    Ld = &ladder_for(dev);
    mine = free_slot(*Ld, status);
    words_dev = Ld->slot[mine].host_dev + 2;
    counts = Ld->slot[mine].count + 1;
  } else {
    lk_mem.lock();
    MemberStatus& ms = member_status(dev);
    for (int e = 0; e < 2 * M; ++e) ms.host[e] = 0.0;
    status = at::from_blob(ms.host, {M, 2}, at::TensorOptions().dtype(at::kDouble));
    words_dev = ms.dev;
    counts = ms.count;
  }
  if (B == 0) return {acq, status};

  int Qp = 0, nrows = 0, nC = 0;
  ck(bo_post_geometry(B, q, n, &Qp, &nrows, &nC), "post_geometry");
  const bool kxt = np * int64_t(nrows) * 8 <= kxt_cap;
  int nsmall = 0;
  int64_t wmem = -1;
  if (kxt) {
    ck(bo_post_small_plan(B, q, n, &nsmall), "post_small_plan");
    if (nsmall == 0 && M > 1) ck(bo_post_members_work(M, B, q, n, &wmem), "post_members_work");
  }
  int kc = 0;
  int64_t we = 0;
  if (nsmall == 0 && wmem < 0) ck(bo_post_split_plan(B, q, n, 0, &kc, &we), "post_split_plan");
  const int nparts = nsmall > 0 ? nsmall : nC;
  const int64_t wsz = wmem >= 0 ? wmem : (kc ? we : 0);

  // one workspace (offsets in doubles, 16-B aligned)
  auto al2 = [](int64_t v) { return (v + 1) & ~int64_t(1); };
  const int64_t s_xq = al2(int64_t(nrows) * 8), s_kt = kxt ? al2(np * nrows) : 0,
                s_sp = al2(int64_t(nparts) * nrows * 16), s_mp = al2(int64_t(nparts) * nrows);
  const int64_t per = s_xq + s_kt + s_sp + s_mp;
  const int64_t o_work = per * M;
  const int64_t o_mean = o_work + al2(std::max<int64_t>(wsz, 0));
  const int64_t o_L = o_mean + al2(int64_t(M) * B * q);
  const int64_t o_jit = o_L + al2(int64_t(M) * B * q * q);
  const int64_t o_info = o_jit + al2(int64_t(M) * B);
  const int64_t o_qw = o_info + al2((int64_t(M) * B + 1) / 2);
  const int64_t total = o_qw + al2(8 * int64_t(B));
  auto ws = at::empty({total}, f64);
  double* w = ws.data_ptr<double>();
  const double* Kt_p[8];
  const double* U_p[8];
  const double* b_p[8];
  double* S_p[8];
  double* m_p[8];
  double* Xq_p[8];
  const double* ls_p[8];
  const double* xt_p[8];
  double* Ktw_p[8];
  for (int m = 0; m < M; ++m) {
    double* base = w + per * m;
    Xq_p[m] = base;
    Ktw_p[m] = kxt ? base + s_xq : nullptr;
    Kt_p[m] = Ktw_p[m];
    S_p[m] = base + s_xq + s_kt;
    m_p[m] = base + s_xq + s_kt + s_sp;
    U_p[m] = U[m].data_ptr<double>();
    b_p[m] = beta[m].data_ptr<double>();
    ls_p[m] = lengthscale[m].data_ptr<double>();
    xt_p[m] = Xt_scaled[m].data_ptr<double>();
    if (!kxt)
      ck(bo_prepare_rows(X.data_ptr<double>(), B, q, d, ls_p[m], Xq_p[m], st), "prepare_rows");
  }
  if (kxt)  // every member's rows and K*x^T in one launch
    ck(bo_post_kxt_rows_members(M, int(kind), X.data_ptr<double>(), B, q, d, ls_p, xt_p,
                                outputscale.data(), n, Xq_p, Ktw_p, st), "post_kxt_rows_members");
  hipEvent_t t0 = nullptr;
  {
    std::lock_guard<std::mutex> tl(g_time_mu);
    if (g_time_on) t0 = timing_event(st);
  }
  if (nsmall > 0) {
    double* const* no_rt = nullptr;
    ck(bo_post_small_batched(M, Kt_p, U_p, b_p, S_p, m_p, no_rt, B, q, n, np, st), "post_small_batched");
  } else if (wmem >= 0) {
    ck(bo_post_partials_members(M, Kt_p, U_p, b_p, S_p, m_p, nullptr, Xq_p[0], B, q, n, np,
                                w + o_work, st), "post_partials_members");
  } else {
    for (int m = 0; m < M; ++m) {
      BoPostPartialsArgs pa{};
      pa.struct_size = sizeof(pa);
      pa.abi_version = BO_ABI_VERSION;
      pa.kind = int(kind);
      pa.B = B;
      pa.q = q;
      pa.d = d;
      pa.Xq = Xq_p[m];
      pa.Xt_scaled = Xt_scaled[m].data_ptr<double>();
      pa.n = n;
      pa.U = U_p[m];
      pa.ldu = np;
      pa.beta = b_p[m];
      pa.outputscale = outputscale[m];
      pa.Spart = S_p[m];
      pa.mpart = m_p[m];
      pa.kc_len = kc;
      pa.work = kc ? w + o_work : nullptr;
      pa.Kt = Kt_p[m];
      ck(bo_post_partials_v(&pa, st), "post_partials");
    }
  }
  if (t0) {
    std::lock_guard<std::mutex> tl(g_time_mu);
    g_time_ev.emplace_back(t0, timing_event(st));
  }
  double* mean = w + o_mean;
  double* Lq = w + o_L;
  {  // every member's finalisation in one launch (grid B x M)
    const double* xq_c[8];
    const double* sp_c[8];
    const double* mp_c[8];
    double* mo[8];
    double* lo_[8];
    int* io[8];
    double* jo[8];
    double* so[8];
    int* co[8];
    for (int m = 0; m < M; ++m) {
      xq_c[m] = Xq_p[m];
      sp_c[m] = S_p[m];
      mp_c[m] = m_p[m];
      mo[m] = mean + int64_t(m) * B * q;
      lo_[m] = Lq + int64_t(m) * B * q * q;
      io[m] = reinterpret_cast<int*>(w + o_info) + int64_t(m) * B;
      jo[m] = w + o_jit + int64_t(m) * B;
      so[m] = words_dev + 2 * m;
      co[m] = counts + m;
    }
    // max_tries 6: botorch/__init__.py:47 (cholesky_max_tries); jitter 1e-8: [G] cholesky_jitter
    ck(bo_qmc_finalize_members(M, int(kind), B, q, xq_c, sp_c, mp_c, n, outputscale.data(),
                               constant.data(), ymean.data(), ystd.data(), 6, 1e-8, mo, lo_, io, jo,
                               nsmall, so, co, nullptr, 0, 0, nullptr, 0, st),
       "qmc_finalize_members");
  }
  BoQehviArgs qa{};
  qa.struct_size = sizeof(qa);
  qa.abi_version = BO_ABI_VERSION;
  qa.B = B;
  qa.q = q;
  qa.m = M;
  qa.S = static_cast<int32_t>(Z.size(0));
  qa.mean = mean;
  qa.L = Lq;
  qa.Z = Z.data_ptr<double>();
  qa.cell_lo = cell_lo.data_ptr<double>();
  qa.cell_hi = cell_hi.data_ptr<double>();
  qa.K = static_cast<int32_t>(cell_lo.size(0));
  qa.acq = acq.data_ptr<double>();
  qa.work = w + o_qw;
  qa.work_elems = 8 * int64_t(B);
  ck(bo_qehvi_v(&qa, st), "qehvi");
  if (defer_ladder) publish_slot(*Ld, mine, st, true);
  return {acq, status};
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(bo, m) {
  m.def("qehvi_members_eager(Tensor X, Tensor[] Xt_scaled, Tensor[] U, Tensor[] beta, "
        "Tensor[] lengthscale, float[] outputscale, float[] constant, float[] ymean, float[] ystd, "
        "int kind, int n, Tensor Z, Tensor cell_lo, Tensor cell_hi, int kxt_cap, "
        "bool defer_ladder=False) -> Tensor[]");
  m.def("qmc_acq_native(Tensor X, Tensor Xt_scaled, Tensor U, Tensor Linv, Tensor beta, "
        "Tensor lengthscale, Tensor Z, Tensor? best_f_s, int kind, int mode, int n, "
        "float outputscale, float constant, float ymean, float ystd, float best_f, bool fat, "
        "float tau_relu, float tau_max, bool need_grad, int kxt_cap, bool defer_ladder, "
        "Tensor? Ainv=None, Tensor? alpha=None) -> Tensor[]");
  m.def("qmc_acq_eager(Tensor X, Tensor Xt_scaled, Tensor U, Tensor beta, Tensor lengthscale, "
        "Tensor Z, Tensor? best_f_s, int kind, int mode, int n, float outputscale, float constant, "
        "float ymean, float ystd, float best_f, bool fat, float tau_relu, float tau_max, "
        "int kxt_cap, Tensor? Ainv=None, Tensor? alpha=None, Tensor? cap_status=None, "
        "Tensor? cap_count=None) -> Tensor[]");
  m.def("qmc_acq_backward_native(Tensor dacq, Tensor acq, Tensor mean, Tensor L, Tensor Z, "
        "Tensor? best_f_s, Tensor Xq, Tensor Rt, Tensor Linv, Tensor U, Tensor Xt_scaled, "
        "Tensor alpha, Tensor lengthscale, int kind, int mode, int d, int n, float outputscale, "
        "float ystd, float best_f, bool fat, float tau_relu, float tau_max) -> Tensor");
  m.def("ladder_defer(Tensor info, Tensor jitter) -> Tensor");
  m.def("ladder_poll(int device) -> Tensor", &ladder_poll);
  m.def("post_timing(bool on) -> ()", &post_timing);
  m.def("post_timing_read() -> Tensor", &post_timing_read);
  m.def("last_backward_route() -> int", &last_backward_route);
  m.def("pinned_status() -> Tensor", &pinned_status);
}

TORCH_LIBRARY_IMPL(bo, CUDA, m) {
  m.impl("qmc_acq_native", &qmc_acq_native);
  m.impl("qmc_acq_eager", &qmc_acq_eager);
  m.impl("qmc_acq_backward_native", &qmc_acq_backward_native);
  m.impl("ladder_defer", &ladder_defer);
  m.impl("qehvi_members_eager", &qehvi_members_eager);
}
