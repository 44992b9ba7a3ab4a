#!/usr/bin/env python3
"""Task trace of the persistent Cholesky DAG (bo_probe_chol_dag): where the
n = 4096 factorisation + inverse spends its time.  Prints the span, per-type
task time sums, the CRIT(k) chain (start/end, gap to its predecessor) and the
idle fraction of the workgroups.  BO_N overrides n."""
import ctypes
import json
import os
import sys

import torch
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _toolslib  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd import kernels  # noqa: E402
from botorch_amd._lib import check, lib  # noqa: E402
from oracle.gp import covar  # noqa: E402

TYPES = ["CRIT", "TRSM", "COLUPD", "XSTEP"]


def main():
    n = int(os.environ.get("BO_N", "4096"))
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    X = torch.rand(n, 6, generator=g, dtype=torch.float64)
    A0 = (covar(X, X, torch.full((6,), 0.5, dtype=torch.float64), x1_eq_x2=True)
          + 1e-3 * torch.eye(n, dtype=torch.float64)).tril().to(dev)
    np_ = kernels.padded_order(n)
    A = torch.eye(np_, dtype=torch.float64, device=dev)
    Linv = torch.empty_like(A)
    work = torch.empty_like(A)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    trace = torch.zeros(8 * 40000 + 8 * 1024, dtype=torch.int64, device=dev)
    nt = ctypes.c_int(0)
    out = {}
    for rep in range(3):
        A[:n, :n] = A0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        check(_toolslib.tools().bo_probe_chol_dag(kernels._p(A), kernels._p(Linv), np_, kernels._p(info),
                                      kernels._p(work), kernels._p(trace), ctypes.byref(nt),
                                      kernels._stream(dev)), "probe_chol_dag")
        e1.record()
        torch.cuda.synchronize()
        out[f"ms_rep{rep}"] = e0.elapsed_time(e1)
    ntask = nt.value
    tr = trace[: 4 * ntask].view(ntask, 4).cpu()
    st, en, pk, wt = tr[:, 0], tr[:, 1], tr[:, 2], tr[:, 3]
    t0 = int(st.min())
    typ = (pk >> 16) & 0xff
    k = (pk >> 24) & 0xffff
    j = (pk >> 40) & 0xffff
    blk = pk & 0xffff
    dur = (en - st).double() / 100.0  # us
    out.update(n=n, info=int(info.item()), tasks=ntask, span_us=float(en.max() - t0) / 100.0)
    out["per_type_us"] = {TYPES[t]: float(dur[typ == t].sum()) for t in range(4)}
    out["per_type_count"] = {TYPES[t]: int((typ == t).sum()) for t in range(4)}
    out["per_type_wait_us"] = {TYPES[t]: float(wt[typ == t].double().sum() / 100.0) for t in range(4)}
    out["per_type_mean_us"] = {TYPES[t]: float(dur[typ == t].mean()) for t in range(4) if (typ == t).any()}
    nblk = int(blk.max()) + 1
    busy = float(dur.sum())
    out["blocks"] = nblk
    out["busy_frac"] = busy / (nblk * out["span_us"])
    crit = (typ == 0).nonzero().flatten()
    rows = []
    prev_end = None
    for idx in crit.tolist():
        s_, e_ = (int(st[idx]) - t0) / 100.0, (int(en[idx]) - t0) / 100.0
        rows.append([int(k[idx]), round(s_, 1), round(e_, 1), round(e_ - s_, 1),
                     None if prev_end is None else round(e_ - prev_end, 1)])
        prev_end = e_
    out["crit_k_start_end_dur_step"] = rows
    ct = trace[4 * ntask: 4 * ntask + 8 * (n // 64)].view(-1, 8).cpu()
    ph = (ct[:, 1:4] - ct[:, 0:3]).double() / 100.0
    out["crit_phase_us_mean"] = {"potrf": float(ph[:, 0].mean()), "trtri": float(ph[:, 1].mean()),
                                 "store_publish": float(ph[:, 2].mean()),
                                 "diag0": float(((ct[:, 4] - ct[:, 0]).double() / 100.0).mean()),
                                 "loop3": float(((ct[:, 5] - ct[:, 4]).double() / 100.0).mean()),
                                 "merges": float(((ct[:, 1] - ct[:, 5]).double() / 100.0).mean()),
                                 # column-owner factor: waves 1 and 3 start their own columns
                                 "w1_start": float(((ct[:, 6] - ct[:, 0]).double() / 100.0).mean()),
                                 "w3_start": float(((ct[:, 7] - ct[:, 0]).double() / 100.0).mean())}
    pre = [(int(ct[kk, 0]) - int(st[i])) / 100.0 for kk, i in enumerate(crit.tolist())]
    out["crit_pre_us_mean"] = sum(pre) / len(pre)
    ph = trace[4 * ntask + 8 * (np_ // 64): 4 * ntask + 8 * (np_ // 64) + 8 * ntask].view(ntask, 8).cpu()
    for t in (0, 1, 2, 3):
        sel = typ == t
        tiles = max(1, int(ph[sel, 3].sum()))
        out[f"{TYPES[t]}_per_tile_us"] = {"commit": float(ph[sel, 0].sum()) / 100.0 / tiles,
                                          "of_which_operand_wait": float(ph[sel, 5].sum()) / 100.0 / tiles,
                                          "mfma": float(ph[sel, 1].sum()) / 100.0 / tiles,
                                          "store_publish": float(ph[sel, 2].sum()) / 100.0 / tiles,
                                          "prefetched_frac": float(ph[sel, 4].sum()) / tiles,
                                          "tiles": tiles}
    # the tasks that touch the last tile row after the second-to-last CRIT
    # (what the final diagonal step waited on)
    import numpy as np
    nq = lib().bo_chol_dag_tasks(np_ // 64, None, 0)
    qb = np.zeros(4 * nq, dtype=np.int32)
    lib().bo_chol_dag_tasks(np_ // 64, qb.ctypes.data_as(ctypes.c_void_p), nq)
    qb = qb.reshape(nq, 4)
    T = np_ // 64
    crit_end = {int(k[i]): int(en[i]) for i in crit.tolist()}
    t62 = crit_end.get(T - 2, int(en.max()))
    tail = []
    for t in range(ntask):
        x, kk, jj, w = (int(v) for v in qb[t])
        i0, i1 = w & 0xFFFF, w >> 16
        if int(en[t]) > t62 - 3000 and (i1 > T - 1 or (x & 0xFF) == 0):
            tail.append([TYPES[x & 0xFF], kk, jj, i0, i1, max(1, x >> 16), (x >> 8) & 0xFF,
                         round((int(st[t]) - t0) / 100.0, 1), round((int(en[t]) - t0) / 100.0, 1),
                         int(blk[t])])
    tail.sort(key=lambda r: r[7])
    out["tail_tasks_type_k_j_i0_i1_nk_fin_start_end_block"] = [r for r in tail if r[0] != "XSTEP"] + \
        [r for r in tail if r[0] == "XSTEP"][-8:]
    # per diagonal step: when its inputs were published (relative to the
    # CRIT task's start): D_{k-1} (CRIT(k-1) end), the last updates of
    # A(k, k-1) and A(k, k) (the COLUPD tasks ending at step k - 2)
    ends = {}
    for t in range(ntask):
        x, kk, jj, w = (int(v) for v in qb[t])
        if (x & 0xFF) != 2:
            continue
        nk_ = max(1, x >> 16)
        i0, i1 = w & 0xFFFF, w >> 16
        for i in range(i0, i1):
            if jj in (i, i - 1):  # tiles (i, i) and (i, i - 1)
                ends.setdefault((i, jj), []).append((kk + nk_ - 1, int(en[t]), int(st[t]), nk_, kk))
    crit_in = []
    for idx in crit.tolist():
        kk = int(k[idx])
        if kk < 2:
            continue
        s0 = int(st[idx])
        row = [kk, round((crit_end.get(kk - 1, s0) - s0) / 100.0, 1)]
        for jj in (kk - 1, kk):
            c = [e for e in ends.get((kk, jj), []) if e[0] == kk - 2]
            row.append(round((c[0][1] - s0) / 100.0, 1) if c else None)
            row.append(c[0][3] if c else None)
        crit_in.append(row)
    out["crit_inputs_k_Dprev_Akk1_nk_Akk_nk_us_after_start"] = crit_in
    # the history of tile (k, k) and of tile row k of L for a few steps: every
    # task writing them (type, k, j, i0, i1, nk, queue slot, start, end, block)
    hist = {}
    for kk in [int(s) for s in os.environ.get("BO_TRACE_K", "26,27,28,29,30").split(",")]:
        rows_ = []
        for t in range(ntask):
            x, k2, jj, w = (int(v) for v in qb[t])
            i0, i1 = w & 0xFFFF, w >> 16
            ty = x & 0xFF
            if (ty == 2 and jj == kk and i0 <= kk < i1) or (ty == 1 and i0 <= kk < i1 and k2 >= kk - 5) or \
               (ty == 0 and kk - 5 <= k2 <= kk):
                rows_.append([TYPES[ty], k2, jj, i0, i1, max(1, x >> 16), t,
                              round((int(st[t]) - t0) / 100.0, 1), round((int(en[t]) - t0) / 100.0, 1),
                              int(blk[t])])
        rows_.sort(key=lambda r: r[7])
        hist[kk] = [r for r in rows_ if r[8] > (crit_end.get(kk - 5, t0) - t0) / 100.0]
    out["diag_history_type_k_j_i0_i1_nk_slot_start_end_block"] = hist
    # the last finishing tasks
    last = torch.argsort(en, descending=True)[:8]
    out["last_tasks"] = [[TYPES[int(typ[i])], int(k[i]), int(j[i]), round((int(st[i]) - t0) / 100.0, 1),
                          round((int(en[i]) - t0) / 100.0, 1)] for i in last.tolist()]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
