"""HIP kernels through the C ABI vs. the CPU oracle / torch fp64 references."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _hartmann_data(n, seed=0, d=6):
    from botorch_amd.test_functions import Hartmann
    from oracle.sampling import draw_sobol_samples
    lo = torch.zeros(d, dtype=torch.float64)
    X = draw_sobol_samples(lo, lo + 1, n, 1, seed).squeeze(1)
    Y = Hartmann(dim=6, negate=True)(X[:, :6]).unsqueeze(-1)
    return X, Y


def test_mfma_f64_layout():
    from botorch_amd import kernels
    out = kernels.probe_mfma_layout(DEV).cpu()
    np.testing.assert_array_equal(out[:, :4].numpy(), out[:, 4:].numpy())


@pytest.mark.parametrize("M,N,K", [(64, 64, 64), (130, 70, 33), (300, 257, 129), (1, 5, 3)])
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
def test_gemm_matches_torch(M, N, K, ta, tb):
    from botorch_amd import kernels
    g = torch.Generator().manual_seed(M * 7 + N)
    A = torch.randn(K, M, generator=g, dtype=torch.float64) if ta else torch.randn(M, K, generator=g, dtype=torch.float64)
    B = torch.randn(N, K, generator=g, dtype=torch.float64) if tb else torch.randn(K, N, generator=g, dtype=torch.float64)
    C0 = torch.randn(M, N, generator=g, dtype=torch.float64)
    ref = 0.5 * ((A.T if ta else A) @ (B.T if tb else B)) - 2.0 * C0
    out = kernels.gemm(A.to(DEV), B.to(DEV), ta, tb, alpha=0.5, beta=-2.0, C=C0.clone().to(DEV))
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-12, atol=1e-11)


@pytest.mark.parametrize("M,N,K,batch", [(4, 4, 256, 1024), (16, 16, 3, 7), (1, 16, 33, 5), (9, 2, 100, 3),
                                         (256, 4, 4, 64), (77, 1, 256, 3), (300, 16, 17, 2)])
@pytest.mark.parametrize("ta,tb", [(False, True), (True, False), (True, True)])
def test_gemm_small_batched(M, N, K, batch, ta, tb):
    """N <= 16 with M <= 16 or K <= 256 take the one-wave-per-16-rows kernel."""
    from botorch_amd import kernels
    g = torch.Generator().manual_seed(M + 3 * N + K)
    A = torch.randn(batch, *((K, M) if ta else (M, K)), generator=g, dtype=torch.float64)
    B = torch.randn(batch, *((N, K) if tb else (K, N)), generator=g, dtype=torch.float64)
    C0 = torch.randn(batch, M, N, generator=g, dtype=torch.float64)
    ref = 2.0 * ((A.mT if ta else A) @ (B.mT if tb else B)) + 0.5 * C0
    out = kernels.gemm(A.to(DEV), B.to(DEV), ta, tb, alpha=2.0, beta=0.5, C=C0.clone().to(DEV))
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-12, atol=1e-11)


@pytest.mark.parametrize("M,N,K,flags", [(3968, 128, 128, 4), (2432, 128, 128, 1), (200, 100, 37, 0),
                                          (1000, 33, 256, 2)])
def test_gemm_strip_panels(M, N, K, flags):
    """The blocked Cholesky panel shapes (rem x 128 x 128, triangular / lower-C flags)."""
    from botorch_amd import kernels
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    Bm = torch.randn(N, K, generator=g, dtype=torch.float64)
    C0 = torch.randn(M, N, generator=g, dtype=torch.float64)
    # flags promise structural zeros (the tiled kernel skips zero k-ranges at
    # tile granularity), so the operands hold them
    A = torch.tril(A) if flags & 2 else A
    Bm = torch.triu(Bm.T).T.contiguous() if flags & 4 else Bm  # op(B) = B^T upper
    ref = -1.0 * (A @ Bm.T) + C0
    out = kernels.gemm(A.to(DEV), Bm.to(DEV), False, True, alpha=-1.0, beta=1.0,
                       C=C0.clone().to(DEV), flags=flags).cpu()
    if flags & 1:
        torch.testing.assert_close(torch.tril(out), torch.tril(ref), rtol=1e-12, atol=1e-11)
        torch.testing.assert_close(torch.triu(out, 1), torch.triu(C0, 1))
    else:
        torch.testing.assert_close(out, ref, rtol=1e-12, atol=1e-11)


def test_gemm_small_flags():
    from botorch_amd import kernels, _lib
    g = torch.Generator().manual_seed(5)
    L = torch.randn(12, 12, generator=g, dtype=torch.float64)  # lower part used
    B = torch.randn(12, 7, generator=g, dtype=torch.float64)
    out = kernels.gemm(L.to(DEV), B.to(DEV), flags=_lib.GEMM_A_LOWER).cpu()
    torch.testing.assert_close(out, torch.tril(L) @ B, rtol=1e-12, atol=1e-12)
    P = torch.randn(10, 30, generator=g, dtype=torch.float64)
    C = torch.randn(10, 10, generator=g, dtype=torch.float64)
    out = kernels.gemm(P.to(DEV), P.to(DEV), False, True, alpha=-1.0, beta=1.0,
                       C=C.clone().to(DEV), flags=_lib.GEMM_LOWER_C).cpu()
    torch.testing.assert_close(torch.tril(out), torch.tril(C - P @ P.T), rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(torch.triu(out, 1), torch.triu(C, 1))
    U = torch.randn(9, 9, generator=g, dtype=torch.float64)
    X = torch.randn(5, 9, generator=g, dtype=torch.float64)
    out = kernels.gemm(X.to(DEV), U.to(DEV), flags=_lib.GEMM_B_UPPER).cpu()
    torch.testing.assert_close(out, X @ torch.triu(U), rtol=1e-12, atol=1e-12)


def test_gemm_batched_and_large():
    from botorch_amd import kernels
    g = torch.Generator().manual_seed(1)
    A = torch.randn(3, 700, 300, generator=g, dtype=torch.float64)
    B = torch.randn(3, 300, 650, generator=g, dtype=torch.float64)
    out = kernels.gemm(A.to(DEV), B.to(DEV))
    torch.testing.assert_close(out.cpu(), A @ B, rtol=1e-12, atol=1e-10)
    A = torch.randn(2048, 512, generator=g, dtype=torch.float64)
    B = torch.randn(512, 2048, generator=g, dtype=torch.float64)
    out = kernels.gemm(A.to(DEV), B.to(DEV))
    torch.testing.assert_close(out.cpu(), A @ B, rtol=1e-12, atol=1e-10)


def test_gemm_triangular_flags():
    from botorch_amd import kernels, _lib
    g = torch.Generator().manual_seed(2)
    n = 200
    Lw = torch.tril(torch.randn(n, n, generator=g, dtype=torch.float64))
    B = torch.randn(n, 90, generator=g, dtype=torch.float64)
    out = kernels.gemm(Lw.to(DEV), B.to(DEV), flags=_lib.GEMM_A_LOWER)
    torch.testing.assert_close(out.cpu(), Lw @ B, rtol=1e-12, atol=1e-11)
    P = torch.randn(n, 40, generator=g, dtype=torch.float64)
    C = torch.randn(n, n, generator=g, dtype=torch.float64)
    out = kernels.gemm(P.to(DEV), P.to(DEV), False, True, alpha=-1.0, beta=1.0,
                       C=C.clone().to(DEV), flags=_lib.GEMM_LOWER_C).cpu()
    ref = C - P @ P.T
    torch.testing.assert_close(torch.tril(out), torch.tril(ref), rtol=1e-12, atol=1e-11)
    torch.testing.assert_close(torch.triu(out, 1), torch.triu(C, 1))


@pytest.mark.parametrize("n", [20, 128, 333, 1024, 2900])
def test_cholesky_inverse_matches_torch(n):
    from botorch_amd import kernels
    g = torch.Generator().manual_seed(n)
    M = torch.randn(n, n, generator=g, dtype=torch.float64)
    A = M @ M.T / n + torch.eye(n, dtype=torch.float64)
    L, Linv, info = kernels.cholesky_inverse(A.to(DEV))
    assert info == 0
    Lr = torch.linalg.cholesky(A)
    torch.testing.assert_close(L.cpu(), Lr, rtol=1e-10, atol=1e-12)
    torch.testing.assert_close(Linv.cpu(), torch.linalg.inv(Lr), rtol=1e-9, atol=1e-11)


def test_cholesky_reports_not_pd():
    from botorch_amd import kernels
    A = torch.eye(100, dtype=torch.float64)
    A[57, 57] = -1.0
    _, _, info = kernels.cholesky_inverse(A.to(DEV))
    assert info == 58


def _oracle_model(n, d=6, ls=None, noise=1e-3, const=0.1):
    from oracle.gp import ExactGPOracle, GPHyper
    X, Y = _hartmann_data(n, d=d)
    h = GPHyper(ls if ls is not None else torch.full((d,), 0.35, dtype=torch.float64), noise, const)
    return X, Y, ExactGPOracle(X, Y, h), h


def _device_cache(X, Y, h, orc):
    from botorch_amd import kernels
    return kernels.build_gp_cache(X.to(DEV), orc.train_y.to(DEV), h.lengthscale.to(DEV),
                                  h.noise, h.constant)


@pytest.mark.parametrize("n", [37, 256, 1000])
def test_gp_cache_matches_oracle(n):
    X, Y, orc, h = _oracle_model(n)
    c = _device_cache(X, Y, h, orc)
    torch.testing.assert_close(c.U[:n, :n].cpu(), orc.LinvT, rtol=1e-8, atol=1e-9)
    torch.testing.assert_close(c.alpha.cpu(), orc.alpha, rtol=1e-7, atol=1e-8)


@pytest.mark.parametrize("n,B,q", [(37, 5, 3), (256, 33, 8), (300, 64, 16), (1000, 20, 1), (513, 9, 5)])
def test_posterior_matches_oracle(n, B, q):
    from botorch_amd import kernels, _lib
    X, Y, orc, h = _oracle_model(n)
    c = _device_cache(X, Y, h, orc)
    g = torch.Generator().manual_seed(B)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64)
    pp = kernels.post_partials(c, Xc.to(DEV))
    out = kernels.qmc_finalize(c, pp, _lib.QMC_POSTERIOR, orc.ymean.item(), orc.ystd.item())
    mean_r, cov_r = orc.posterior(Xc)
    torch.testing.assert_close(out["mean"].cpu(), mean_r, rtol=1e-4, atol=1e-8)
    var_r = cov_r.diagonal(dim1=-2, dim2=-1)
    var = out["cov"].diagonal(dim1=-2, dim2=-1).cpu()
    torch.testing.assert_close(var, var_r, rtol=1e-4, atol=1e-10)
    torch.testing.assert_close(out["cov"].cpu(), cov_r, rtol=1e-4, atol=1e-9)


@pytest.mark.parametrize("q", list(range(1, 17)))
def test_qmc_root_every_q_and_ladder(q):
    """The q x q root of qmc_kernel (QMC_CHOL) at every q: the 8- and 16-wide
    entry layouts of ladder_factor, rows past q masked.  The root of the
    finalised covariance against torch's Cholesky of the same matrix.  A
    t-batch whose points repeat has a rank-1 covariance: whether its first
    zero pivot rounds to + or - is arithmetic-dependent, so it is held to the
    ladder's contract (psd_safe_cholesky, [G]): the jitter is 0 or one of
    jitter0 * 10^i, and L L^T reproduces cov + jitter I."""
    from botorch_amd import kernels, _lib
    X, Y, orc, h = _oracle_model(256, noise=1e-4)
    c = _device_cache(X, Y, h, orc)
    g = torch.Generator().manual_seed(100 + q)
    Xc = torch.rand(6, q, 6, generator=g, dtype=torch.float64)
    if q > 1:
        Xc[5, 1:] = Xc[5, 0]  # t-batch 5: one point repeated -> rank-1 covariance
    pp = kernels.post_partials(c, Xc.to(DEV))
    out = kernels.qmc_finalize(c, pp, _lib.QMC_CHOL, orc.ymean.item(), orc.ystd.item(), want_L=True)
    cov, L = out["cov"].cpu(), out["L"].cpu()
    info, jit = out["info"].cpu(), out["jitter"].cpu()
    assert (info == 0).all()
    torch.testing.assert_close(L[:5], torch.linalg.cholesky(cov[:5]), rtol=1e-9, atol=1e-12)
    assert (jit[:5] == 0).all()
    j5 = jit[5].item()
    assert j5 == 0.0 or any(j5 == pytest.approx(kernels.CHOLESKY_JITTER_F64 * 10.0 ** i, rel=1e-12)
                            for i in range(kernels.CHOLESKY_MAX_TRIES))
    A5 = cov[5] + j5 * torch.eye(q, dtype=torch.float64)
    torch.testing.assert_close(L[5] @ L[5].T, A5, rtol=1e-9, atol=1e-12)
    assert torch.equal(L[5], L[5].tril())


@pytest.mark.parametrize("n,B,q,split", [(1024, 64, 8, None), (1024, 64, 8, 64), (1000, 20, 3, 128),
                                         (513, 9, 5, 256), (300, 33, 16, 64), (4096, 64, 16, None),
                                         (1000, 20, 3, -1), (300, 33, 16, -1), (2048, 40, 16, -1)])
def test_post_partials_split_k(n, B, q, split):
    """Split plans (uniform chunks, or stream-K shares of the concatenated
    k-steps; ordered reduction of each cut tile) against the one-pass kernel
    and the oracle: same Spart / mpart / R^T up to fp64 summation order."""
    from botorch_amd import kernels, _lib
    X, Y, orc, h = _oracle_model(n)
    c = _device_cache(X, Y, h, orc)
    g = torch.Generator().manual_seed(n + B)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64).to(DEV)
    kc, _ = kernels.split_plan(B, q, n)
    if split is None:
        assert kc == -1  # C2 geometry (32 tiles) and a rank's b = 64 share of C3: stream-K
    one = kernels.post_partials(c, Xc, store_R=True, split=0)
    spl = kernels.post_partials(c, Xc, store_R=True, split=split, small=False)
    # the split-k plan without the K*x^T buffer (kernel rows
    # evaluated between the MFMAs) -- the path taken above the KXT cap
    nok = kernels.post_partials(c, Xc, store_R=True, split=split, kxt=False)
    # fp64 summation order only: atol grows with the k-range summed (n);
    # 4.7e-13 observed at n = 4096 on an element of 5e-3 (sums with cancellation)
    atol = 2.5e-13 * max(1.0, n / 1024)
    for a, b in ((one.Spart, spl.Spart), (one.mpart, spl.mpart), (one.Rt, spl.Rt),
                 (one.Spart, nok.Spart), (one.mpart, nok.mpart), (one.Rt, nok.Rt)):
        torch.testing.assert_close(b, a, rtol=1e-11, atol=atol)
    if split is None and kernels.small_plan(B, q, n) > 0:
        # the library's choice here: the small-grid kernel (pair partials, R^T
        # row-major) -- the same R^T, and the same sums over its partials
        sml = kernels.post_partials(c, Xc, store_R=True)
        assert sml.Spart.shape[0] == kernels.padded_order(n) // 64
        torch.testing.assert_close(sml.Rt, one.Rt, rtol=1e-11, atol=atol)
        torch.testing.assert_close(sml.Spart.sum(0), one.Spart.sum(0), rtol=1e-11, atol=atol)
        torch.testing.assert_close(sml.mpart.sum(0), one.mpart.sum(0), rtol=1e-11, atol=atol)
    out = kernels.qmc_finalize(c, spl, _lib.QMC_POSTERIOR, orc.ymean.item(), orc.ystd.item())
    mean_r, cov_r = orc.posterior(Xc.cpu())
    torch.testing.assert_close(out["mean"].cpu(), mean_r, rtol=1e-4, atol=1e-8)
    torch.testing.assert_close(out["cov"].cpu(), cov_r, rtol=1e-4, atol=1e-9)


@pytest.mark.parametrize("n,B,q,S", [(256, 16, 4, 128), (1024, 64, 8, 256)])
def test_qei_matches_oracle(n, B, q, S):
    from botorch_amd import kernels, _lib
    from oracle.acquisition import qei
    from oracle.sampling import draw_sobol_normal_samples
    X, Y, orc, h = _oracle_model(n)
    c = _device_cache(X, Y, h, orc)
    g = torch.Generator().manual_seed(q)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64)
    Z = draw_sobol_normal_samples(q, S, 0)
    best_f = Y.max().item()
    pp = kernels.post_partials(c, Xc.to(DEV))
    out = kernels.qmc_finalize(c, pp, _lib.QMC_QEI, orc.ymean.item(), orc.ystd.item(),
                               Z=Z.to(DEV), best_f=best_f, want_L=True)
    ref = qei(orc, Xc, Z, best_f)
    assert (out["info"].cpu() == 0).all()
    torch.testing.assert_close(out["acq"].cpu(), ref, rtol=1e-2, atol=1e-6)
    # much tighter in practice: the same fp64 algorithm
    torch.testing.assert_close(out["acq"].cpu(), ref, rtol=1e-7, atol=1e-10)


@pytest.mark.parametrize("d,n,seed", [(1, 4, 0), (3, 16, 1234), (8, 256, 0), (16, 512, 0), (40, 64, 7)])
def test_sobol_normal_matches_golden(golden, d, n, seed):
    from botorch_amd import kernels
    z = kernels.sobol_normal(d, n, seed, DEV).cpu().numpy()
    ref = golden[f"sobol_normal_d{d}_n{n}_s{seed}"]
    np.testing.assert_allclose(z, ref, rtol=4e-15, atol=4e-15)


def test_not_psd_raises():
    from botorch_amd import kernels
    from botorch_amd.exceptions import NotPSDError
    X = torch.rand(50, 6, dtype=torch.float64)
    y = torch.randn(50, dtype=torch.float64)
    with pytest.raises(NotPSDError):
        kernels.build_gp_cache(X.to(DEV), y.to(DEV), torch.full((6,), 0.3, dtype=torch.float64, device=DEV),
                               noise=-1.0, constant=0.0)


def test_sobol_transform_accuracy_dense_grid():
    """z(u) for every 30-bit u on a dense grid (state = 0, shift = u * 2^30)
    against torch's CPU erfinv path (the reference's NormalQMCEngine)."""
    from botorch_amd import kernels, _lib
    import ctypes
    g = torch.Generator().manual_seed(0)
    ints = torch.cat([torch.randint(0, 2 ** 30, (20000,), generator=g),
                      torch.arange(0, 64), 2 ** 30 - 1 - torch.arange(0, 64),
                      2 ** 29 + torch.arange(-64, 64)]).to(torch.int64)
    dim = ints.numel()
    state = torch.zeros(dim, 30, dtype=torch.int64, device=DEV)
    shift = ints.to(DEV)
    out = torch.empty(1, dim, dtype=torch.float64, device=DEV)
    _lib.check(_lib.lib().bo_sobol_normal(ctypes.c_void_p(state.data_ptr()), ctypes.c_void_p(shift.data_ptr()),
                                          dim, 1, 0, 0, ctypes.c_void_p(out.data_ptr()),
                                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    u = ints.to(torch.float64) / 2 ** 30
    v = 0.5 + (1 - torch.finfo(torch.float64).eps) * (u - 0.5)
    ref = torch.erfinv(2 * v - 1) * math.sqrt(2)
    err = (out.cpu().squeeze(0) - ref).abs() / ref.abs().clamp_min(1.0)
    i = int(err.argmax())
    assert err.max() < 4e-15, f"max err {err.max():.3e} at u={u[i].item()!r} z={ref[i].item()!r} got {out.cpu()[0, i].item()!r}"


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("n1,n2,d,outer,inner", [(13, 300, 50, 3, 2), (4, 4, 6, 16, 64), (256, 256, 50, 2, 1)])
def test_covar_batched_matches_torch(kind, n1, n2, d, outer, inner):
    """bo_covar_batched: per-(outer, inner) lengthscales / outputscales, X1 per
    inner member, X2 shared (the SAAS K*x and K** launches)."""
    from botorch_amd import kernels
    g = torch.Generator().manual_seed(n1 + n2 + d)
    X1 = torch.rand(inner, n1, d, generator=g, dtype=torch.float64)
    X2 = torch.rand(n2, d, generator=g, dtype=torch.float64)
    ls = 0.2 + torch.rand(outer, d, generator=g, dtype=torch.float64)
    os_ = 0.5 + torch.rand(outer, generator=g, dtype=torch.float64)
    K = torch.empty(outer, inner, n1, n2, dtype=torch.float64, device=DEV)
    kernels.covar_batched(kind, X1.to(DEV), (0, n1 * d), n1, X2.to(DEV), (0, 0), n2, d, ls.to(DEV),
                          (d, 0), os_.to(DEV), (1, 0), K, (inner * n1 * n2, n1 * n2), n2, outer, inner)
    r = torch.cdist(X1.unsqueeze(0) / ls.view(outer, 1, 1, d), (X2 / ls.view(outer, 1, d)).unsqueeze(1))
    if kind == 0:
        ref = torch.exp(-0.5 * r * r)
    else:
        s5 = math.sqrt(5.0) * r
        ref = (1 + s5 + s5 * s5 / 3) * torch.exp(-s5)
    ref = os_.view(outer, 1, 1, 1) * ref
    torch.testing.assert_close(K.cpu(), ref, rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("n,B,q,rq", [(4096, 512, 16, 1), (1000, 40, 4, 7), (300, 64, 16, 16)])
def test_post_partials_cross_term(n, B, q, rq):
    """Fused cross term Cx = Qc K*x^T (last column tile's workgroups) against
    Qc U R^T from the stored R^T; Spart / mpart unchanged by it."""
    from botorch_amd import kernels
    X, Y, orc, h = _oracle_model(n)
    c = _device_cache(X, Y, h, orc)
    g = torch.Generator().manual_seed(n + rq)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64).to(DEV)
    P = torch.zeros(rq, c.np, dtype=torch.float64)
    P[:, :n] = torch.randn(rq, n, generator=g, dtype=torch.float64)
    Qc = kernels.gemm(P.to(DEV), c.U, transB=True)            # rq x np = P U^T
    kc, _ = kernels.split_plan(B, q, n)
    ref = kernels.post_partials(c, Xc, store_R=True, split=0)
    pp = kernels.post_partials(c, Xc, split=0, cross=Qc)
    assert pp.Cx is not None and pp.Rt is None
    want = P.to(DEV) @ ref.Rt[: c.np]                          # P R^T
    torch.testing.assert_close(pp.Cx, want, rtol=1e-10, atol=1e-12)
    torch.testing.assert_close(pp.Spart, ref.Spart, rtol=0, atol=0)
    torch.testing.assert_close(pp.mpart, ref.mpart, rtol=0, atol=0)
    if kc:  # split-k plans fall back to R^T for the caller's GEMM
        sp = kernels.post_partials(c, Xc, cross=Qc)
        assert sp.Cx is None and sp.Rt is not None


def test_posterior_full_c3_matches_oracle():
    """The default C3 plan (n = 4096, 512 t-batches x q = 16: one pass, grouped
    8 x 8 super-tile schedule, K*x^T B operands from L2) on all 512 t-batches,
    checked against the oracle on t-batches from the first, middle and last
    super-tiles, and against the path that evaluates K*x inside the kernel."""
    from botorch_amd import _lib, kernels
    X, Y, orc, h = _oracle_model(4096)
    c = _device_cache(X, Y, h, orc)
    g = torch.Generator().manual_seed(11)
    Xc = torch.rand(512, 16, 6, generator=g, dtype=torch.float64)
    kc, _ = kernels.split_plan(512, 16, 4096)
    assert kc == 0
    pp = kernels.post_partials(c, Xc.to(DEV))
    out = kernels.qmc_finalize(c, pp, _lib.QMC_POSTERIOR, orc.ymean.item(), orc.ystd.item())
    idx = torch.tensor([0, 1, 7, 8, 255, 256, 300, 504, 510, 511])
    mr, cr = orc.posterior(Xc[idx])
    torch.testing.assert_close(out["mean"].cpu()[idx], mr, rtol=1e-4, atol=1e-9)
    torch.testing.assert_close(out["cov"].cpu()[idx], cr, rtol=1e-4, atol=1e-9)
    pe = kernels.post_partials(c, Xc.to(DEV), kxt=False)
    oe = kernels.qmc_finalize(c, pe, _lib.QMC_POSTERIOR, orc.ymean.item(), orc.ystd.item())
    torch.testing.assert_close(out["mean"], oe["mean"], rtol=1e-11, atol=1e-12)
    torch.testing.assert_close(out["cov"], oe["cov"], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("n", [37, 300, 1000, 4096])
def test_ainv_lower_tiles(n):
    """bo_ainv: A^{-1} = L^{-T} L^{-1} on the stream-K posterior tiles equals
    the GEMM of the cached inverse on every lower 128 x 128 tile (the part the
    MLL gradient reads), and the oracle's inverse at small n."""
    from botorch_amd import kernels
    X, Y, orc, h = _oracle_model(n)
    c = _device_cache(X, Y, h, orc)
    Ai = kernels.ainv(c)
    Li = c.Linv
    ref = Li.T @ Li
    tiles = torch.arange(n, device=Ai.device) // 128
    low = tiles.view(-1, 1) >= tiles.view(1, -1)  # the n x n block (the pad is not summed)
    Ai, ref = Ai[:n, :n], ref[:n, :n]
    torch.testing.assert_close(Ai[low], ref[low], rtol=1e-10, atol=1e-10 * float(ref.abs().max()))
    if n <= 1000:  # the oracle's (K + s2 I)^{-1} = L^{-T} L^{-1}
        want = orc.LinvT @ orc.LinvT.T
        lown = low.cpu()
        torch.testing.assert_close(Ai.cpu()[lown], want[lown], rtol=1e-7,
                                   atol=1e-9 * float(want.abs().max()))
