"""GPU parity of the dense float64 primitives (C-ABI through everest_amd.ops) against the
torch-CPU float64 oracle.  Tolerances: 1e-12 relative-to-scale for exact-arithmetic
restatements (GEMM, kernel assembly), 1e-10 for factorizations/solves."""
import os

import numpy as np
import pytest
import torch

from oracle import gp as ogp

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a):
    return torch.as_tensor(a, dtype=torch.float64, device=DEV)


@pytest.mark.parametrize("shape", [(1, 1, 1), (17, 33, 5), (64, 64, 64), (130, 70, 257), (513, 300, 129)])
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
def test_gemm_f64_mfma(shape, ta, tb):
    from everest_amd import ops

    M, N, K = shape
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    A = torch.randn(3, K, M, generator=g, dtype=torch.float64) if ta else torch.randn(3, M, K, generator=g, dtype=torch.float64)
    B = torch.randn(3, N, K, generator=g, dtype=torch.float64) if tb else torch.randn(3, K, N, generator=g, dtype=torch.float64)
    C0 = torch.randn(3, M, N, generator=g, dtype=torch.float64)
    ref = 1.5 * ((A.transpose(1, 2) if ta else A) @ (B.transpose(1, 2) if tb else B)) - 0.5 * C0
    C = _t(C0).contiguous()
    ops.gemm(_t(A), _t(B), ta, tb, alpha=1.5, beta=-0.5, out=C)
    err = (C.cpu() - ref).abs().max().item()
    assert err <= 1e-12 * max(1.0, ref.abs().max().item()) * max(1, K) ** 0.5


def test_gemm_asymmetric_identity():
    """A = I with an asymmetric B catches row/col swaps in the MFMA C/D map."""
    from everest_amd import ops

    B = torch.arange(64 * 48, dtype=torch.float64).reshape(64, 48)
    C = ops.gemm(_t(torch.eye(64)), _t(B))
    assert torch.equal(C.cpu(), B)


@pytest.mark.parametrize("kind", [0, 1, 2, 3])
@pytest.mark.parametrize("n1,n2,d", [(1, 1, 1), (37, 91, 6), (256, 256, 6), (130, 65, 32)])
def test_kernel_matrix(kind, n1, n2, d):
    from everest_amd import ops

    rng = np.random.default_rng(n1 + n2 + d + kind)
    X1 = rng.uniform(-1, 2, (n1, d))
    X2 = rng.uniform(-1, 2, (n2, d))
    ls = rng.uniform(0.2, 2.0, (3, d))
    lo, hi = -1.0 * np.ones(d), 2.0 * np.ones(d)
    os_ = np.array([1.0, 2.0, 0.5])
    K = ops.kernel_matrix(_t(X1), _t(X2), _t(ls), kind, shift1=_t(lo), scale1=_t(1 / (hi - lo)), shift2=_t(lo),
                          scale2=_t(1 / (hi - lo)), outputscale=_t(os_)).cpu()
    for b in range(3):
        ref = ogp.kernel_matrix(torch.tensor((X1 - lo) / (hi - lo)), torch.tensor((X2 - lo) / (hi - lo)),
                                torch.tensor(ls[b]), kind, os_[b])
        tol = 1e-13 if d < 16 else 1e-11     # d >= 16: matrix-core distance expansion (GPyTorch's sq_dist)
        assert torch.allclose(K[b], ref, rtol=1e-12, atol=tol)


@pytest.mark.parametrize("n", [1, 7, 32, 33, 100, 256, 513])
def test_cholesky_plain(n):
    from everest_amd import ops

    g = torch.Generator().manual_seed(n)
    A = torch.randn(4, n, n + 3, generator=g, dtype=torch.float64)
    A = A @ A.transpose(1, 2) + 1e-3 * torch.eye(n, dtype=torch.float64)
    L, jit, info = ops.cholesky(_t(A))
    ref = torch.linalg.cholesky(A)
    assert info.cpu().eq(0).all() and jit.cpu().eq(0).all()
    assert torch.allclose(L.cpu(), ref, rtol=1e-10, atol=1e-10 * ref.abs().max().item())


def test_cholesky_jitter_ladder():
    """Rank-deficient PSD matrices need jitter; singular-negative ones fail -> NotPSDError."""
    from everest_amd import ops

    g = torch.Generator().manual_seed(0)
    V = torch.randn(3, 40, 10, generator=g, dtype=torch.float64)
    A = V @ V.transpose(1, 2)                       # rank 10 < 40
    A[1] = A[1] + torch.eye(40, dtype=torch.float64)  # p.d.: no jitter
    L, jit, info = ops.cholesky(_t(A), 1e-8, 3, raise_on_fail=False)
    Lr, jr = ogp.psd_safe_cholesky(A)
    assert info.cpu().tolist() == [0, 0, 0]
    assert jit.cpu()[1].item() == 0.0
    assert torch.allclose(jit.cpu(), jr)
    assert torch.allclose(L.cpu(), Lr, atol=1e-8)
    neg = -torch.eye(5, dtype=torch.float64).unsqueeze(0)
    with pytest.raises(ops.NotPSDError):
        ops.cholesky(_t(neg))
    nan = torch.full((1, 4, 4), float("nan"), dtype=torch.float64)
    _, _, info = ops.cholesky(_t(nan), raise_on_fail=False)
    assert info.cpu().item() == 1


@pytest.mark.parametrize("n,nrhs", [(1, 1), (50, 3), (64, 64), (200, 130), (280, 512), (512, 17), (513, 70)])
@pytest.mark.parametrize("trans", [False, True])
def test_trsm_and_inverse(n, nrhs, trans):
    from everest_amd import ops

    g = torch.Generator().manual_seed(n + nrhs)
    A = torch.randn(2, n, n, generator=g, dtype=torch.float64)
    L = torch.linalg.cholesky(A @ A.transpose(1, 2) + n * torch.eye(n, dtype=torch.float64))
    B = torch.randn(2, n, nrhs, generator=g, dtype=torch.float64)
    X = _t(B).contiguous()
    ops.trsm(_t(L), X, transpose=trans)
    ref = torch.linalg.solve_triangular(L.transpose(1, 2) if trans else L, B, upper=trans)
    assert torch.allclose(X.cpu(), ref, rtol=1e-10, atol=1e-11)
    Li = ops.tri_inv(_t(L)).cpu()
    assert torch.allclose(Li, torch.linalg.inv(L), rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("d,kind", [(16, 0), (32, 3), (40, 1), (64, 2)])
def test_kernel_matrix_wide_mfma(d, kind):
    """d >= 16 runs the matrix-core distance expansion: symmetric (diagonal exactly k(0) +
    noise) and cross calls vs explicit differences in float64."""
    from everest_amd import ops

    rng = np.random.default_rng(d)
    n1, n2, B = 300, 130, 2
    lo, hi = np.zeros(d), np.full(d, 2.0)
    X1 = rng.uniform(0, 2, size=(n1, d))
    X2 = rng.uniform(0, 2, size=(n2, d))
    ls = rng.uniform(0.5, 2.0, size=(B, d))
    noise = np.array([1e-3, 2e-2])
    t = lambda a: torch.tensor(a, dtype=torch.float64, device="cuda")  # noqa: E731

    def ref(A, Bm, b):
        U = torch.tensor((A - lo) / (hi - lo) / ls[b]); V = torch.tensor((Bm - lo) / (hi - lo) / ls[b])
        d2 = ((U[:, None, :] - V[None, :, :]) ** 2).sum(-1)
        r = torch.sqrt(torch.clamp(d2, min=1e-30))
        if kind == 0:
            return torch.exp(-0.5 * d2)
        if kind == 1:
            return torch.exp(-r)
        if kind == 2:
            return (1 + 3 ** 0.5 * r) * torch.exp(-(3 ** 0.5) * r)
        return (1 + 5 ** 0.5 * r + 5.0 / 3.0 * d2) * torch.exp(-(5 ** 0.5) * r)

    inv = t(1.0 / (hi - lo))
    Ks = ops.kernel_matrix(t(X1), t(X1), t(ls), kind, shift1=t(lo), scale1=inv, shift2=t(lo), scale2=inv,
                           diag_add=t(noise)).cpu()
    Kc = ops.kernel_matrix(t(X1), t(X2), t(ls), kind, shift1=t(lo), scale1=inv, shift2=t(lo), scale2=inv).cpu()
    for b in range(B):
        Rs = ref(X1, X1, b) + noise[b] * torch.eye(n1, dtype=torch.float64)
        assert torch.allclose(Ks[b], Rs, rtol=1e-10, atol=1e-11)
        # zero distance on the diagonal: k(0) (kind 1 takes sqrt(1e-30) like GPyTorch) + noise to ~1 ulp;
        # a rounded expansion would leave d2 ~ 1e-15, i.e. r ~ 3e-8 there
        assert torch.allclose(torch.diagonal(Ks[b]), torch.diagonal(Rs), rtol=0, atol=2.0 ** -49)
        assert torch.allclose(Kc[b], ref(X1, X2, b), rtol=1e-10, atol=1e-11)


@pytest.mark.parametrize("n1,n2,d,kind", [(2048, 2048, 32, 3), (1100, 1900, 16, 0), (1030, 1090, 64, 1),
                                          (257, 1031, 32, 2)])
def test_kernel_matrix_wide_ragged_and_bounded(n1, n2, d, kind):
    """The matrix-core kernel-matrix kernel (d >= 16) at config 5's shape and ragged edges,
    called through the C-ABI into a buffer with a sentinel tail: nothing is written past the
    n1 x n2 matrix (out-of-range tile entries are computed on zero padding and not stored),
    every entry matches the float64 restatement, identical rows give the exact k(0) + noise."""
    from everest_amd import ops

    rng = np.random.default_rng(n1 + d)
    X1 = rng.uniform(0, 2, size=(n1, d))
    X2 = rng.uniform(0, 2, size=(n2, d))
    X2[: min(n1, n2) // 3] = X1[: min(n1, n2) // 3]          # identical rows on the diagonal tiles
    ls = rng.uniform(0.5, 2.0, size=(1, d))
    t = lambda a: torch.tensor(a, dtype=torch.float64, device="cuda")  # noqa: E731
    sh, sc, noise = t(np.zeros(d)), t(np.full(d, 0.5)), t([1e-3])
    buf = torch.full((n1 * n2 + 4096,), -7.0, dtype=torch.float64, device="cuda")   # sentinel tail
    x1, x2, lt = t(X1), t(X2), t(ls)
    ops.call("evr_kernel_matrix", ops._stream(), kind, 1, n1, n2, d, x1.data_ptr(), sh.data_ptr(), sc.data_ptr(),
             x2.data_ptr(), sh.data_ptr(), sc.data_ptr(), lt.data_ptr(), 0, noise.data_ptr(), buf.data_ptr())
    buf = buf.cpu()
    assert (buf[n1 * n2:] == -7.0).all()
    K = buf[: n1 * n2].view(n1, n2)
    U, V = torch.tensor(X1 * 0.5 / ls[0]), torch.tensor(X2 * 0.5 / ls[0])
    d2 = ((U[:, None, :] - V[None, :, :]) ** 2).sum(-1)
    r = torch.sqrt(torch.clamp(d2, min=1e-30))
    ref = {0: lambda: torch.exp(-0.5 * d2), 1: lambda: torch.exp(-r),
           2: lambda: (1 + 3 ** 0.5 * r) * torch.exp(-(3 ** 0.5) * r),
           3: lambda: (1 + 5 ** 0.5 * r + 5.0 / 3.0 * d2) * torch.exp(-(5 ** 0.5) * r)}[kind]()
    m = min(n1, n2)
    ref[torch.arange(m), torch.arange(m)] += 1e-3
    assert torch.allclose(K, ref, rtol=1e-10, atol=1e-11), float((K - ref).abs().max())
    k0 = {0: 1.0, 1: float(np.exp(-1e-15)), 2: None, 3: None}[kind]
    if k0 is not None:
        diag = torch.diagonal(K)[: m // 3]
        assert torch.allclose(diag, torch.full_like(diag, k0 + 1e-3), rtol=0, atol=2.0 ** -49)


@pytest.mark.parametrize("n,d,kind,norm", [(300, 16, 0, True), (300, 32, 3, False), (130, 64, 2, True),
                                           (2048, 32, 3, False), (65, 40, 1, True)])
def test_kernel_matrix_symmetric_tiles_bitwise(n, d, kind, norm):
    """K(X, X) through the lower-tile kernel (kmat_mfma_sym: each tile computed once, written
    in place and transposed; selected when both operands are the same tensor) equals the
    all-tiles kernel on a copy of X bitwise, and is exactly symmetric."""
    from everest_amd import ops

    rng = np.random.default_rng(n + d)
    B = 2
    X = torch.tensor(rng.uniform(0, 2, size=(n, d)), device="cuda")
    ls = torch.tensor(rng.uniform(0.5, 2.0, size=(B, d)), device="cuda")
    noise = torch.tensor([1e-3, 2e-2], device="cuda", dtype=torch.float64)
    kw = {}
    if norm:
        sh = torch.zeros(d, dtype=torch.float64, device="cuda")
        sc = torch.full((d,), 0.5, dtype=torch.float64, device="cuda")
        kw = dict(shift1=sh, scale1=sc, shift2=sh, scale2=sc)   # the same tensors: the symmetric path
    Ks = ops.kernel_matrix(X, X, ls, kind, diag_add=noise, **kw).cpu()
    Kf = ops.kernel_matrix(X, X.clone(), ls, kind, diag_add=noise, **kw).cpu()
    assert torch.equal(Ks, Kf)
    assert torch.equal(Ks, Ks.transpose(1, 2))


@pytest.mark.parametrize("variant", ["rl"])
@pytest.mark.parametrize("n", [64, 65, 130, 513, 1024])
def test_fused_cholesky_inverse_matches_torch_and_v1(n, variant, monkeypatch):
    """The one-launch-per-block Cholesky variants — "rl" (default: panel recomputed by every
    consumer, in-place panel pass at the end) — and the one-
    launch-per-row triangular inverse, against torch and against the three-launch-per-block
    v1 path."""
    from everest_amd import ops

    monkeypatch.setenv("EVR_CHOL", variant)
    g = torch.Generator().manual_seed(n)
    A = torch.randn(3, n, n + 5, generator=g, dtype=torch.float64)
    A = A @ A.transpose(1, 2) / n + 1e-2 * torch.eye(n, dtype=torch.float64)
    L, Li, jit, info = ops.cholesky_inverse(_t(A))
    ref = torch.linalg.cholesky(A)
    assert info.cpu().eq(0).all() and jit.cpu().eq(0).all()
    assert torch.allclose(L.cpu(), ref, rtol=1e-10, atol=1e-11 * ref.abs().max().item())
    assert torch.allclose(Li.cpu(), torch.linalg.inv(ref), rtol=1e-8, atol=1e-9 * torch.linalg.inv(ref).abs().max().item())
    assert torch.equal(torch.triu(L, 1).cpu(), torch.zeros_like(ref)) and torch.equal(torch.triu(Li, 1).cpu(), torch.zeros_like(ref))
    monkeypatch.setenv("EVR_CHOL", "v1")
    L1, Li1, _, _ = ops.cholesky_inverse(_t(A))
    assert torch.allclose(L, L1, rtol=1e-12, atol=1e-13 * ref.abs().max().item())
    assert torch.allclose(Li, Li1, rtol=1e-10, atol=1e-11 * Li1.abs().max().item())


@pytest.mark.parametrize("variant", ["rl", "v1"])
def test_fused_cholesky_failure_and_ladder(variant, monkeypatch):
    """A member failing in a late diagonal block reports a pivot index past block 2 and gets
    the psd_safe_cholesky per-member jitter."""
    from everest_amd import ops

    monkeypatch.setenv("EVR_CHOL", variant)
    g = torch.Generator().manual_seed(3)
    V = torch.randn(2, 200, 150, generator=g, dtype=torch.float64)
    A = V @ V.transpose(1, 2)                      # rank 150 of 200: fails past block 2
    A[0] = A[0] + torch.eye(200, dtype=torch.float64)
    _, _, info = ops.cholesky(_t(A), 1e-8, 0, raise_on_fail=False)
    inf = info.cpu().tolist()
    assert inf[0] == 0 and (inf[1] == 0 or inf[1] > 128)
    L, jit, info = ops.cholesky(_t(A), 1e-8, 3, raise_on_fail=False)
    Lr, jr = ogp.psd_safe_cholesky(A)
    assert torch.allclose(jit.cpu(), jr)
    assert torch.allclose(L.cpu(), Lr, atol=1e-7)


def test_trsm16_matches_torch_solve():
    """The 16-column forward substitution (n <= 512, the qNEHVI baseline solve G = L_b^-1 E)
    against torch's triangular solve, and the 64-column tile kernel (the transposed solve)."""
    from everest_amd import ops

    g = torch.Generator().manual_seed(7)
    n, nrhs = 280, 96
    A = torch.randn(3, n, n, generator=g, dtype=torch.float64)
    L = torch.linalg.cholesky(A @ A.transpose(1, 2) + 1e-3 * torch.eye(n, dtype=torch.float64))
    B = torch.randn(3, n, nrhs, generator=g, dtype=torch.float64)
    X = _t(B).contiguous()
    ops.trsm(_t(L), X)
    ref = torch.linalg.solve_triangular(L, B, upper=False)
    assert torch.allclose(X.cpu(), ref, rtol=1e-9, atol=1e-9 * ref.abs().max())


@pytest.mark.parametrize("n", [16, 64, 65, 130, 280, 512, 513, 1024])
def test_tri_inv_col_bitwise_equals_row_kernel(n, monkeypatch):
    """The one-launch 16-column-panel triangular inverse (n <= 1024, the GP fit's L^-1) runs
    tri_inv_row_kernel's accumulation sequence per element: bitwise equal to the per-block-row
    launches (EVR_TRIINV=row), including ragged n and the zero upper triangle."""
    from everest_amd import ops

    g = torch.Generator().manual_seed(n + 11)
    A = torch.randn(5, n, n + 3, generator=g, dtype=torch.float64)
    A = _t(A @ A.transpose(1, 2) / n + 1e-2 * torch.eye(n, dtype=torch.float64))
    monkeypatch.setenv("EVR_TRIINV", "col")
    L, Li, _, info = ops.cholesky_inverse(A)
    monkeypatch.setenv("EVR_TRIINV", "row")
    L0, Li0, _, info0 = ops.cholesky_inverse(A)
    assert info.cpu().eq(0).all() and info0.cpu().eq(0).all()
    assert torch.equal(L, L0)
    assert torch.equal(Li, Li0)
    Lc = L.cpu()
    eye = torch.eye(n, dtype=torch.float64).expand(5, n, n)
    assert torch.allclose(Li.cpu() @ Lc, eye, atol=1e-8)


@pytest.mark.parametrize("n", [16, 64, 65, 130, 280, 512, 513, 1024])
def test_fused_inverse_matches_separate(n, monkeypatch):
    """The inverse formed right-looking inside the Cholesky launches (B_ij -= L_ik Dinv_k B_kj
    beside each step's trailing tiles, X_kj = Dinv_k B_kj at the end): the factor is bitwise
    the separate path's, the inverse agrees to rounding (another summation order) and has
    the zero upper triangle; ragged n included."""
    from everest_amd import ops

    g = torch.Generator().manual_seed(n + 29)
    A = torch.randn(5, n, n + 3, generator=g, dtype=torch.float64)
    A = _t(A @ A.transpose(1, 2) / n + 1e-2 * torch.eye(n, dtype=torch.float64))
    monkeypatch.delenv("EVR_TRIINV", raising=False)
    L, Li, _, info = ops.cholesky_inverse(A)
    monkeypatch.setenv("EVR_TRIINV", "col")
    L0, Li0, _, info0 = ops.cholesky_inverse(A)
    assert info.cpu().eq(0).all() and info0.cpu().eq(0).all()
    assert torch.equal(L, L0)
    err = float((Li - Li0).abs().max() / Li0.abs().max())
    assert err <= 1e-12, err
    assert torch.equal(torch.triu(Li, 1), torch.zeros_like(Li))
    eye = torch.eye(n, dtype=torch.float64).expand(5, n, n)
    assert torch.allclose(Li.cpu() @ L.cpu(), eye, atol=1e-8)
