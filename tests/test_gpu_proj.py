"""GPU: fused qNEHVI projection path (qnehvi_proj.hip) vs the unfused kernels on the same
state: R = M Kx, partial-norm sampling vs evr_qnehvi_samples, and the backward GEMM with
generated gR vs evr_qnehvi_samples_backward + M^T gR."""
import numpy as np
import pytest
import torch

from tests.helpers import device_gp, make_problem

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,d,m,S,b", [(120, 6, 5, 64, 200), (70, 4, 3, 40, 33), (40, 3, 2, 17, 1)])
def test_fused_projection_matches_unfused(n, d, m, S, b):
    from everest_amd import ops
    from everest_amd.acquisition import QNEHVI

    X, Y, lo, hi, hyp = make_problem(n=n, d=d, m=m, seed=n + b)
    gp = device_gp(X, Y, lo, hi, hyp)
    q = QNEHVI(gp, X, X, -1.1 * np.ones(m), -np.ones(m), np.zeros(m), S=S, sampler_seed=3, prune_baseline=True,
               prune_seed=4, prune_samples=256)
    st = q.state
    Xc = torch.tensor(lo + (hi - lo) * np.random.default_rng(b).uniform(size=(b, d)), device="cuda")
    Kx = gp.cross(Xc)
    R0 = ops.gemm(q.M, Kx)
    G0, L0, f0 = ops.qnehvi_samples(st, R0, b)
    R1, P = ops.qnehvi_project(st, q.M, Kx, b)
    G1, L1, f1 = ops.qnehvi_samples_norms(st, R1, P, b)
    assert torch.allclose(R1, R0, rtol=1e-12, atol=1e-13 * R0.abs().max().item())   # GEMM backends round differently
    assert torch.equal(f0, f1)
    assert torch.allclose(L1, L0, rtol=1e-9, atol=1e-12)
    assert torch.allclose(G1, G0, rtol=1e-10, atol=1e-12)
    dG = torch.randn(G0.shape, dtype=torch.float64, device="cuda", generator=torch.Generator("cuda").manual_seed(1))
    gR = ops.qnehvi_samples_backward(st, R0, L0, dG, b)
    dK0 = ops.gemm(q.M, gR, transA=True)
    dK1 = ops.qnehvi_project_backward(st, q.M, R1, L1, dG, b)
    scale = dK0.abs().max()
    assert torch.allclose(dK1, dK0, rtol=1e-8, atol=1e-11 * scale)


@pytest.mark.parametrize("graph", [True, False])
def test_native_plan_matches_op_chain(graph, monkeypatch):
    """evr_qnehvi_plan (one C-ABI call, hipGraph replay) == the op-by-op chain, bitwise (same
    kernels, same order, deterministic reductions); repeated runs reuse the captured graph."""
    from everest_amd.acquisition import QNEHVI

    monkeypatch.setenv("EVR_GRAPH", "1" if graph else "0")
    n, d, m, S = 90, 5, 4, 48
    X, Y, lo, hi, hyp = make_problem(n=n, d=d, m=m, seed=33)
    gp = device_gp(X, Y, lo, hi, hyp)
    q = QNEHVI(gp, X, X, -1.1 * np.ones(m), -np.ones(m), np.zeros(m), S=S, sampler_seed=5, prune_baseline=True,
               prune_seed=6, prune_samples=256)
    rng = np.random.default_rng(0)
    for b in (20, 20, 130, 1):
        Xc = torch.tensor(lo + (hi - lo) * rng.uniform(size=(b, d)), device="cuda")
        a0, g0 = q.forward_backward_ops(Xc)
        a1, g1 = q.forward_backward(Xc)
        if b <= 32:
            # restart batches run the M-streaming small-batch kernels (qnehvi_small.hip): the
            # same algebra in a different summation order
            assert torch.allclose(a1, a0, rtol=1e-10, atol=1e-13 * a0.abs().max())
            assert torch.allclose(g1, g0, rtol=1e-8, atol=1e-11 * g0.abs().max())
            assert torch.allclose(q.forward(Xc), q.forward_ops(Xc), rtol=1e-10, atol=1e-13 * a0.abs().max())
            a0, g0 = a1, g1
        else:
            assert torch.equal(a0, a1) and torch.equal(g0, g1)
            assert torch.equal(q.forward(Xc), q.forward_ops(Xc))
        ah, gh = q.eval_host(Xc.cpu().numpy(), True)
        assert np.array_equal(ah, a0.cpu().numpy()) and np.array_equal(gh, g0.cpu().numpy())


@pytest.mark.parametrize("split", [False, True])
def test_small_batch_kernels_match_tile_path(split, monkeypatch):
    """b <= 32: qs_fwd / qs_bwd (M-streaming, K_x staged in LDS, cross-gradient in the
    epilogue) against the 64 x 64-tile path (EVR_SMALL=0) on the same acquisition, for the
    fused-root and the split (L^-1; G; H^T; alpha^T) operator layouts."""
    from everest_amd.acquisition import QNEHVI

    n, d, m, S = 150, 6, 3, 64
    X, Y, lo, hi, hyp = make_problem(n=n, d=d, m=m, seed=21)
    gp = device_gp(X, Y, lo, hi, hyp)
    q = QNEHVI(gp, X, X, -1.1 * np.ones(m), -np.ones(m), np.zeros(m), S=S, sampler_seed=2, prune_baseline=True,
               prune_seed=3, prune_samples=256, root="split" if split else "fused")
    rng = np.random.default_rng(1)
    for b in (1, 7, 20, 32):
        Xc = torch.tensor(lo + (hi - lo) * rng.uniform(size=(b, d)), device="cuda")
        q._plans = {}
        monkeypatch.setenv("EVR_SMALL", "0")
        a0, g0 = q.forward_backward(Xc)
        f0 = q.forward(Xc)
        q._plans = {}
        monkeypatch.setenv("EVR_SMALL", "1")
        a1, g1 = q.forward_backward(Xc)
        f1 = q.forward(Xc)
        assert torch.allclose(a1, a0, rtol=1e-10, atol=1e-13 * a0.abs().max()), (a1 - a0).abs().max()
        assert torch.allclose(f1, f0, rtol=1e-10, atol=1e-13 * a0.abs().max())
        assert torch.allclose(g1, g0, rtol=1e-8, atol=1e-11 * g0.abs().max()), (g1 - g0).abs().max()
        a2, g2 = q.forward_backward(Xc)                 # repeat: bitwise
        assert torch.equal(a2, a1) and torch.equal(g2, g1)


def test_small_batch_ops_equal_plan():
    """The b <= 32 pieces exposed through the C-ABI (evr_qnehvi_small_forward / _samples /
    _backward, what bench.py times per op) chained by hand give the plan's values bitwise."""
    from everest_amd import ops
    from everest_amd.acquisition import QNEHVI

    n, d, m, S = 120, 5, 3, 256
    X, Y, lo, hi, hyp = make_problem(n=n, d=d, m=m, seed=23)
    gp = device_gp(X, Y, lo, hi, hyp)
    q = QNEHVI(gp, X, X, -1.1 * np.ones(m), -np.ones(m), np.zeros(m), S=S, sampler_seed=2, prune_seed=3,
               prune_samples=256)
    Xc = torch.tensor(lo + (hi - lo) * np.random.default_rng(4).uniform(size=(13, d)), device="cuda")
    b = Xc.shape[0]
    st, md = q.state, q.model
    assert ops.qnehvi_small_applies(st, b, d)
    Kx = gp.cross(Xc)
    R, P = ops.qnehvi_small_forward(st, md, Kx, b)
    G, L22, flags = ops.qnehvi_small_samples(st, R, P, b)
    # the plan's restart scan is the one-launch kernel (hvi_kdb: equal to the three-launch
    # chain's dG to rounding), its acq the sample mean formed inside the dX reduction
    assert ops.hvi_restart_fb_applies(st, b)
    acq, dG = ops.hvi_forward_backward(st, G, b, flags)
    sval, dG3 = ops.hvi_restart_fb(st, G, b)
    assert torch.allclose(dG3, dG, rtol=1e-12, atol=1e-15 * dG.abs().max().item())
    dX = ops.qnehvi_small_backward(st, md, Xc, R, L22, dG3, b)
    a_ref, g_ref = q.forward_backward(Xc)
    assert torch.equal(dX, g_ref)
    assert torch.allclose(acq, a_ref, rtol=1e-12, atol=0) and torch.allclose(ops.mean_over_samples(sval), a_ref,
                                                                               rtol=1e-14, atol=0)


def test_restart_chain_is_batch_invariant():
    """The whole b <= 32 evaluation chain (kernel matrix, projection, fused sampling + wave scan,
    backward, dX reduction) gives every candidate bitwise the same value and gradient whether
    it is evaluated in the full restart batch or in a slice of it (what a rank of the sharded
    joint restart problem evaluates, optim._Shard)."""
    from everest_amd.acquisition import QNEHVI

    n, d, m, S = 120, 5, 3, 256
    X, Y, lo, hi, hyp = make_problem(n=n, d=d, m=m, seed=29)
    gp = device_gp(X, Y, lo, hi, hyp)
    q = QNEHVI(gp, X, X, -1.1 * np.ones(m), -np.ones(m), np.zeros(m), S=S, sampler_seed=2, prune_seed=3,
               prune_samples=256)
    Xc = lo + (hi - lo) * np.random.default_rng(6).uniform(size=(20, d))
    a, g = q.eval_host(Xc, True)
    for sl in (slice(0, 10), slice(10, 20), slice(3, 10)):
        a2, g2 = q.eval_host(Xc[sl], True)
        assert np.array_equal(a2, a[sl]) and np.array_equal(g2, g[sl])


def test_restart_backward_device_and_host_chains_equal():
    """The restart backward's training-row classes (qs_tail.hpp: the split root's L^-1 and G
    rows, weighted into one class; the fused root's C rows) run as the backward launch's own
    workgroups: the device chain and the host-driven evaluation are bitwise equal for both
    roots, and the two roots agree to the cancellation-free rounding of this state."""
    from everest_amd.acquisition import QNEHVI

    n, d, m, S = 90, 5, 4, 48
    X, Y, lo, hi, hyp = make_problem(n=n, d=d, m=m, seed=35)
    gp = device_gp(X, Y, lo, hi, hyp)
    Xc = torch.tensor(lo + (hi - lo) * np.random.default_rng(3).uniform(size=(20, d)), device="cuda")
    out = {}
    for root in ("split", "fused"):
        q = QNEHVI(gp, X, X, -1.1 * np.ones(m), -np.ones(m), np.zeros(m), S=S, sampler_seed=5, prune_baseline=True,
                   prune_seed=6, prune_samples=256, root=root)
        a, g = q.forward_backward(Xc)
        ah, gh = q.eval_host(Xc.cpu().numpy(), True)
        assert np.array_equal(ah, a.cpu().numpy()) and np.array_equal(gh, g.cpu().numpy())
        out[root] = (a, g)
    a0, g0 = out["split"]
    assert torch.allclose(out["fused"][0], a0, rtol=1e-7, atol=1e-12)
    assert torch.allclose(out["fused"][1], g0, rtol=1e-5, atol=1e-8 * g0.abs().max())