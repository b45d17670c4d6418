"""Oracle parity at the BASELINE.json sizes themselves (not only at small n).

* configs[2]: DTLZ2(d=6, m=5), n_train=512, S=256, prune over
  2048 draws, b=512 candidates — the exact state bench.py measures.  The oracle (torch-CPU
  fp64, BoTorch's computation shape) prunes, decomposes all 256 samples into cells with its
  own Python partition and evaluates qNEHVI + autograd on a subset of the same candidates;
  the device runs the whole 512-candidate batch through the native plan (kd2 sparse scan,
  12-bit key fields at m=5, ~6k cells per sample, 769-row fused root).
* configs[4] (config 5): 4 continuous + 4x7 one-hot (d_eff=32), Matérn-5/2 ARD,
  n_train=2048, qEI: Cholesky(2048) vs LAPACK, posterior moments vs the oracle, qEI
  forward + backward vs oracle autograd.

Tolerances are the ones the smaller parity tests use (north star: 1e-4 posterior, 1e-3
qNEHVI); the oracle's own parity against BoTorch is unpinned (oracle/__init__.py).
"""
import numpy as np
import pytest
import torch

from oracle import gp as ogp
from oracle import qnehvi as oq

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def config3():
    import bench

    dev = torch.device("cuda", 0)
    n, d, m, S = 512, 6, 5, 256
    X, Y, gp, hypers, acqf, _, _ = bench.build_state(n, d, m, S, dev)
    states = []
    Xn = torch.tensor(X)
    for j, h in enumerate(hypers):
        y = torch.tensor(Y[:, j])
        states.append(ogp.GPState(X=Xn, y=(y - h.y_mean) / h.y_std, lengthscale=torch.tensor(h.lengthscale),
                                  noise=h.noise, constant=h.constant, y_mean=h.y_mean, y_std=h.y_std))
    objective = oq.Objective(-torch.ones(m, dtype=torch.float64), torch.zeros(m, dtype=torch.float64))
    ref = torch.full((m,), -1.1, dtype=torch.float64)
    return dict(X=X, Xn=Xn, acqf=acqf, states=states, objective=objective, ref=ref, n=n, d=d, m=m, S=S, dev=dev)


def test_config3_prune_matches_oracle(config3):
    """prune_baseline over 2048 Sobol-normal draws (seed 4321, bench.build_state)."""
    c = config3
    zp = oq.base_samples(2048, c["n"], c["m"], 4321)
    idx, probs = oq.prune_baseline(c["states"], c["Xn"], c["objective"], c["ref"], zp, chunk=32)
    assert np.array_equal(np.sort(c["acqf"].base_rows), idx.numpy())
    dp = np.asarray(c["acqf"].stats.prune_probs)
    # identical draws; a dominance test may flip only on an exact tie of rounded samples
    assert np.abs(dp - probs.numpy()).max() <= 1.0 / 2048


@pytest.fixture(scope="module")
def oracle3(config3):
    """The oracle's qNEHVI at the bench state, with its own 256 Python partitions (built once)."""
    c = config3
    acqf, m, S = c["acqf"], c["m"], c["S"]
    nb = acqf.nb
    idx = torch.as_tensor(np.sort(acqf.base_rows))
    zb = oq.base_samples(S, nb, m, 1234)
    zn = oq.base_samples(S, nb + 1, m, 1234)[:, nb:nb + 1]
    orc = oq.QNEHVI(c["states"], c["Xn"][idx], c["objective"], c["ref"], zb, zn)
    return dict(orc=orc, idx=idx, zb=zb, zn=zn)


def test_config3_qnehvi_values_and_grads_match_oracle(config3, oracle3):
    import bench

    c = config3
    acqf = c["acqf"]
    orc = oracle3["orc"]
    assert acqf.stats.total_cells == sum(cc.shape[1] for cc in orc.cells)
    assert acqf.stats.max_cells == max(cc.shape[1] for cc in orc.cells)

    Xc = bench.candidates(512, c["d"], seed=2, device=c["dev"])
    acq, dX = acqf.forward_backward(Xc)            # b = 512 through the native plan
    sub = torch.arange(0, 512, 32)                 # 16 candidates checked against the oracle
    xt = Xc.cpu()[sub].clone().requires_grad_(True)
    ref = orc.forward(xt.unsqueeze(1))
    ref.sum().backward()
    a = acq.cpu()[sub]
    assert (ref.detach() > 0).sum() >= 4           # the subset exercises non-zero improvements
    assert torch.allclose(a, ref.detach(), rtol=1e-6, atol=1e-10), (a, ref)
    g = dX.cpu()[sub]
    scale = xt.grad.abs().max()
    assert torch.allclose(g, xt.grad, rtol=1e-5, atol=1e-7 * scale), (g - xt.grad).abs().max()


def test_config3_batch_split_equals_full_batch(config3):
    """The 512-candidate plan against 20-candidate plans (the L-BFGS restart size) on the
    same candidates: equal up to the summation-order rounding of the different GEMM /
    split-K reductions the two batch sizes select (f64: ~1e-15 relative on R).  That rounding
    is amplified by the cancellation in L22^2 = s^2 (kxx - |R|^2) next to training points:
    where 1 - |R|^2 / kxx falls to ~1e-11 the computed L22^2 (R's absolute rounding ~1e-9 at
    the bench state's ~1e4 operator entries) is noise, and either path may land below zero
    and take the psd_safe floor (tools/diag_split.py: exact L22 1e-6, one path 1e-6, the
    other 1e-4) — the reference's own Cholesky of the joint covariance rounds the same way.
    Those candidates (one path's L22 an order of magnitude off the other's in some output)
    are held to the north-star bar, 1e-3 of the batch's largest value; every other
    candidate to 1e-7 (measured 1.6e-11 absolute on values up to ~1e-2)."""
    import bench
    from everest_amd import ops

    c = config3
    acqf = c["acqf"]
    Xc = bench.candidates(512, c["d"], seed=3, device=c["dev"])
    a_full, g_full = acqf.forward_backward(Xc)
    parts = [acqf.forward_backward(Xc[i:i + 20]) for i in range(0, 500, 20)]
    a_p = torch.cat([p[0] for p in parts])
    g_p = torch.cat([p[1] for p in parts])
    # the two paths' posterior root L22 per (output, candidate)
    st, Kx = acqf.state, acqf._cross(Xc)
    RA, PA = ops.qnehvi_project(st, acqf.M, Kx, 512)
    _, LA, _ = ops.qnehvi_samples_norms(st, RA, PA, 512)
    LB = []
    for i in range(0, 500, 20):
        RB, PB = ops.qnehvi_small_forward(st, acqf.model, Kx[:, :, i:i + 20].contiguous(), 20)
        LB.append(ops.qnehvi_small_samples(st, RB, PB, 20)[1])
    LB = torch.cat(LB, 1)
    # one path at the psd floor and the other not: their L22 differ by orders of magnitude
    # (the rounding noise of an unclamped L22 is ~10 % at the bench state's smallest variances)
    la, lb = LA[:, :500].abs(), LB.abs()
    ill = (torch.maximum(la, lb) > 10.0 * torch.minimum(la, lb)).any(0)
    well = ~ill
    amax = a_full.abs().max().item()
    da = (a_full[:500] - a_p).abs()
    print(f"batch split: {int(ill.sum())} cancellation-bound candidates; max |diff| well-conditioned "
          f"{float(da[well].max()):.3e}, all {float(da.max()):.3e}")
    assert torch.allclose(a_full[:500][well], a_p[well], rtol=1e-7, atol=1e-7 * amax), float(da[well].max())
    assert float(da.max()) <= 1e-3 * amax, float(da.max())
    assert int(ill.sum()) <= 50, int(ill.sum())   # a handful next to training points, not a drift
    scale = g_full.abs().max().item()
    dg = (g_full[:500] - g_p).abs()
    assert torch.allclose(g_full[:500][well], g_p[well], rtol=1e-6, atol=1e-6 * scale), float(dg[well].max())


def test_config3_qlognehvi_values_and_grads_match_oracle(config3, oracle3):
    """qLogNEHVI (MoboStrategy's default) at the BASELINE state: same GPs, prune / sampler
    seeds, pruned baseline and partitions as the qNEHVI bench state; the b = 20 restart batch
    (all 20 candidates) and a 16-candidate subset of a b = 512 batch against the oracle's
    fat-smoothed log HVI and its autograd gradients."""
    import bench
    from everest_amd import ops
    from everest_amd.acquisition import QLogNEHVI

    c = config3
    acqf, m, S = c["acqf"], c["m"], c["S"]
    qa = QLogNEHVI(acqf.gp, c["X"], c["X"], -1.1 * np.ones(m), -np.ones(m), np.zeros(m), S=S, sampler_seed=1234,
                   prune_baseline=True, prune_seed=4321)
    assert np.array_equal(np.sort(qa.base_rows), oracle3["idx"].numpy())
    assert qa.stats.total_cells == acqf.stats.total_cells
    olog = oq.QLogNEHVI(c["states"], c["Xn"][oracle3["idx"]], c["objective"], c["ref"], oracle3["zb"],
                        oracle3["zn"], cells=oracle3["orc"].cells)
    for b, sub in ((20, torch.arange(20)), (512, torch.arange(0, 512, 32))):
        Xc = bench.candidates(b, c["d"], seed=2, device=c["dev"])
        acq, dX = qa.forward_backward(Xc)
        xt = Xc.cpu()[sub].clone().requires_grad_(True)
        ref = olog.forward(xt.unsqueeze(1))
        ref.sum().backward()
        assert torch.isfinite(acq).all() and torch.isfinite(ref).all()
        a = acq.cpu()[sub]
        r = ref.detach()
        # log values: an absolute error e in log space is a relative error e in the HVI itself.
        # North-star bar (1e-3 relative on qNEHVI values) for EVERY candidate, whatever its
        # HVI; candidates with HVI > 1e-6 (log HVI > -14, where the ~1e-13 absolute rounding of
        # the L22^2 = var - |L21|^2 cancellation is below 1e-6 relative) are held to 1e-6
        err = (a - r).abs()
        worst = int(err.argmax())
        print(f"qlog b={b}: max |d log| {float(err.max()):.3e} at log HVI {float(r[worst]):.2f}; "
              f"min log HVI {float(r.min()):.2f}")
        assert (err <= 1e-3).all(), (b, [(float(x), float(y)) for x, y, bad in zip(a, r, err > 1e-3) if bad])
        # the 1e-6 class also leaves out candidates whose new-point variance given the
        # baseline's samples (L22^2 = s^2 (kxx - |R|^2), R = C k through the fused root) has
        # cancelled to below 1e-6 of the prior in some output: R's entries carry ~1e-12 absolute
        # rounding (C's entries are ~1e4-1e5 at this state), so the computed L22^2 carries
        # ~2e-12 of s^2 kxx — over 1e-6 of itself there, and device and oracle round it
        # differently (tools/qlog_diag.py: the qNEHVI values of such a candidate differ by the
        # same 5.6e-4 as its log values).  Which candidates these are moves with the fitted state
        Xs = Xc[sub.to(Xc.device)].contiguous()
        R, P = ops.qnehvi_small_forward(qa.state, qa.model, qa.gp.cross(Xs), Xs.shape[0])
        L22 = ops.qnehvi_small_samples(qa.state, R, P, Xs.shape[0])[1]
        rel = (L22 ** 2 / (qa.gp.ys[:, None] ** 2 * qa.gp.kxx[:, None])).min(0).values.cpu()
        well = (r > -14.0) & (rel > 1e-6)
        print(f"qlog b={b}: {int(((r > -14.0) & (rel <= 1e-6)).sum())} candidates with log HVI > -14 at the "
              f"cancelled-variance floor (held to 1e-3 only)")
        assert (err[well] <= 1e-6).all(), (b, [(float(x), float(y)) for x, y, e in zip(a[well], r[well], err[well])
                                               if e > 1e-6])
        # gradients: the backward contracts the fused root C = Lv^T L^-1 (entries ~1e4-1e5 at
        # this state) against gR, so each dK entry is an O(1) sum of O(1e5) terms and carries
        # ~1e-11 absolute rounding whatever the summation order; through d log HVI / dx =
        # (d HVI / dx) / HVI and the 1 / L22 of the new-point root that reaches a few 1e-5 of a
        # candidate's gradient scale (measured 1.2e-5 on the b = 512 path; the oracle's own
        # Cholesky-solve path rounds differently).  Held to 1e-4 of each candidate's gradient
        # scale where the new-point variance has not cancelled (rel > 1e-6, as above), 1e-3 where
        # it has cancelled to 1e-8 .. 1e-6 of the prior but the HVI is not negligible (log HVI
        # > -14); below that the rounding of L22^2 reaches the gradient through 1 / L22 (a
        # candidate at rel = 7e-9 in one output differs by a few 1e-2 of its gradient scale at
        # one fitted state), and so does the fat-smoothed tail of a zero-HVI candidate: only
        # finite there
        g = dX.cpu()[sub]
        gr = xt.grad
        row_err = (g - gr).abs().amax(1) / gr.abs().amax(1).clamp_min(1e-300)
        tight = rel > 1e-6
        mid = ~tight & (rel > 1e-8) & (r > -14.0)
        for name, sel, bar in (("tight", tight, 1e-4), ("mid", mid, 1e-3)):
            if int(sel.sum()):
                print(f"qlog b={b}: {name}: {int(sel.sum())} candidates, max row-relative gradient error "
                      f"{float(row_err[sel].max()):.3e}")
                assert (row_err[sel] <= bar).all(), (b, name, row_err)
        print(f"qlog b={b}: max row-relative gradient error, all candidates {float(row_err.max()):.3e}")
        assert torch.isfinite(g).all()


@pytest.fixture(scope="module")
def config5():
    import everest_amd.data_models as dm
    from everest_amd import strategies
    from tests.helpers import mixed_domain, mixed_f

    dom = mixed_domain()
    X = strategies.map(dm.RandomStrategy(domain=dom, seed=13)).ask(2048)
    exps = X.copy()
    exps["y"] = mixed_f(X)
    exps["valid_y"] = 1
    spec = dm.SingleTaskGPSurrogate(inputs=dom.inputs, outputs=dom.outputs, kernel=dm.MaternKernel(nu=2.5))
    s = strategies.map(dm.SoboStrategy(domain=dom, acquisition_function=dm.qEI(), seed=1,
                                       surrogate_specs=dm.BotorchSurrogates(surrogates=[spec]),
                                       categorical_method="FREE", num_raw_samples=256, num_restarts=4))
    s.tell(exps)
    st = s.surrogates.surrogates[0].state
    Xn = torch.tensor((st["X"] - st["lo"]) / (st["hi"] - st["lo"]))
    o = ogp.GPState(X=Xn, y=torch.tensor((st["y"] - st["y_mean"]) / st["y_std"]),
                    lengthscale=torch.tensor(st["lengthscale"]), noise=st["noise"], constant=st["constant"],
                    y_mean=st["y_mean"], y_std=st["y_std"], kind=ogp.MATERN25)
    return dict(s=s, st=st, o=o, Xn=Xn, d=Xn.shape[1])


def test_config5_cholesky_2048(config5):
    from everest_amd import ops

    gp = config5["s"].model
    assert gp.Xn.shape == (2048, 32)
    K = ops.kernel_matrix(gp.Xn, gp.Xn, gp.ls, gp.kind, diag_add=gp.noise)
    L, jit, info = ops.cholesky(K)
    Kc = K.cpu()
    ref = torch.linalg.cholesky(Kc[0])
    assert int(info.cpu()[0]) == 0 and float(jit.cpu()[0]) == 0.0
    assert torch.allclose(L.cpu()[0], ref, rtol=1e-9, atol=1e-11)
    # the oracle's own kernel matrix (sq-dist expansion, GPyTorch form) at d_eff = 32
    Ko = ogp.kernel_matrix(config5["Xn"], config5["Xn"], config5["o"].lengthscale, ogp.MATERN25)
    Ko = Ko + config5["o"].noise * torch.eye(2048, dtype=torch.float64)
    # GPyTorch's expansion |x|^2 + |x'|^2 - 2 x.x' of the scaled inputs loses ~eps * |x/ls|^2
    # to cancellation (the device forms the differences explicitly); the fitted one-hot
    # lengthscales can be ~1e-4, so the bound scales with sum_k 1/ls_k^2
    err = (Kc[0] - Ko).abs()
    k = int(err.argmax())
    i, j = divmod(k, 2048)
    canc = 8 * 2.2e-16 * float((1.0 / config5["o"].lengthscale ** 2).sum())
    assert torch.allclose(Kc[0], Ko, rtol=1e-10, atol=max(1e-11, canc)), (err.max().item(), i, j, canc)


def test_config5_posterior_matches_oracle(config5):
    s, o, st = config5["s"], config5["o"], config5["st"]
    rng = np.random.default_rng(4)
    Xs = rng.uniform(size=(300, config5["d"]))
    Xs[:, 4:] = (Xs[:, 4:] > 0.8).astype(np.float64)      # one-hot-like columns
    Xs[:20] = st["X"][:20]                                 # on training points
    for obs in (False, True):
        mean, var = s.model.posterior(torch.tensor(Xs, device="cuda"), observation_noise=obs)
        rm, rv = ogp.posterior(o, torch.tensor((Xs - st["lo"]) / (st["hi"] - st["lo"])), observation_noise=obs)
        assert torch.allclose(mean[0].cpu(), rm, rtol=1e-4, atol=1e-6 * o.y_std), (mean[0].cpu() - rm).abs().max()
        assert torch.allclose(var[0].cpu(), rv, rtol=1e-4, atol=1e-8 * o.y_std ** 2), (var[0].cpu() - rv).abs().max()


def test_config5_qei_matches_oracle(config5):
    s, o = config5["s"], config5["o"]
    acqf = s._get_acqfs(1)[0]
    st = config5["st"]
    rm, _ = ogp.posterior(o, config5["Xn"])
    best_f = float((-rm).max())
    # posterior mean at 2048 training points through K^-1 (noise ~1e-4): both sides carry the
    # conditioning of K; 1e-6 relative is well inside the north star's 1e-4
    assert abs(acqf.best_f - best_f) <= 1e-6 * max(1.0, abs(best_f))
    rng = np.random.default_rng(6)
    Xc = rng.uniform(size=(512, config5["d"]))
    Xc[:, 4:] = 0.0
    for i in range(4):                                     # one category per categorical
        Xc[np.arange(512), 4 + 7 * i + rng.integers(0, 7, 512)] = 1.0
    sub = np.arange(0, 512, 16)
    x = torch.tensor((Xc[sub] - st["lo"]) / (st["hi"] - st["lo"]), requires_grad=True)
    # the reference best_f, then a lowered incumbent (best_f is a plain input of the kernel):
    # a 2048-point design leaves random candidates almost no improvement over the true best_f
    mc, _ = ogp.posterior(o, x.detach())
    for lowered in (False, True):
        # lowered: the median objective mean over the checked candidates
        acqf.best_f = float(np.median(-mc.numpy())) if lowered else best_f
        acq, dX = acqf.forward_backward(torch.tensor(Xc, device="cuda"))
        x.grad = None
        ref = oq.qei([o], x.unsqueeze(1), acqf.best_f, acqf.z.cpu().unsqueeze(-1), a=-1.0, bconst=0.0)
        ref.sum().backward()
        if lowered:
            assert (ref.detach() > 0).sum() >= 4
        assert torch.allclose(acq.cpu()[sub], ref.detach(), rtol=1e-6, atol=1e-10)
        gref = x.grad / torch.tensor(st["hi"] - st["lo"])      # d/dX_raw
        assert torch.allclose(dX.cpu()[sub], gref, rtol=1e-5, atol=1e-8 * max(gref.abs().max().item(), 1e-30))
