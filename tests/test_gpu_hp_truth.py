"""qNEHVI / qLogNEHVI at the BASELINE config-3 state against the high-precision truth
(tests/golden/hp_truth.json: 60-digit mpmath posterior roots, tests/golden/make_hp_truth.py),
not against another f64 implementation — the adjudicator where the device and the oracle
disagree.  Reference call site: bofire/strategies/predictives/qnehvi.py:39-52 (cache_root=True:
the new point's root L21 = L_b^-1 Sigma_bx, L22^2 = Sigma_xx - |L21|^2, which cancels to
1e-7 .. 1e-11 of the prior variance at this state for ordinary Sobol candidates).

The state is rebuilt from the fixture's hyperparameters (tests/golden/hp_state.json, the
device fit of bench.build_state), so later changes of the fit's rounding do not move it.
Candidates: the b = 20 Sobol batch of seed 2, every 32nd of the b = 512 batch of seed 2, each
at its own batch size (the restart-batch kernels) and all inside one b = 512 batch (the MFMA
engine path); 16 candidates 1e-2 .. 1e-6 from training points (near16, below).

Bars (ten times inside the north star's 1e-3), printed with their maxima:
* values: relative error <= 1e-4 wherever the truth's HVI > 1e-9 (absolute 1e-12 below);
  qLogNEHVI |d log| <= 1e-4 there and <= 1e-3 for every candidate;
* gradients: row-relative error <= 1e-4 wherever HVI > 1e-9.
Measured (round 6, split root): values 2.2e-6, gradients 1.5e-5; the fused root missed by
5.6e-4 / 2.6e-2 on the same candidates (tools/hp_eval.py, profiles/r06/c/hp_eval.json).
"""
import json
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def hp():
    import bench
    from everest_amd.acquisition import QLogNEHVI, QNEHVI
    from everest_amd.gp import GPBatch, GPHyper

    with open(os.path.join(GOLDEN, "hp_state.json")) as f:
        st = json.load(f)
    with open(os.path.join(GOLDEN, "hp_truth.json")) as f:
        tr = json.load(f)
    dev = torch.device("cuda", 0)
    n, d, m, S = st["n"], st["d"], st["m"], st["S"]
    X = np.random.default_rng(st["x_seed"]).uniform(size=(n, d))
    Y = bench.dtlz2(X, m)
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev)  # noqa: E731
    hypers = [GPHyper(np.asarray(h["lengthscale"]), h["noise"], h["constant"], h["y_mean"], h["y_std"])
              for h in st["hypers"]]
    gp = GPBatch(t(X), t(Y), hypers, 0, t(np.zeros(d)), t(np.ones(d)))
    kw = dict(S=S, sampler_seed=st["sampler_seed"], prune_baseline=True, prune_seed=st["prune_seed"])
    acqf = QNEHVI(gp, X, X, st["ref"] * np.ones(m), -np.ones(m), np.zeros(m), **kw)
    qa = QLogNEHVI(gp, X, X, st["ref"] * np.ones(m), -np.ones(m), np.zeros(m), **kw)
    assert np.array_equal(np.sort(acqf.base_rows), st["base_rows"])
    assert acqf.stats.total_cells == tr["total_cells"] == st["total_cells"]
    return dict(st=st, tr=tr["sets"], acqf=acqf, qa=qa, dev=dev, d=d)


def _check(name, a, ga, T, GT, log):
    """a, ga: device values / gradients; T, GT: truth.  Returns the printed maxima."""
    a, ga, T, GT = (np.asarray(v, dtype=np.float64) for v in (a, ga, T, GT))
    if log:
        verr = np.abs(a - T)
        big = T > math.log(1e-9)
        vbad = np.where(big, verr > 1e-4, verr > 1e-3)
    else:
        verr = np.abs(a - T) / np.maximum(np.abs(T), 1e-300)
        verr[(a == 0) & (T == 0)] = 0.0
        big = T > 1e-9
        vbad = np.where(big, verr > 1e-4, np.abs(a - T) > 1e-12)
    gerr = np.abs(ga - GT).max(1) / np.maximum(np.abs(GT).max(1), 1e-300)
    gbad = big & (gerr > 1e-4)
    vmax = float(verr[big].max()) if big.any() else 0.0
    gmax = float(gerr[big].max()) if big.any() else 0.0
    print(f"{name}: max value error {vmax:.3e}, max row-relative gradient error {gmax:.3e} "
          f"({int(big.sum())} candidates with HVI > 1e-9)")
    assert not vbad.any(), (name, [(int(i), float(a[i]), float(T[i])) for i in np.nonzero(vbad)[0]])
    assert not gbad.any(), (name, [(int(i), float(gerr[i])) for i in np.nonzero(gbad)[0]])
    return vmax, gmax


@pytest.mark.parametrize("which", ["sobol20", "sobol512sub"])
def test_qnehvi_and_qlog_match_high_precision_truth(hp, which):
    import bench

    st, tr, dev = hp["st"], hp["tr"], hp["dev"]
    xs = np.asarray(st["sets"][which])
    T = tr[which]
    # each set at its own batch size (b <= 32: the restart-batch kernels) ...
    Xc = torch.tensor(xs, device=dev)
    for acq, key in ((hp["acqf"], "qnehvi"), (hp["qa"], "qlog")):
        a, g = acq.forward_backward(Xc)
        _check(f"{which} b={len(xs)} {key}", a.cpu(), g.cpu(), T[key], T[key + "_grad"], key == "qlog")
    # ... and inside a b = 512 batch (the MFMA-engine projections)
    big = bench.candidates(512, hp["d"], seed=5, device="cpu").numpy()
    big[:len(xs)] = xs
    Xb = torch.tensor(big, device=dev)
    for acq, key in ((hp["acqf"], "qnehvi"), (hp["qa"], "qlog")):
        a, g = acq.forward_backward(Xb)
        _check(f"{which} b=512 {key}", a.cpu()[:len(xs)], g.cpu()[:len(xs)], T[key], T[key + "_grad"],
               key == "qlog")


def test_near_training_points_match_truth_to_f64_resolution(hp):
    """near16: candidates 1e-2 .. 1e-6 from training points (12 of them next to baseline rows).
    There the exact L22^2 / (s^2 kxx) is 1e-13 .. 1e-19 — below f64's resolution of Sigma_xx
    (~1e-16 absolute) — so no f64 evaluation of the reference's formula resolves L22 (the
    oracle, BoTorch's computation shape, is off by up to 5e-7 absolute / O(1) relative there,
    tests/test_hp_truth_oracle.py).  Held: qNEHVI values within 2e-6 absolute (1.5e-3 of the
    state's largest HVI, 1.3e-3), exact where the truth is 0; qLogNEHVI |d log| <= 1e-3 where
    the truth's HVI > 8e-7 (log > -14) and L22 is resolvable in f64 (exact L22^2 / (s^2 kxx)
    >= 1e-14 in every output; below that the log of a ~1e-6 HVI moves by up to 2e-3 with the
    rounding of L22^2); both batch paths.  Maxima printed."""
    import bench

    st, tr, dev = hp["st"], hp["tr"]["near16"], hp["dev"]
    xs = np.asarray(st["sets"]["near16"])
    big = bench.candidates(512, hp["d"], seed=5, device="cpu").numpy()
    big[:len(xs)] = xs
    for path, Xc in (("b=16", xs), ("b=512", big)):
        a, _ = hp["acqf"].forward_backward(torch.tensor(Xc, device=dev))
        la, _ = hp["qa"].forward_backward(torch.tensor(Xc, device=dev))
        a, la = a.cpu().numpy()[:len(xs)], la.cpu().numpy()[:len(xs)]
        t, lt = np.asarray(tr["qnehvi"]), np.asarray(tr["qlog"])
        err = np.abs(a - t)
        lerr = np.abs(la - lt)
        sel = (lt > -14.0) & (np.asarray(tr["rel"]).min(0) >= 1e-14)
        print(f"near16 {path}: max |d qNEHVI| {err.max():.3e}; |d log| where log HVI > -14: "
              f"{np.array2string(lerr[lt > -14.0], precision=2)}; held to 1e-3: {int(sel.sum())} candidates")
        assert (err <= 2e-6).all(), (path, err)
        assert (a[t == 0] == 0).all(), (path, a[t == 0])
        assert (lerr[sel] <= 1e-3).all(), (path, lerr)
