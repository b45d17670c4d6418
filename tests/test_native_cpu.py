"""CPU: the C-ABI library loads, exports every symbol include/everest_amd.h declares, its
host-side box decomposition matches the oracle, errors surface as messages, and the device
ops refuse CPU tensors (no CPU fallback)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "everest_amd.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|long long|void|const char\*)\s+(evr_\w+)\s*\(", hdr, re.M)))


def test_library_exports_header_symbols():
    from everest_amd import _native

    lib = _native.load()
    syms = _declared_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) <= set(_native.EXPORTED_SYMBOLS) | {"evr_cells_free"}
    assert lib.evr_version() == 1


def test_error_path_message():
    from everest_amd import _native

    lib = _native.load()
    out = ctypes.c_void_p()
    st = lib.evr_box_decompose(0, 1, 1, None, 0, 0, 0, None, None, 1, ctypes.byref(out))
    assert st != 0 and b"bad arguments" in lib.evr_last_error()


@pytest.mark.parametrize("m,n,S", [(2, 15, 4), (3, 25, 6), (5, 30, 3)])
def test_host_box_decomposition_matches_oracle(m, n, S):
    from everest_amd import ops
    from oracle.multiobjective import hvi_from_cells, nondominated_cells, pareto_above_ref

    rng = np.random.default_rng(m * 100 + n)
    obj = -rng.uniform(size=(S, n, m))
    obj[:, 3] = obj[:, 2]                      # exact duplicates are deduplicated
    ref = -1.1 * np.ones(m)
    lo, hi, off = ops.box_decompose(obj, ref, None, 3, layout="sij")
    for s in range(S):
        c = nondominated_cells(pareto_above_ref(torch.tensor(obj[s]), torch.tensor(ref)), torch.tensor(ref))
        assert off[s + 1] - off[s] == c.shape[1]
        y = torch.tensor(-rng.uniform(size=(40, m)) * 0.95)
        mine = torch.stack([torch.tensor(lo[off[s]:off[s + 1]]), torch.tensor(hi[off[s]:off[s + 1]])])
        assert torch.allclose(hvi_from_cells(y, c), hvi_from_cells(y, mine), atol=1e-14, rtol=0)
    # layout 'jis' gives identical cells
    lo2, hi2, off2 = ops.box_decompose(np.ascontiguousarray(obj.transpose(2, 1, 0)), ref, None, 2, layout="jis")
    assert np.array_equal(off, off2) and np.array_equal(lo, lo2) and np.array_equal(hi, hi2)


def test_box_decomposition_empty_front_single_cell():
    from everest_amd import ops

    obj = -2.0 * np.ones((2, 3, 3))            # every point worse than the reference
    lo, hi, off = ops.box_decompose(obj, -1.1 * np.ones(3), None, 1, layout="sij")
    assert list(off) == [0, 1, 2]
    assert np.allclose(lo, -1.1) and np.isinf(hi).all()


def test_device_ops_refuse_cpu_tensors():
    from everest_amd import ops

    X = torch.zeros(4, 2, dtype=torch.float64)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.kernel_matrix(X, X, torch.ones(1, 2, dtype=torch.float64))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.cholesky(torch.eye(3, dtype=torch.float64))


@pytest.mark.parametrize("dim,seed", [(1, 0), (5, 17), (64, 123456), (2561, 987654)])
def test_sobol_scramble_matches_torch_engine(dim, seed):
    """evr_sobol_scramble reproduces SobolEngine(dim, scramble=True, seed) state bit for bit
    (mt19937 stream of torch.Generator.manual_seed, LMS matrices, random shift)."""
    from everest_amd import _native

    V = torch.zeros(dim, 30, dtype=torch.long)
    torch._sobol_engine_initialize_state_(V, dim)
    shift = torch.empty(dim, dtype=torch.long)
    assert _native.load().evr_sobol_scramble(dim, seed, V.data_ptr(), shift.data_ptr()) == 0
    eng = torch.quasirandom.SobolEngine(dim, scramble=True, seed=seed)
    assert torch.equal(V, eng.sobolstate)
    assert torch.equal(shift, eng.shift)


def test_sobol_gray_code_closed_form_matches_engine():
    """Point k = shift ^ XOR_{bits of gray(k)} V (the device kernel's indexing) equals the
    engine's sequential draw; point 0 goes through float32 like SobolEngine._first_point."""
    dim, n = 7, 300
    eng = torch.quasirandom.SobolEngine(dim, scramble=True, seed=31)
    u = eng.draw(n, dtype=torch.float64)
    V, sh = eng.sobolstate, eng.shift
    for k in (0, 1, 2, 3, 5, 127, 128, 255, 299):
        x = sh.clone()
        if k == 0:
            ref = sh.to(torch.float32).to(torch.float64) / 2 ** 30
        else:
            g = k ^ (k >> 1)
            b = 0
            while g:
                if g & 1:
                    x ^= V[:, b]
                g >>= 1
                b += 1
            ref = x.to(torch.float64) / 2 ** 30
        assert torch.equal(u[k], ref), k


def test_torch_operator_library_registers_ops():
    """The TORCH_LIBRARY(everest_amd) operators load and register on CPU (no compute: they
    reject CPU tensors — no CPU fallback)."""
    from everest_amd import torch_ops

    ns = torch_ops.load()
    for name in ("kernel_matrix", "cholesky", "gp_posterior", "qnehvi_forward", "qnehvi_forward_backward",
                 "qnehvi_backward"):
        assert hasattr(ns, name)
    assert hasattr(torch.classes.everest_amd, "QnehviAcq")
    x = torch.zeros(3, 2, dtype=torch.float64)
    with pytest.raises((RuntimeError, NotImplementedError)):
        ns.kernel_matrix(x, x, torch.ones(2, dtype=torch.float64), 0)


def _sorted_cells(lo, hi):
    rows = np.concatenate([lo, hi], 1)
    return rows[np.lexsort(rows.T[::-1])]


@pytest.mark.parametrize("m,n,alpha", [(3, 25, 1e-3), (3, 40, 0.05), (4, 30, 0.01), (5, 20, 0.2)])
def test_host_approximate_partition_matches_oracle(m, n, alpha):
    """alpha > 0: evr_box_decompose_approx vs the oracle's restatement of [upstream]
    NondominatedPartitioning(alpha) — the same cell set, bit for bit; the approximation only
    drops volume (HVI <= exact) and alpha -> 0 recovers the exact partition."""
    from everest_amd import ops
    from oracle.multiobjective import approximate_cells, hvi_from_cells, nondominated_cells, pareto_above_ref

    rng = np.random.default_rng(7 * m + n)
    S = 3
    obj = -rng.uniform(size=(S, n, m))
    obj[:, 4] = obj[:, 1]
    ref = -1.1 * np.ones(m)
    lo, hi, off = ops.box_decompose(obj, ref, None, 2, layout="sij", alpha=alpha)
    lo0, hi0, off0 = ops.box_decompose(obj, ref, None, 2, layout="sij")
    y = torch.tensor(-rng.uniform(size=(64, m)) * 0.9)
    for s in range(S):
        pf = pareto_above_ref(torch.tensor(obj[s]), torch.tensor(ref))
        c = approximate_cells(pf, torch.tensor(ref), alpha)
        a, b = off[s], off[s + 1]
        assert b - a == c.shape[1]
        assert np.array_equal(_sorted_cells(lo[a:b], hi[a:b]), _sorted_cells(c[0].numpy(), c[1].numpy()))
        mine = torch.stack([torch.tensor(lo[a:b]), torch.tensor(hi[a:b])])
        exact = torch.stack([torch.tensor(lo0[off0[s]:off0[s + 1]]), torch.tensor(hi0[off0[s]:off0[s + 1]])])
        h, h0 = hvi_from_cells(y, mine), hvi_from_cells(y, exact)
        assert (h <= h0 + 1e-14).all()
        c_full = approximate_cells(pf, torch.tensor(ref), 0.0)       # no approximation: exact region
        assert torch.allclose(hvi_from_cells(y, c_full), hvi_from_cells(y, nondominated_cells(pf, torch.tensor(ref))),
                              atol=1e-13, rtol=0)


def test_approximate_partition_m2_is_exact_and_alpha_bounds():
    """m = 2 takes the exact partition whatever alpha ([upstream] _partition_space_2d);
    a negative or non-finite alpha is refused."""
    from everest_amd import _native, ops

    rng = np.random.default_rng(3)
    obj = -rng.uniform(size=(2, 20, 2))
    ref = -1.1 * np.ones(2)
    a = ops.box_decompose(obj, ref, None, 1, layout="sij", alpha=0.3)
    b = ops.box_decompose(obj, ref, None, 1, layout="sij")
    assert all(np.array_equal(x, z) for x, z in zip(a, b))
    with pytest.raises(RuntimeError, match="bad arguments"):
        ops.box_decompose(obj, ref, None, 1, layout="sij", alpha=-0.1)
    assert hasattr(_native.load(), "evr_box_decompose_approx")


def test_evaluation_chain_kernels_use_no_scratch():
    """Register spills / dynamically indexed private arrays land in scratch memory, whose
    traffic goes through L2 and HBM on every launch (hvi_kdb<5> wrote ~58 MB of scratch per
    launch before round 4).  The code-object metadata of the built library must show zero
    private-segment bytes for the restart chain, the evaluation pass, the fit and the
    construction kernels at the configs' shapes (m <= 5 objectives, d <= 32 inputs)."""
    import re
    import shutil
    import sys

    if not shutil.which("/opt/rocm/lib/llvm/bin/llvm-readelf"):
        pytest.skip("ROCm llvm tools not installed")
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import kernel_resources as kr

    ks = kr.kernels(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "everest_amd", "_lib",
                                 "libeverest_amd.so"))
    names = dict(zip(kr.demangle(sorted(ks)), [ks[k] for k in sorted(ks)]))
    hot = re.compile(r"evr::(qs_fwd|qs_bwd|qs_dx_reduce|hvi_kdb<[1-5]>|hvi_kdw<[1-5]>|hvi_kd2<[1-5],|hvi_kd3<[1-5]>|hvi_thresholds|"
                     r"hvi_reduce|kmat_kernel|kmat_mfma_kernel|kmat_mfma_sym|qn_samples_norms|qn_proj|qn_gen_gr|qn_bwd_coef|"
                     r"qn_mean_row|qn_norms_rows|kcross_grad_kernel<(8|16|32)>|kls_grad_kernel|chol_|tri_inv|"
                     r"trsm16|pareto_f32_kernel<[1-5]>|bd_build_kernel<[1-5],|cells_kd_kernel<[1-5],|"
                     r"sobol|mll_|posterior_finalize|hvi_logk_kernel<[1-5], (true|false), 2|hvi_log_reduce)")
    checked = {k: v for k, v in names.items() if hot.search(k)}
    assert len(checked) > 40, sorted(checked)
    spill = {k: v.get("scratch") for k, v in checked.items() if v.get("scratch")}
    assert not spill, spill


def test_lbfgsb_advance_matches_generator_state_machine():
    """evr_lbfgsb_advance (the per-member step of the native GP-fit driver, evr_mll_fit_rounds)
    applies optim.lbfgsb_steps' state machine — evaluation counting, NEW_X iterations, the
    maxiter / maxfun stops, the final status — to the same native L-BFGS-B: on a host
    objective (5-d Rosenbrock, and a bounded quadratic that hits maxiter) both drivers visit
    the same iterates bitwise and stop with the same counts."""
    from everest_amd import _native
    from everest_amd.optim import LBFGSB_FG, _EPS, lbfgsb_steps

    lib = _native.load()

    def rosen(x):
        f, g = 0.0, np.zeros_like(x)
        for i in range(len(x) - 1):
            f += 100 * (x[i + 1] - x[i] ** 2) ** 2 + (1 - x[i]) ** 2
            g[i] += -400 * x[i] * (x[i + 1] - x[i] ** 2) - 2 * (1 - x[i])
            g[i + 1] += 200 * (x[i + 1] - x[i] ** 2)
        return f, g

    def quad(x):
        w = np.arange(1.0, len(x) + 1.0)
        return float(np.sum(w * (x - 0.3) ** 2)), 2 * w * (x - 0.3)

    cases = ((rosen, np.array([-1.2, 1.0, 0.5, -0.3, 0.8]), np.full(5, -np.inf), np.full(5, np.inf), 15000),
             (quad, np.full(4, 2.0), np.full(4, 0.5), np.full(4, 3.0), 2))
    for fun, x0, lb, ub, maxiter in cases:
        n = len(x0)
        gen = lbfgsb_steps(x0, lb, ub, maxiter=maxiter)
        xs_gen, x = [], next(gen)
        try:
            while True:
                xs_gen.append(x.copy())
                x = gen.send(fun(x))
        except StopIteration as stop:
            res = stop.value
        h = ctypes.c_void_p()
        lo, hi = np.ascontiguousarray(lb), np.ascontiguousarray(ub)
        _native.check(lib.evr_lbfgsb_create(n, 10, lo.ctypes.data, hi.ctypes.data, 2.220446049250313e-09 / _EPS,
                                            1e-5, 20, ctypes.byref(h)), "evr_lbfgsb_create")
        try:
            X = np.zeros(n)
            task, nit, nfev, st = (np.zeros(1, dtype=np.int32) for _ in range(4))
            task[0] = lib.evr_lbfgsb_start(h, np.ascontiguousarray(x0).ctypes.data, X.ctypes.data)
            xs_adv = []
            while task[0] == LBFGSB_FG:
                xs_adv.append(X.copy())
                f, g = fun(X.copy())
                g = np.ascontiguousarray(g, dtype=np.float64)
                _native.check(lib.evr_lbfgsb_advance(h, ctypes.c_double(f), g.ctypes.data, X.ctypes.data,
                                                     task.ctypes.data, nit.ctypes.data, nfev.ctypes.data,
                                                     st.ctypes.data, maxiter, 15000), "evr_lbfgsb_advance")
        finally:
            lib.evr_lbfgsb_destroy(h)
        assert len(xs_adv) == len(xs_gen)
        assert all(np.array_equal(a, b) for a, b in zip(xs_adv, xs_gen))
        assert (int(nit[0]), int(nfev[0]), int(st[0])) == (res.nit, res.nfev, res.status)
        assert np.array_equal(X, res.x)


def _hit_and_run_restated(A, b, N, x0, n, seed, n_burnin, n_thinning):
    """Plain-Python restatement of csrc/polytope.cpp's chain (the counter-based SplitMix64
    variates, Box-Muller cos branch, index-order sums): the native sampler must equal it step
    for step."""
    import math

    M64 = (1 << 64) - 1

    def uni(c):
        z = (seed + (c + 1) * 0x9E3779B97F4A7C15) & M64
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        z ^= z >> 31
        return (z >> 11) * 2.0 ** -53

    d, k = N.shape
    x = [float(v) for v in x0]
    out, per = [], 2 * k + 1
    for it in range(n_burnin + n * n_thinning):
        c0 = it * per
        z = [math.sqrt(-2.0 * math.log(1.0 - uni(c0 + 2 * j))) * math.cos(6.283185307179586 * uni(c0 + 2 * j + 1))
             for j in range(k)]
        r, nr2 = [], 0.0
        for i in range(d):
            s = 0.0
            for j in range(k):
                s += float(N[i, j]) * z[j]
            r.append(s)
            nr2 += s * s
        nr = math.sqrt(nr2)
        if nr > 0.0:
            r = [v / nr for v in r]
            tmax = tmin = None
            for q in range(A.shape[0]):
                ar = ax = 0.0
                for i in range(d):
                    ar += float(A[q, i]) * r[i]
                    ax += float(A[q, i]) * x[i]
                if ar > 1e-14 or ar < -1e-14:
                    t = (float(b[q]) - ax) / ar
                    if ar > 1e-14:
                        tmax = t if tmax is None or t < tmax else tmax
                    else:
                        tmin = t if tmin is None or t > tmin else tmin
            u = uni(c0 + 2 * k)
            lo_, hi_ = (tmin if tmin is not None else 0.0), (tmax if tmax is not None else 0.0)
            step = lo_ + (hi_ - lo_) * u
            x = [xi + step * ri for xi, ri in zip(x, r)]
        if it >= n_burnin and (it - n_burnin) % n_thinning == n_thinning - 1:
            out.append(list(x))
    return np.array(out)


def test_hit_and_run_native_chain_equals_restatement():
    """evr_hit_and_run (the raw-candidate sampler of optimize_acqf under linear constraints,
    [upstream] HitAndRunPolytopeSampler, bofire/strategies/predictives/botorch.py:384-405)
    equals the plain-Python restatement bitwise: a Detergent-like 5-d box with two linear
    inequalities, and the same with one equality (null-space directions)."""
    from everest_amd.optim import _as_Ab, hit_and_run_chain

    d = 5
    bounds = np.array([[0.0] * d, [1.0, 0.8, 0.6, 1.0, 0.5]])
    ineq = [([0, 1, 2], [-1.0, -1.0, -1.0], -1.2), ([2, 3, 4], [1.0, 1.0, 1.0], 0.2)]
    A, b = _as_Ab(d, bounds, ineq)
    x0 = np.array([0.2, 0.2, 0.2, 0.3, 0.1])
    assert (A @ x0 < b).all()
    for N, seed in ((np.eye(d), 12345), (np.linalg.svd(np.ones((1, d)))[2][1:].T, 2 ** 63 + 7)):
        got = hit_and_run_chain(A, b, N, x0, 40, seed, 50, 3)
        want = _hit_and_run_restated(A, b, N, x0, 40, seed, 50, 3)
        assert got.shape == (40, d)
        assert np.array_equal(got, want), np.abs(got - want).max()


def test_hit_and_run_samples_feasible_and_uniform():
    """Properties of the native sampler at the optimizer's defaults (burn-in 10000, thinning
    32): every sample inside the polytope; on the triangle {x, y >= 0, x + y <= 1} the sample
    mean is the centroid (1/3, 1/3) and each of the four congruent sub-triangles holds a
    quarter of the samples; with an equality constraint every sample lies on it."""
    from everest_amd.optim import hit_and_run

    bounds = np.array([[0.0, 0.0], [1.0, 1.0]])
    X = hit_and_run(bounds, [([0, 1], [-1.0, -1.0], -1.0)], [], 4000, seed=3)
    assert X.shape == (4000, 2)
    assert (X >= -1e-12).all() and (X.sum(1) <= 1.0 + 1e-12).all()
    assert np.abs(X.mean(0) - 1.0 / 3.0).max() < 0.02
    mid = (X[:, 0] >= 0.5).mean(), (X[:, 1] >= 0.5).mean(), (X.sum(1) <= 0.5).mean()
    assert all(abs(f - 0.25) < 0.03 for f in mid), mid
    bounds3 = np.array([[0.0] * 3, [1.0] * 3])
    Y = hit_and_run(bounds3, [], [([0, 1, 2], [1.0, 1.0, 1.0], 1.0)], 500, seed=9, n_burnin=200, n_thinning=4)
    assert np.abs(Y.sum(1) - 1.0).max() < 1e-10 and (Y >= -1e-12).all()
    # seeded: the same seed gives the same samples, another seed others
    assert np.array_equal(Y, hit_and_run(bounds3, [], [([0, 1, 2], [1.0, 1.0, 1.0], 1.0)], 500, seed=9,
                                         n_burnin=200, n_thinning=4))
