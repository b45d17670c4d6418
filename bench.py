#!/usr/bin/env python
"""Benchmark of the qNEHVI hot path on MI355X (BASELINE.json metric: QnehviStrategy.ask()
candidates/sec + GP posterior ms, n=512 d=6 m=5).

A *step* is one full ``QnehviStrategy.ask()`` of BASELINE configs[3] (SURVEY.md §8(d)
config 4) through the BoFire-compatible API: DTLZ2(dim=6, m=5), X_train ~ U[0,1]^6 (n=512,
seed 0), noise-free Y, reference point 1.1 -> -1.1, 5 exact RBF GPs fitted once by tell()
on the device; each ask builds qNEHVI as BoFire does (prune_baseline over 2048 draws, cached
root, S=256 Sobol-normal samples, exact box decompositions), screens 1024 raw Sobol
candidates and runs 20 L-BFGS-B restarts (q=1) on the analytic device gradient.  ``value``
= (raw samples + optimiser evaluations x batch) / ask wall time — SURVEY.md §8(d)'s
definition of ask() candidates/s — over K timed asks after W warm-up asks.

Also reported: ``eval_pass`` (one forward + backward over b=512 candidates resident in HBM
through the native plan, the unit raw screening is made of, with its per-kernel rooflines
and PMC traffic), the per-kernel table at the restart batch (the top-level ``roofline`` is
its dominant op), the GP posterior of the ask's fitted model, and the CPU baseline (the
reference-structure oracle on the host cores, composed from bounded samples of each ask
phase).

Multi-GPU (one process per GPU, RCCL): ``--gpus N`` spawns N ranks itself (or runs under
torchrun with WORLD_SIZE = N).  One ask is a sequential, latency-bound optimisation — the
20 restarts are ONE joint L-BFGS-B problem (batch_limit = num_restarts, BoFire's default)
whose every iteration waits on the previous evaluation — so N GPUs serve N asks: ``value``
at N > 1 is replicas (weak scaling), every rank running the complete N = 1 workload with
its own seed and no collective in the timed region.  ``sharded_ask`` then times the single
ask sharded over the ranks (config 4's layout): raw screening in N shards
with an all-gather of the values, the joint restart problem replicated on every rank with
each rank evaluating its slice per iteration and all-gathering (value, gradient).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import re
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP64_TFLOPS = 78.6     # MI355X FP64 vector & matrix (AMD spec; = 1/2 the FP32 vector peak 157.3 TF)
PEAK_HBM_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def dtlz2(X: np.ndarray, m: int) -> np.ndarray:
    k = X.shape[1] - m + 1
    g = ((X[..., -k:] - 0.5) ** 2).sum(-1)
    fs = []
    for i in range(m):
        idx = m - 1 - i
        f = (1 + g) * np.cos(X[..., :idx] * math.pi / 2).prod(-1)
        if i > 0:
            f = f * np.sin(X[..., idx] * math.pi / 2)
        fs.append(f)
    return np.stack(fs, -1)


def build_state(n: int, d: int, m: int, S: int, device, prune_samples: int = 2048):
    from everest_amd.acquisition import QNEHVI
    from everest_amd.gp import GPBatch, fit_single

    rng = np.random.default_rng(0)
    X = rng.uniform(size=(n, d))
    Y = dtlz2(X, m)
    lo, hi = np.zeros(d), np.ones(d)
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=device)  # noqa: E731
    Xn = t(X)
    ls_prior = (math.sqrt(2) + 0.5 * math.log(d), math.sqrt(3))  # bofire/priors/mapper.py:43-50
    t0 = time.perf_counter()
    hypers = [fit_single(Xn, Y[:, j], 0, ls_prior, (-4.0, 1.0)) for j in range(m)]
    torch.cuda.synchronize()
    t_fit = time.perf_counter() - t0
    gp = GPBatch(Xn, t(Y), hypers, 0, t(lo), t(hi))
    t0 = time.perf_counter()
    acqf = QNEHVI(gp, X, X, -1.1 * np.ones(m), -np.ones(m), np.zeros(m), S=S, sampler_seed=1234,
                  prune_baseline=True, prune_seed=4321, prune_samples=prune_samples)
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t0
    return X, Y, gp, hypers, acqf, t_fit, t_build


def candidates(b: int, d: int, seed: int, device):
    eng = torch.quasirandom.SobolEngine(d, scramble=True, seed=seed)
    return eng.draw(b, dtype=torch.float64).to(device)


def op_chain(acqf, Xc):
    """The evaluation chain op by op (the kernels the native plan runs), as closures over
    fixed inputs so that each op can be launched repeatedly (idempotent)."""
    from everest_amd import ops

    st, gp, b = acqf.state, acqf.gp, Xc.shape[0]
    Kx = gp.cross(Xc)
    if ops.qnehvi_small_applies(st, b, Xc.shape[1]):
        # restart batches: the plan's b <= 32 kernels (the cross-covariance gradient is fused
        # into proj_bwd there, so there is no separate kernel_grad op)
        md = acqf.model
        R, P = ops.qnehvi_small_forward(st, md, Kx, b)
        G, L22, flags = ops.qnehvi_small_samples(st, R, P, b)
        if ops.hvi_restart_fb_applies(st, b):
            # the plan's one-launch restart scan (hvi_kd3: thresholds + scan + split reduction)
            _, dG = ops.hvi_restart_fb(st, G, b)
            scan = lambda: ops.hvi_restart_fb(st, G, b)   # noqa: E731
        else:
            _, dG = ops.hvi_forward_backward(st, G, b, flags)
            scan = lambda: ops.hvi_forward_backward(st, G, b, flags)   # noqa: E731
        return {
            "kernel_matrix": lambda: gp.cross(Xc),
            "proj_fwd": lambda: ops.qnehvi_small_forward(st, md, Kx, b),
            "samples": lambda: ops.qnehvi_small_samples(st, R, P, b),
            "hvi_fwd_bwd": scan,
            "proj_bwd": lambda: ops.qnehvi_small_backward(st, md, Xc, R, L22, dG, b),
        }
    R, P = ops.qnehvi_project(st, acqf.M, Kx, b)
    G, L22, flags = ops.qnehvi_samples_norms(st, R, P, b)
    acq, dG = ops.hvi_forward_backward(st, G, b, flags)
    dKx = ops.qnehvi_project_backward(st, acqf.M, R, L22, dG, b)
    return {
        "kernel_matrix": lambda: gp.cross(Xc),
        "proj_fwd": lambda: ops.qnehvi_project(st, acqf.M, Kx, b),
        "samples": lambda: ops.qnehvi_samples_norms(st, R, P, b),
        "hvi_fwd_bwd": lambda: ops.hvi_forward_backward(st, G, b, flags),
        "proj_bwd": lambda: ops.qnehvi_project_backward(st, acqf.M, R, L22, dG, b),
        "kernel_grad": lambda: ops.kernel_cross_grad(gp.Xn, Xc, gp.ls, dKx, gp.kind, shift2=gp.lo,
                                                     scale2=gp.inv_range),
    }


def kernel_times(acqf, Xc, reps=10):
    """Average device time (ms) of each op of the chain: ``reps`` launches of the op are
    captured into one HIP graph on torch's current stream (the stream every evr_* call is
    enqueued on) and the replay is bracketed by HIP events, so the figure is the kernels'
    back-to-back duration, free of host enqueue gaps (it agrees with rocprofv3's per-kernel
    averages).  Falls back to eager launches between events if capture is refused."""
    out, how = {}, "hip-graph replay"
    for name, f in op_chain(acqf, Xc).items():
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(reps):
                    f()
            g.replay()
            torch.cuda.synchronize()
            e0.record()
            g.replay()
            e1.record()
        except RuntimeError:
            how = "eager launches"
            torch.cuda.synchronize()
            e0.record()
            for _ in range(reps):
                f()
            e1.record()
        torch.cuda.synchronize()
        out[name] = e0.elapsed_time(e1) / reps
    return out, how


def scan_counts(acqf, Xc):
    """Exact work of the sparse HVI scan at this batch (device counters of hvi_kd): passing
    (candidate, group) pairs, evaluated (cell, candidate) terms, (candidate, group) tests."""
    from everest_amd import ops

    st = acqf.state
    if not st.grp_off:
        return {"group_pairs": 0, "terms": 0, "group_tests": 0}
    b = Xc.shape[0]
    ctr = torch.zeros(4, dtype=torch.int64, device=Xc.device)
    R, P = ops.qnehvi_project(st, acqf.M, acqf.gp.cross(Xc), b)
    G, L22, flags = ops.qnehvi_samples_norms(st, R, P, b)
    st.scan_counters = ctr.data_ptr()
    try:
        ops.hvi_forward_backward(st, G, b, flags)
        c = ctr.cpu().numpy()
    finally:
        st.scan_counters = None
    return {"group_pairs": int(c[0]), "terms": int(c[1]), "group_tests": int(c[2])}


def _event_ms(fn, reps=20, warm=3):
    """Average device time of fn() over ``reps`` back-to-back calls, bracketed by HIP events
    on torch's current stream (the stream every evr_* call is enqueued on)."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def cholesky_figures(device):
    """Batched psd_safe Cholesky (evr_cholesky) and Cholesky + inverse (the GP fit's MLL
    factorisation) timed with HIP events on device-resident SPD inputs; TF/s against the f64
    MFMA peak (n^3/3 flops per factorisation, + n^3/3 for the inverse)."""
    from everest_amd import ops

    out = {}
    for n, B, inv in ((512, 5, True), (2048, 1, False)):
        g = torch.Generator().manual_seed(n)
        A = torch.randn(B, n, n + 7, generator=g, dtype=torch.float64)
        A = (A @ A.transpose(1, 2) / n + 1e-2 * torch.eye(n, dtype=torch.float64)).to(device)
        f = (lambda: ops.cholesky_inverse(A)) if inv else (lambda: ops.cholesky(A))
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        flops = B * n ** 3 / 3 * (2 if inv else 1)
        out[f"{'cholesky_inverse' if inv else 'cholesky'}_n{n}_b{B}"] = {
            "ms": round(ms, 4), "achieved": round(flops / ms / 1e9, 3), "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
            "frac": round(flops / ms / 1e9 / PEAK_FP64_TFLOPS, 4),
            "note": "includes the jitter-ladder host check (one device->host info copy per call)"}
    return out


def gp_posterior_ms(device, gp=None, n_test=1024, reps=20):
    """GP posterior (mean + var, observation_noise=False) of 1024 Sobol test points.
    Default: config 2 (SingleTaskGP RBF, n_train=256, d=6, one output, fixed hypers); with
    ``gp`` the given batched model (the metric's n=512, d=6, m=5 shape from build_state)."""
    from everest_amd.gp import GPBatch, GPHyper

    if gp is None:
        rng = np.random.default_rng(0)
        X = rng.uniform(size=(256, 6))
        y = dtlz2(X, 5)[:, :1]
        h = GPHyper(lengthscale=np.full(6, 0.8), noise=1e-3, constant=0.0, y_mean=float(y.mean()),
                    y_std=float(y.std(ddof=1)))
        t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=device)  # noqa: E731
        gp = GPBatch(t(X), t(y), [h], 0, t(np.zeros(6)), t(np.ones(6)))
    d = gp.Xn.shape[1]
    Xs = torch.quasirandom.SobolEngine(d, scramble=True, seed=1).draw(n_test, dtype=torch.float64).to(device)
    return _event_ms(lambda: gp.posterior(Xs), reps=reps)


def config1_loop(seed=7):
    """BASELINE configs[0] (README.md:82-104): the Detergent benchmark, QnehviStrategy at the
    data model's defaults (512 MC samples, 1024 raw samples, 8 restarts, batch_limit 8, two
    linear inequality constraints: hit-and-run raw samples, SLSQP restarts on the device
    gradient), 2 random initial experiments then 4 x (tell -> ask(1) -> f).  Wall time of
    every tell and ask (synchronised); the first tell / ask include the process's first use
    of those code paths."""
    import everest_amd.data_models as dm
    from everest_amd import strategies
    from everest_amd.benchmarks import Detergent

    bm = Detergent()
    rnd = strategies.map(dm.RandomStrategy(domain=bm.domain, seed=19))
    exps = bm.f(rnd.ask(2), return_complete=True)
    s = strategies.map(dm.QnehviStrategy(domain=bm.domain, seed=seed))
    tells, asks, phases = [], [], []
    for it in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.tell(exps)
        torch.cuda.synchronize()
        tells.append(time.perf_counter() - t0)
        if it == 4:
            break
        t0 = time.perf_counter()
        c = s.ask(candidate_count=1)
        torch.cuda.synchronize()
        asks.append(time.perf_counter() - t0)
        st = s.last_ask_stats
        construction = float(getattr(s.last_acqf, "timings", {}).get("total", 0.0))
        phases.append({"construction": construction, "raw_draw": st.t_raw_draw,
                       "raw_screening": st.t_raw - st.t_raw_draw, "restarts": st.t_opt,
                       "other": asks[-1] - construction - st.t_raw - st.t_opt,
                       "restart_evals": int(st.opt_evals), "driver": st.chunks[0]["driver"] if st.chunks else None})
        exps = bm.f(c[bm.domain.inputs.get_keys()], return_complete=True)
    r = lambda v: [round(x, 4) for x in v]  # noqa: E731
    return {"workload": "BASELINE configs[0]: Detergent, QnehviStrategy defaults (S=512, raw 1024, 8 restarts, "
                        "SLSQP under 2 linear constraints), 2 initial + 4 ask/tell rounds",
            "ask_s": r(asks), "tell_s": r(tells), "ask_s_median": round(float(np.median(asks)), 4),
            "tell_s_median": round(float(np.median(tells)), 4), "experiments": s.num_experiments,
            "phases_median_s": {k: round(float(np.median([p[k] for p in phases])), 4)
                                for k in ("construction", "raw_draw", "raw_screening", "restarts", "other")},
            "restart_evals": [p["restart_evals"] for p in phases],
            "driver": s.last_ask_stats.chunks[0]["driver"] if s.last_ask_stats.chunks else None}


def build_provenance():
    """everest_amd/_lib/build_info.json (written by the Makefile next to the libraries): the
    commit the shipped .so files were built from and their SHA-256."""
    try:
        with open(os.path.join(ROOT, "everest_amd", "_lib", "build_info.json")) as f:
            info = json.load(f)
        return {"commit": info.get("commit"), "dirty": info.get("dirty"), "built_utc": info.get("built_utc"),
                "compiler": info.get("compiler"),
                "sha256": {k: v.get("sha256", "")[:16] for k, v in info.get("libs", {}).items()}}
    except (OSError, ValueError):
        return None


def cpu_baseline(acqf, hypers, X, Y, Xc_cpu, chunk=8, budget_s=12.0):
    """Reference-structure CPU restatement (oracle/, torch-CPU fp64, BoTorch computation
    shape: joint posterior over [X_base; x] per forward, per-sample cell scan, autograd
    backward) timed on the host cores over a BOUNDED sample of the same workload: chunks of
    ``chunk`` candidates (BoFire's default batch_limit = 8,
    bofire/data_models/strategies/predictives/botorch.py:101-108) from the same candidate
    batch, forward+backward each, until ``budget_s`` of CPU wall time is spent.  The cells
    are injected from the device build so only the evaluation is timed."""
    from oracle import gp as ogp
    from oracle import qnehvi as oq

    Xn = torch.tensor(X)
    states = []
    for j, h in enumerate(hypers):
        y = torch.tensor(Y[:, j])
        states.append(ogp.GPState(X=Xn, y=(y - h.y_mean) / h.y_std, lengthscale=torch.tensor(h.lengthscale),
                                  noise=h.noise, constant=h.constant, y_mean=h.y_mean, y_std=h.y_std))
    nb = acqf.nb
    off = acqf.cells.off.cpu().numpy()
    lo, hi = (t.cpu() for t in acqf.cells.explicit())
    cells = [torch.stack([lo[off[s]:off[s + 1]], hi[off[s]:off[s + 1]]]) for s in range(acqf.S)]
    zq = acqf.zq.cpu().unsqueeze(1)
    zb = torch.zeros(acqf.S, nb, acqf.m, dtype=torch.float64)
    orc = oq.QNEHVI(states, Xn[torch.as_tensor(acqf.base_rows)], oq.Objective(-torch.ones(acqf.m),
                    torch.zeros(acqf.m, dtype=torch.float64)), torch.full((acqf.m,), -1.1, dtype=torch.float64),
                    zb, zq, cells=cells)
    done, spent, i = 0, 0.0, 0
    while spent < budget_s and (i + 1) * chunk <= Xc_cpu.shape[0]:
        x = Xc_cpu[i * chunk:(i + 1) * chunk].clone().requires_grad_(True)
        t0 = time.perf_counter()
        v = orc.forward(x.unsqueeze(1))
        v.sum().backward()
        spent += time.perf_counter() - t0
        done += chunk
        i += 1
    return spent, done, orc, states


def cpu_ask_estimate(orc, states, acqf, Xc_cpu, ask, prune_sub=128, prune_samples=2048, box_samples=2):
    """Reference-structure CPU ``QnehviStrategy.ask()`` wall time for the ask that was timed
    on the GPU (same problem, same raw-sample and restart counts, the GPU ask's optimiser
    evaluation count), composed from bounded samples of each phase with the oracle
    (torch-CPU fp64, BoTorch's computation shape):
      * prune_baseline over ``prune_sub`` of the ``prune_samples`` posterior draws (x ratio);
      * the per-sample box decomposition of ``box_samples`` MC samples (x S);
      * raw screening: forward-only in chunks of batch_limit (= restarts, BoFire's default),
        two chunks timed, scaled to raw_samples;
      * restarts: one joint forward+backward of ``restarts`` candidates (one L-BFGS-B
        function evaluation), scaled to the GPU ask's evaluation count.
    Returns a dict (seconds per phase, total, and the ask speedup)."""
    from oracle import qnehvi as oq
    from oracle.multiobjective import nondominated_cells, pareto_above_ref

    out = {}
    n, m = orc.models[0].X.shape[0], len(states)
    Xn = orc.models[0].X
    z = oq.base_samples(prune_sub, n, m, 7)
    t0 = time.perf_counter()
    oq.prune_baseline(states, Xn, orc.obj, orc.ref, z)
    out["prune_s"] = (time.perf_counter() - t0) * prune_samples / prune_sub
    zb = oq.base_samples(box_samples, orc.Xb.shape[0], m, 11)
    mean_b, _ = oq.joint_posterior(states, orc.Xb)
    obj_b = orc.obj(mean_b.unsqueeze(0) + torch.einsum("jik,skj->sij", orc.L_base, zb))
    t0 = time.perf_counter()
    for s in range(box_samples):
        nondominated_cells(pareto_above_ref(obj_b[s], orc.ref), orc.ref)
    out["box_decomposition_s"] = (time.perf_counter() - t0) * acqf.S / box_samples
    r = ask["restarts"]
    t0 = time.perf_counter()
    with torch.no_grad():
        for k in range(2):
            orc.forward(Xc_cpu[k * r:(k + 1) * r].unsqueeze(1))
    out["raw_screening_s"] = (time.perf_counter() - t0) / (2 * r) * ask["raw_samples"]
    x = Xc_cpu[:r].clone().requires_grad_(True)
    t0 = time.perf_counter()
    orc.forward(x.unsqueeze(1)).sum().backward()
    opt_evals = ask["evals"] - ask["raw_samples"]
    out["restarts_s"] = (time.perf_counter() - t0) / r * opt_evals
    tot = sum(out.values())
    out = {k: round(v, 2) for k, v in out.items()}
    out["total_s"] = round(tot, 2)
    out["gpu_ask_s"] = ask["ask_s"]
    out["ask_speedup"] = round(tot / ask["ask_s"], 1)
    out["sample"] = (f"prune {prune_sub}/{prune_samples} draws, box decomposition {box_samples}/{acqf.S} samples, "
                     f"raw screening 2 chunks of {r}, one joint forward+backward of {r} restarts; "
                     f"{opt_evals} optimiser evaluations from the GPU ask")
    return out


class _OracleAcqf:
    """The oracle's reference-structure qNEHVI (torch-CPU fp64) behind optimize_acqf's
    acquisition protocol: forward in chunks of ``chunk`` candidates (BoTorch evaluates the raw
    samples in batch_limit chunks), forward_backward by autograd over the joint restart batch
    (gen_candidates_scipy's acq(X).sum().backward())."""

    dev = torch.device("cpu")

    def __init__(self, orc, chunk):
        self.orc, self.chunk = orc, chunk

    def forward(self, X):
        with torch.no_grad():
            return torch.cat([self.orc.forward(X[i:i + self.chunk].unsqueeze(1))
                              for i in range(0, X.shape[0], self.chunk)])

    def forward_backward(self, X):
        x = X.detach().clone().requires_grad_(True)
        v = self.orc.forward(x.unsqueeze(1))
        v.sum().backward()
        return v.detach(), x.grad


def cpu_full_ask(s, restarts, raw, S, seed=0):
    """One FULL, un-extrapolated reference-structure QnehviStrategy.ask() on the host cores
    (oracle/, torch-CPU fp64, BoTorch's computation shape) for the ask the GPU times: prune
    over 2048 posterior draws, S per-sample Python box decompositions, ``raw`` raw samples in
    chunks of batch_limit, then scipy L-BFGS-B over the joint ``restarts`` problem with the
    autograd gradient, on the GPU ask's fitted GPs.  Returns a dict of phase times and
    evaluation counts (minutes of CPU work: run with --cpu-full-ask, not by default)."""
    from everest_amd.optim import optimize_acqf
    from oracle import gp as ogp
    from oracle import qnehvi as oq

    states = []
    for sur in s.surrogates.surrogates:
        st = sur.state
        states.append(ogp.GPState(X=torch.tensor((st["X"] - st["lo"]) / (st["hi"] - st["lo"])),
                                  y=torch.tensor((st["y"] - st["y_mean"]) / st["y_std"]),
                                  lengthscale=torch.tensor(st["lengthscale"]), noise=st["noise"],
                                  constant=st["constant"], y_mean=st["y_mean"], y_std=st["y_std"]))
    m = len(states)
    Xn = states[0].X
    obj = oq.Objective(-torch.ones(m, dtype=torch.float64), torch.zeros(m, dtype=torch.float64))
    ref = torch.tensor(s.get_adjusted_refpoint(), dtype=torch.float64)
    out = {}
    t0 = time.perf_counter()
    # a heartbeat on stderr every 30 s (minutes of CPU work: a silent run looks hung)
    import threading

    stop = threading.Event()

    def beat():
        while not stop.wait(30.0):
            print(f"[cpu_full_ask] {time.perf_counter() - t0:.0f} s, phases done: {sorted(out)}", file=sys.stderr,
                  flush=True)

    threading.Thread(target=beat, daemon=True).start()
    zp = oq.base_samples(2048, Xn.shape[0], m, seed + 1)
    idx, _ = oq.prune_baseline(states, Xn, obj, ref, zp, chunk=32)
    out["prune_s"] = time.perf_counter() - t0
    nb = int(idx.shape[0])
    t1 = time.perf_counter()
    zb = oq.base_samples(S, nb, m, seed + 2)
    zn = oq.base_samples(S, nb + 1, m, seed + 2)[:, nb:nb + 1]
    orc = oq.QNEHVI(states, Xn[idx], obj, ref, zb, zn)
    out["baseline_and_box_decomposition_s"] = time.perf_counter() - t1
    gen = torch.Generator().manual_seed(seed)
    bounds = np.array([[0.0] * Xn.shape[1], [1.0] * Xn.shape[1]])
    x, v, st = optimize_acqf(_OracleAcqf(orc, restarts), bounds, restarts, raw,
                             {"batch_limit": restarts, "maxiter": 2000, "optimizer": "scipy"}, gen)
    out["raw_screening_s"] = st.t_raw
    out["restarts_s"] = st.t_opt
    out["total_s"] = time.perf_counter() - t0
    stop.set()
    out.update(n_base=nb, cells_total=int(sum(c.shape[1] for c in orc.cells)), raw_evals=st.raw_evals,
               opt_evals=st.opt_evals, optimizer_iterations=st.opt_iters, best_value=v,
               candidates_per_s=round((st.raw_evals + st.opt_evals) / out["total_s"], 3))
    return {k: (round(v, 3) if isinstance(v, float) else v) for k, v in out.items()}


def _traffic(path, key, launched):
    """Per-launch HBM bytes of op ``key`` from the committed PMC summary (FETCH_SIZE doubled
    per MI355X_MICROARCH.md's gfx950 correction, + WRITE_SIZE), or None.  The entry counts
    only if its PMC pass saw the kernel this run launches for the op (regex ``launched``
    against the entry's kernel names): a figure captured on an earlier kernel is dropped."""
    import re

    try:
        with open(path) as f:
            tab = json.load(f)
    except (OSError, ValueError):
        return None
    ent = tab.get(key)
    if not ent or "bytes_per_launch" not in ent or ent["bytes_per_launch"] <= 0:
        return None
    if not any(re.search(launched, k) for k in ent.get("kernels", [])):
        return None
    return ent


def _launched_kernel(acqf, op, b, d):
    """Regex of the kernel name(s) the evaluation chain launches for ``op`` at batch b."""
    from everest_amd import ops

    if op != "hvi_fwd_bwd":
        return {"kernel_matrix": r"kmat_kernel", "samples": r"qn_samples_norms",
                "proj_fwd": r"qs_fwd" if ops.qnehvi_small_applies(acqf.state, b, d) else r"Cijk_|qn_proj_fwd",
                "proj_bwd": r"qs_bwd" if ops.qnehvi_small_applies(acqf.state, b, d) else r"Cijk_|qn_proj_bwd",
                "kernel_grad": r"kcross_grad"}.get(op, re.escape(op))
    if ops.qnehvi_small_applies(acqf.state, b, d) and ops.hvi_restart_fb_applies(acqf.state, b):
        # the one-launch restart scan (hvi.hip hvi_kdw)
        return r"hvi_kdw<"
    return r"hvi_kd2?<|hvi_tiled<"


def make_ask_strategy(n: int, S: int, raw: int, restarts: int, world: int, dist=None, seed: int = 1,
                      batch_limit: int = 0):
    """QnehviStrategy of config 4 (DTLZ2(6, 5), n_train = n, S MC samples, ``raw`` Sobol raw
    samples, ``restarts`` L-BFGS-B restarts) through the BoFire-compatible API, fitted once
    (tell).  batch_limit = restarts at every N (the data model's default,
    bofire/data_models/strategies/predictives/botorch.py:101-108): one joint problem whose
    evaluations the ranks shard; raw screening is sharded over the ranks with an all-gather of
    the values.  ``batch_limit`` > 0 overrides it (1: every restart its own
    problem, the independent-restart layout BoFire forces under NChooseK / product
    constraints, bofire/strategies/predictives/botorch.py:114-126).  Returns (strategy, tell_s)."""
    import pandas as pd

    import everest_amd.data_models as dm
    from everest_amd import strategies
    from everest_amd.benchmarks import DTLZ2

    bm = DTLZ2(dim=6, num_objectives=5)
    Xd = pd.DataFrame(np.random.default_rng(0).uniform(size=(n, 6)), columns=bm.domain.inputs.get_keys())
    s = strategies.map(dm.QnehviStrategy(domain=bm.domain, ref_point=bm.ref_point, seed=seed, num_sobol_samples=S,
                                         num_raw_samples=raw, num_restarts=restarts,
                                         batch_limit=batch_limit or restarts), dist=dist)
    exps = bm.f(Xd, return_complete=True)
    times = []
    for _ in range(2):      # cold (first GPU work of the process: module loads, plan captures), then warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.tell(exps, replace=True)      # the same n training points both times
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    return s, times


def _ask_evals(s) -> int:
    """Acquisition evaluations of the last ask() over all ranks: raw samples + every
    optimiser function evaluation x its batch (SURVEY.md §8(d) "candidates/s" of ask)."""
    st = s.last_ask_stats
    return int(st.raw_evals + getattr(st, "opt_evals_global", st.opt_evals))


def _spawn_ranks(n: int) -> int:
    """``bench.py --gpus N`` without a launcher: start N fresh ranks (one process per GPU,
    torchrun-style env, RCCL rendezvous on 127.0.0.1) from a parent that never touches HIP,
    stop the others if one fails, and return the first non-zero exit code (else 0)."""
    import socket
    import subprocess

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    return rc


def _rooflines(ktimes, table):
    out = {}
    for k, (bound, w, unit) in table.items():
        if k not in ktimes:
            continue
        t = ktimes[k] * 1e-3
        if unit == "B":
            ach, peak, u = w / t / 1e9, PEAK_HBM_GBS, "GB/s"
        else:
            ach, peak, u = w / t / 1e12, PEAK_FP64_TFLOPS, "TFLOP/s"
        out[k] = {"bound": bound, "achieved": round(ach, 3), "peak": peak, "unit": u, "frac": round(ach / peak, 4),
                  "work_per_launch": w, "launch_ms": round(ktimes[k], 4)}
    return out


def _work_table(acqf, b, S, m, d, sum_cells):
    """SURVEY.md §8(d) algorithmic work per launch of each op at batch b: (bound, work, unit)."""
    Rr, n = acqf.Rr, acqf.nk
    nrt = math.ceil(Rr / 64)
    from everest_amd import ops

    if ops.qnehvi_small_applies(acqf.state, b, d):
        # restart batch: both projections stream the operator M (m x Rr x n) once with a
        # b-column right-hand side — HBM-bound, not matrix-core-bound; the backward also reads
        # the samples' gradient and writes dX (cross-covariance gradient fused)
        nrt16 = math.ceil(Rr / 16)
        return {
            "kernel_matrix": ("hbm", 8.0 * (m * n * b + n * d + b * d + m * d), "B"),
            "proj_fwd": ("hbm", 8.0 * (m * Rr * n + m * n * b + m * Rr * b + 2 * m * nrt16 * b), "B"),
            "samples": ("hbm", 8.0 * m * b * (S + 1 + 2 * nrt16) + 8.0 * S * m * b, "B"),
            "hvi_fwd_bwd": ("hbm", 16.0 * sum_cells * m + 8.0 * b * S * m + 8.0 * b, "B"),
            "proj_bwd": ("hbm", 8.0 * (m * Rr * n + m * Rr * b + S * m * b + n * d + b * d), "B"),
        }
    return {
        "kernel_matrix": ("hbm", 8.0 * (m * n * b + n * d + b * d + m * d), "B"),
        "proj_fwd": ("mfma", 2.0 * m * Rr * n * b, "flop"),
        "samples": ("hbm", 8.0 * m * b * (S + 1 + 2 * nrt) + 8.0 * S * m * b, "B"),
        # scan bytes with every cell read once per forward (explicit [lo, hi] rows, 16 m B per
        # cell) + the samples + the output
        "hvi_fwd_bwd": ("hbm", 16.0 * sum_cells * m + 8.0 * b * S * m + 8.0 * b, "B"),
        "proj_bwd": ("mfma", 2.0 * m * Rr * n * b, "flop"),
        "kernel_grad": ("hbm", 8.0 * (m * n * b + n * d + b * d), "B"),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10, help="timed ask() calls")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--d", type=int, default=6)
    ap.add_argument("--m", type=int, default=5)
    ap.add_argument("--S", type=int, default=256)
    ap.add_argument("--raw", type=int, default=1024)
    ap.add_argument("--restarts", type=int, default=20)
    ap.add_argument("--b", type=int, default=512, help="candidates per rank of the evaluation pass")
    ap.add_argument("--eval-steps", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-full-ask", default=None, metavar="JSON",
                    help="also run one FULL reference-structure ask on the host (minutes) and write it to JSON")
    ap.add_argument("--no-eval-pass", action="store_true", help="skip the b-candidate evaluation-pass figures")
    ap.add_argument("--no-config1", action="store_true", help="skip the configs[0] Detergent ask/tell loop timing")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "hbm_traffic.json"),
                    help="per-launch HBM bytes from a rocprofv3 --pmc pass (tools/pmc_traffic.py)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_spawn_ranks(args.gpus))            # parent: no HIP call before the ranks start
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # EVR_DIST_BACKEND=gloo: a multi-rank rehearsal of the sharded path on fewer GPUs than
    # ranks (ranks share devices round-robin, exchanges through host memory); default RCCL
    backend = os.environ.get("EVR_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)
        world = dist.get_world_size()

    def maxed(dt):
        if dist is None:
            return dt
        tt = torch.tensor([dt], device=device if backend != "gloo" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return tt.item()

    def sync():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    # ---- the step: one full QnehviStrategy.ask() of config 4 per rank.  One ask is a
    # sequential, latency-bound optimisation (the joint L-BFGS-B over the restarts: every
    # iteration waits for the previous one's evaluation), so N GPUs do not shorten it; they
    # serve N asks.  N > 1: replicas — every rank runs the complete N = 1 workload (its own
    # strategy, seed 1 + rank) with no collective in the timed region; value = the asks'
    # evaluations summed over ranks / max-over-ranks time (weak scaling).  The single ask
    # sharded over the ranks (config 4's RCCL layout) is timed afterwards: "sharded_ask". ----
    s, t_tells = make_ask_strategy(args.n, args.S, args.raw, args.restarts, world, None, seed=1 + rank)
    for _ in range(args.warmup):
        s.ask(1)
    sync()
    t0 = time.perf_counter()
    evals = 0
    for _ in range(args.steps):
        s.ask(1)
        evals += _ask_evals(s)
    sync()
    dt = maxed(time.perf_counter() - t0)
    if dist is not None:
        et = torch.tensor([float(evals)], device=device if backend != "gloo" else "cpu")
        dist.all_reduce(et)
        evals = int(et.item())
    value = evals / dt
    ms = dt / args.steps * 1e3
    sharded = None
    if dist is not None:
        s2, _ = make_ask_strategy(args.n, args.S, args.raw, args.restarts, world, dist, seed=1)
        for _ in range(max(1, args.warmup)):
            s2.ask(1)
        sync()
        t1 = time.perf_counter()
        ev2 = 0
        for _ in range(args.steps):
            s2.ask(1)
            ev2 += _ask_evals(s2)
        sync()
        dt2 = maxed(time.perf_counter() - t1)
        st2 = s2.last_ask_stats
        sharded = {"ms_per_ask": round(dt2 / args.steps * 1e3, 3), "evals_per_s": round(ev2 / dt2, 1),
                   "evals_per_ask": round(ev2 / args.steps, 1), "ranks": world,
                   "driver": st2.chunks[0]["driver"] if st2.chunks else None,
                   "note": "the same config-4 ask as N = 1 (seed 1) with its raw screening sharded and its joint "
                           "restart problem evaluated by all ranks (all-gather per L-BFGS-B evaluation); "
                           "latency-bound, so not faster than one GPU"}
        del s2
    acqf_ask = s.last_acqf
    st_ask = s.last_ask_stats
    tm = getattr(acqf_ask, "timings", {})
    phases = {"construction_s": round(tm.get("total", 0.0), 4), "construction": {k: round(v, 4) for k, v in tm.items()},
              "raw_screening_s": round(st_ask.t_raw, 4), "restarts_s": round(st_ask.t_opt, 4),
              "optimizer_iterations": st_ask.opt_iters, "evals_last_ask": _ask_evals(s),
              "driver": st_ask.chunks[0]["driver"] if st_ask.chunks else None}

    # per-op device time at the restart batch one rank evaluates per L-BFGS-B iteration, on
    # the candidates the restarts converged to (the scan's work depends on where the
    # candidates sit: optimised points dominate more cells than random ones)
    sl = st_ask.restart_slice
    b_r = (sl.stop - sl.start) if sl is not None else math.ceil(args.restarts / world)
    if st_ask.restart_X is not None and sl is not None and b_r > 0:
        Xr = torch.as_tensor(np.ascontiguousarray(st_ask.restart_X[sl].reshape(b_r, -1)), dtype=torch.float64,
                             device=device)
        xr_note = "the last ask's optimised restart candidates (this rank's slice)"
    else:
        Xr = candidates(b_r, args.d, seed=5 + rank, device=device)
        xr_note = "Sobol candidates"
    kt_r, how = kernel_times(acqf_ask, Xr)

    eval_pass, kernels_b = None, None
    X = Y = hypers = acqf = None
    if not args.no_eval_pass:
        # ---- evaluation pass: b candidates per rank through the native plan (raw-screening unit)
        X, Y, gp, hypers, acqf, t_fit, t_build = build_state(args.n, args.d, args.m, args.S, device)
        Xc = candidates(args.b, args.d, seed=2 + rank, device=device)
        gathered = [torch.empty(args.b, dtype=torch.float64, device=device) for _ in range(world)]
        plan = acqf.plan(args.b, True)
        plan.X.copy_(Xc)

        def one_pass():
            plan.run()
            if dist is not None:
                if backend == "gloo":
                    dist.all_gather([g.cpu() for g in gathered], plan.acq.cpu())
                else:
                    dist.all_gather(gathered, plan.acq)

        for _ in range(3):
            one_pass()
        sync()
        t0 = time.perf_counter()
        for _ in range(args.eval_steps):
            one_pass()
        sync()
        dte = maxed(time.perf_counter() - t0)
        kt_b, _ = kernel_times(acqf, Xc)
        if rank == 0:
            sum_cells = acqf.stats.total_cells
            kernels_b = _rooflines(kt_b, _work_table(acqf, args.b, args.S, args.m, args.d, sum_cells))
            counts = scan_counts(acqf, Xc)
            if "hvi_fwd_bwd" in kernels_b:
                t = kt_b["hvi_fwd_bwd"] * 1e-3
                useful = counts["terms"] * (6 * args.m + 2)
                kernels_b["hvi_fwd_bwd"]["valu_useful"] = {
                    "achieved": round(useful / t / 1e12, 3), "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(useful / t / 1e12 / PEAK_FP64_TFLOPS, 4), "work_per_launch": float(useful),
                    "note": "(6m+2) flop per evaluated (cell, candidate) term, device-counted"}
                kernels_b["hvi_fwd_bwd"]["scan"] = {
                    "dense_pairs": args.b * sum_cells, "group_tests": counts["group_tests"],
                    "group_pairs": counts["group_pairs"], "terms": counts["terms"]}
                tr = _traffic(args.traffic_json, "hvi_fwd_bwd", _launched_kernel(acqf, "hvi_fwd_bwd", args.b, args.d))
                if tr is not None:
                    kernels_b["hvi_fwd_bwd"]["traffic"] = tr["bytes_per_launch"]
                    kernels_b["hvi_fwd_bwd"]["traffic_source"] = tr["source"]
            eval_pass = {"value": round(world * args.b * args.eval_steps / dte, 1), "unit": "candidates/s",
                         "ms_per_step": round(dte / args.eval_steps * 1e3, 4), "candidates_per_rank": args.b,
                         "note": "one qNEHVI forward + analytic backward over b Sobol candidates resident in HBM "
                                 "through the native plan (the unit raw screening and restarts are made of)",
                         "kernel_ms": {k: round(v, 4) for k, v in kt_b.items()}, "kernels": kernels_b,
                         "n_base": acqf.nb, "cells_total": sum_cells, "cells_max": acqf.stats.max_cells,
                         "box_decomposition": acqf.box_path, "setup_s": {"gp_fit": round(t_fit, 3),
                                                                         "qnehvi_build": round(t_build, 3)}}

    qlog = None
    if not args.no_eval_pass and rank == 0:
        # ---- qLogNEHVI (MoboStrategy's default acquisition) on the same fitted GPs: the dense
        # log-space scan (hvi_log.hip) over every cell, forward + backward, HIP events
        from everest_amd.acquisition import QLogNEHVI

        qa = QLogNEHVI(gp, X, X, -1.1 * np.ones(args.m), -np.ones(args.m), np.zeros(args.m), S=args.S,
                       sampler_seed=1234, prune_baseline=True, prune_seed=4321)
        qlog = {"note": "qLogNEHVI forward + backward (tabulated fat-smoothed log scan over every compressed "
                        "cell), same GPs and seeds as eval_pass; device time between HIP events incl. any host "
                        "syncs",
                "cells_total": qa.stats.total_cells, "box_decomposition": qa.box_path}
        for bb, XX in ((args.b, Xc), (b_r, Xr)):
            qlog[f"b{bb}_ms"] = round(_event_ms(lambda: qa.forward_backward(XX), reps=10), 4)
        del qa

    if rank == 0:
        sum_cells_r = acqf_ask.stats.total_cells
        kernels_r = _rooflines(kt_r, _work_table(acqf_ask, b_r, args.S, args.m, args.d, sum_cells_r))
        dom = max(kt_r, key=kt_r.get)
        roof = None
        if dom in kernels_r:
            r = kernels_r[dom]
            roof = {"bound": r["bound"], "kernel": dom, "achieved": r["achieved"], "peak": r["peak"],
                    "unit": r["unit"], "frac": r["frac"], "traffic": None,
                    "algorithmic_work_per_launch": r["work_per_launch"], "launch_ms": r["launch_ms"],
                    "batch": f"{b_r} restart candidates (one L-BFGS-B evaluation of this rank's chunk)"}
            tr = _traffic(args.traffic_json, f"{dom}@b{b_r}", _launched_kernel(acqf_ask, dom, b_r, args.d))
            if tr is not None:
                roof["traffic"] = tr["bytes_per_launch"]
                roof["traffic_source"] = tr["source"]
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
            threads = max(1, min(share, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))
            torch.set_num_threads(threads)
            if X is None:
                X, Y, gp, hypers, acqf, _, _ = build_state(args.n, args.d, args.m, args.S, device)
            Xcc = candidates(max(args.b, 2 * args.restarts), args.d, seed=2, device=device).cpu()
            t_cpu, nc, orc, ostates = cpu_baseline(acqf, hypers, X, Y, Xcc, budget_s=6.0)
            ask_info = {"restarts": args.restarts, "raw_samples": args.raw, "evals": _ask_evals(s),
                        "ask_s": round(ms * 1e-3, 4)}
            est = cpu_ask_estimate(orc, ostates, acqf, Xcc, ask_info)
            cpu = {"value": round(ask_info["evals"] / est["total_s"], 2), "unit": "candidates/s", "cores": threads,
                   "kind": "port",
                   "sample": "reference-structure QnehviStrategy.ask() on the host (oracle/, torch-CPU fp64, "
                             "BoTorch's computation shape) for the same ask: " + est["sample"] +
                             f"; {est['total_s']} s estimated per ask",
                   "ask_estimate": est,
                   "eval_pass_cpu": {"value": round(nc / t_cpu, 3), "unit": "candidates/s",
                                     "sample": f"forward+backward of {nc} candidates in chunks of 8, {t_cpu:.1f} s"},
                   "cores_note": f"{threads} threads = this job's CPU share (OMP_NUM_THREADS; affinity mask "
                                 f"{share}, os.cpu_count {os.cpu_count()})"}
            full_path = args.cpu_full_ask or os.path.join(ROOT, "profiles", "cpu_full_ask.json")
            if args.cpu_full_ask:
                full = cpu_full_ask(s, args.restarts, args.raw, args.S)
                full.update(cores=threads, gpu_ask_s=round(ms * 1e-3, 4))
                with open(args.cpu_full_ask, "w") as f:
                    json.dump(full, f, indent=1)
            try:
                with open(full_path) as f:
                    full = json.load(f)
                cpu["full_ask_measured"] = dict(full, source=os.path.relpath(full_path, ROOT),
                                                note="one complete un-extrapolated reference-structure ask on the "
                                                     "host cores (bench.py --cpu-full-ask)")
            except (OSError, ValueError):
                pass
            torch.set_num_threads(1)
            t1, n1, _, _ = cpu_baseline(acqf, hypers, X, Y, Xcc, budget_s=4.0)
            cpu["eval_pass_cpu"]["single_thread"] = {"value": round(n1 / t1, 3), "cores": 1,
                                                     "sample": f"{n1} candidates, {t1:.1f} s"}
            torch.set_num_threads(threads)
        gp_ask = s.model
        t_post = gp_posterior_ms(device, gp=gp_ask)
        cfg1 = None if args.no_config1 else config1_loop()
        out = {
            "metric": "QnehviStrategy.ask() candidates/sec + GP posterior ms, n=512 d=6 m=5",
            "value": round(value, 1),
            "unit": "candidates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (DTLZ2 d=6 m=5 train set; GPs fitted on device by tell())",
            "config": {"workload": "full QnehviStrategy.ask() of BASELINE configs[3] (config 4): DTLZ2(d=6,m=5), "
                                   f"n_train={args.n}, S={args.S} MC samples, {args.raw} raw Sobol candidates + "
                                   f"{args.restarts} L-BFGS-B restarts, q=1; value = (raw + optimiser "
                                   "evaluations x batch) / ask wall time, SURVEY.md §8(d)",
                       "n_train": args.n, "d": args.d, "m": args.m, "mc_samples": args.S, "raw_samples": args.raw,
                       "restarts": args.restarts, "batch_limit": args.restarts,
                       "parallelism": (f"replicas: {world} ranks, one full ask each (seeds 1..{world}), no "
                                       "collective in the timed region; the single ask sharded over the ranks in "
                                       "sharded_ask" if world > 1 else "1 rank")},
            "roofline": roof,
            "kernels": kernels_r,
            "kernel_ms": {k: round(v, 4) for k, v in kt_r.items()},
            "kernel_ms_method": f"{how} of 10 launches per op between HIP events (torch current stream), "
                                f"batch {b_r}: {xr_note}",
            "ask": {"ask_s": round(ms * 1e-3, 4), "evals_per_ask": round(evals / args.steps, 1), "tell_s": round(t_tells[1], 3),
                    "tell_cold_s": round(t_tells[0], 3),
                    "phases_last_ask": phases, "n_base": acqf_ask.nb, "cells_total": sum_cells_r,
                    "box_decomposition": acqf_ask.box_path},
            "sharded_ask": sharded,
            "eval_pass": eval_pass,
            "qlognehvi": qlog,
            "linalg": cholesky_figures(device),
            "cpu_baseline": cpu,
            "gp_posterior_ms": round(t_post, 4),
            "gp_posterior": {"ms": round(t_post, 4), "shape": f"n_train={args.n} d={args.d} m={args.m} (the ask's "
                             "fitted model), 1024 test points, mean+var, HIP events",
                             "config2_ms": round(gp_posterior_ms(device), 4)},
            "config1": cfg1,
            "build": build_provenance(),
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
