#!/usr/bin/env python
"""Benchmark of the qNEHVI hot path on MI355X (BASELINE.json metric: QnehviStrategy.ask()
candidates/sec + GP posterior ms, n=512 d=6 m=5).

Workload (BASELINE.json configs[2]): DTLZ2(dim=6, m=5), X_train ~
U[0,1]^6 (n=512, seed 0), noise-free Y, reference point 1.1 -> -1.1 in objective space
(MinimizeObjective), 5 exact RBF GPs fitted once on the device and frozen, qNEHVI built as
BoFire builds it (prune_baseline with 2048 samples, cached root, S=256 Sobol-normal base
samples), q=1.  A *step* = one acquisition evaluation pass (forward + analytic backward,
the unit raw screening and the L-BFGS restarts of ask() are made of) over one batch of
b=512 Sobol candidates already resident in HBM, run through the native evaluation plan
(everest_amd/csrc/qnehvi_plan.hip — the path ask() uses); the per-kernel breakdown comes
from a separate instrumented pass over the same kernels launched one by one.

Multi-GPU (torchrun, one process per GPU, RCCL): every rank evaluates its own 512-candidate
shard (weak scaling); each step ends with the RCCL all-gather of the per-shard acquisition
values that the Boltzmann initial-condition selection needs.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import math
import os
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


class KernelTimer:
    """HIP events on torch's current stream (the stream every everest_amd op launches on)."""

    def __init__(self):
        self.ev = {}

    def start(self, name):
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        return (name, e0)

    def stop(self, tok):
        name, e0 = tok
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self.ev.setdefault(name, []).append((e0, e1))

    def summary(self):
        return {k: float(np.mean([a.elapsed_time(b) for a, b in v])) for k, v in self.ev.items()}


def step(acqf, Xc, timer=None):
    """One evaluation pass: forward + backward over the candidate batch (instrumented)."""
    from everest_amd import ops

    st = acqf.state
    b = Xc.shape[0]
    gp = acqf.gp
    T = timer
    tk = T.start("kernel_matrix") if T else None
    Kx = gp.cross(Xc)
    if T: T.stop(tk); tk = T.start("proj_fwd")
    R, P = ops.qnehvi_project(st, acqf.M, Kx, b)
    if T: T.stop(tk); tk = T.start("samples")
    G, L22, flags = ops.qnehvi_samples_norms(st, R, P, b)
    if T: T.stop(tk); tk = T.start("hvi_fwd_bwd")
    acq, dG = ops.hvi_forward_backward(st, G, b, flags)
    if T: T.stop(tk); tk = T.start("proj_bwd")
    dKx = ops.qnehvi_project_backward(st, acqf.M, R, L22, dG, b)
    if T: T.stop(tk); tk = T.start("kernel_grad")
    dX = ops.kernel_cross_grad(gp.Xn, Xc, gp.ls, dKx, gp.kind, shift2=gp.lo, scale2=gp.inv_range)
    if T: T.stop(tk)
    return acq, dX


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


def gp_posterior_ms(device, reps=20):
    """Config 2: SingleTaskGP RBF posterior (mean+var), n_train=256, d=6, 1024 test points."""
    from everest_amd.gp import GPBatch, GPHyper

    rng = np.random.default_rng(0)
    X = rng.uniform(size=(256, 6))
    y = dtlz2(X, 5)[:, :1]
    h = GPHyper(lengthscale=np.full(6, 0.8), noise=1e-3, constant=0.0, y_mean=float(y.mean()),
                y_std=float(y.std(ddof=1)))
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=device)  # noqa: E731
    gp = GPBatch(t(X), t(y), [h], 0, t(np.zeros(6)), t(np.ones(6)))
    Xs = torch.quasirandom.SobolEngine(6, scramble=True, seed=1).draw(1024, dtype=torch.float64).to(device)
    for _ in range(3):
        gp.posterior(Xs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        gp.posterior(Xs)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def cpu_baseline(acqf, hypers, X, Y, Xc_cpu, chunk=8, budget_s=15.0):
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
    return spent, done


def _traffic(path, kernel):
    """Per-launch HBM bytes of ``kernel`` from the committed PMC summary (FETCH_SIZE doubled
    per MI355X_MICROARCH.md's gfx950 correction, + WRITE_SIZE), or None."""
    try:
        with open(path) as f:
            tab = json.load(f)
    except (OSError, ValueError):
        return None
    ent = tab.get(kernel)
    return ent if ent and "bytes_per_launch" in ent else None


def ask_throughput(n: int, S: int, raw: int = 1024, restarts: int = 20, asks: int = 2):
    """Full QnehviStrategy.ask() (config 4 shape on one GPU: 1024 raw Sobol candidates +
    20 L-BFGS-B restarts, q=1) through the BoFire-compatible strategy API; returns the
    median ask() wall time and acquisition evaluations / s (raw + optimizer evaluations)."""
    import pandas as pd

    import everest_amd.data_models as dm
    from everest_amd import strategies
    from everest_amd.benchmarks import DTLZ2

    bm = DTLZ2(dim=6, num_objectives=5)
    Xd = pd.DataFrame(np.random.default_rng(0).uniform(size=(n, 6)), columns=bm.domain.inputs.get_keys())
    s = strategies.map(dm.QnehviStrategy(domain=bm.domain, ref_point=bm.ref_point, seed=1, num_sobol_samples=S,
                                         num_raw_samples=raw, num_restarts=restarts))
    t0 = time.perf_counter()
    s.tell(bm.f(Xd, return_complete=True))
    torch.cuda.synchronize()
    t_tell = time.perf_counter() - t0
    s.ask(1)  # warm-up (first construction pays one-time allocations)
    ts, evals = [], []
    for _ in range(asks):
        t0 = time.perf_counter()
        s.ask(1)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
        st = s.last_ask_stats
        evals.append(st.raw_evals + st.opt_evals)
    i = int(np.argsort(ts)[len(ts) // 2])
    return {"ask_s": round(ts[i], 4), "evals": int(evals[i]), "evals_per_s": round(evals[i] / ts[i], 1),
            "tell_s": round(t_tell, 3), "raw_samples": raw, "restarts": restarts, "mc_samples": S}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--d", type=int, default=6)
    ap.add_argument("--m", type=int, default=5)
    ap.add_argument("--S", type=int, default=256)
    ap.add_argument("--b", type=int, default=512)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ask", action="store_true", help="skip the full QnehviStrategy.ask() timing")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "hbm_traffic.json"),
                    help="per-launch HBM bytes from a rocprofv3 --pmc pass (tools/pmc_traffic.py)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=device)

    X, Y, gp, hypers, acqf, t_fit, t_build = build_state(args.n, args.d, args.m, args.S, device)
    Xc = candidates(args.b, args.d, seed=2 + rank, device=device)
    gathered = [torch.empty(args.b, dtype=torch.float64, device=device) for _ in range(world)]

    # production path: the native evaluation plan (whole chain in one C-ABI call / hipGraph),
    # candidates already resident in its HBM input buffer
    plan = acqf.plan(args.b, True)
    plan.X.copy_(Xc)

    def one_step(timer=None):
        if timer is None:
            plan.run()
            acq = plan.acq
        else:                       # instrumented op-by-op chain (same kernels) for the breakdown
            acq, _ = step(acqf, Xc, timer)
        if dist is not None:
            dist.all_gather(gathered, acq)
        return acq

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([dt], device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = tt.item()
    ms = dt / args.steps * 1e3
    value = world * args.b * args.steps / dt

    # per-kernel device time (separate instrumented pass, events on the launch stream)
    timer = KernelTimer()
    for _ in range(max(5, args.steps // 2)):
        one_step(timer)
    torch.cuda.synchronize()
    ktimes = timer.summary()

    if rank == 0:
        st = acqf.stats
        sum_cells = st.total_cells
        m = args.m
        b = args.b
        # per-kernel rooflines (SURVEY.md §8(d) work per unit x units per launch / launch time)
        Rr, n, d = acqf.Rr, args.n, args.d
        nrt = math.ceil(Rr / 64)
        counts = scan_counts(acqf, Xc)
        hvi_useful = counts["terms"] * (6 * m + 2)
        table = {
            # (bound, work, unit): bytes for HBM-bound kernels, flops otherwise
            "kernel_matrix": ("hbm", 8.0 * (m * n * b + n * d + b * d + m * d), "B"),
            "proj_fwd": ("mfma", 2.0 * m * Rr * n * b, "flop"),
            "samples": ("hbm", 8.0 * m * b * (args.S + 1 + 2 * nrt) + 8.0 * args.S * m * b, "B"),
            "hvi_fwd_bwd": ("valu", float(hvi_useful), "flop"),
            "proj_bwd": ("mfma", 2.0 * m * Rr * n * b, "flop"),
            "kernel_grad": ("hbm", 8.0 * (m * n * b + n * d + b * d), "B"),
        }
        kernels = {}
        for k, (bound, w, unit) in table.items():
            if k not in ktimes:
                continue
            t = ktimes[k] * 1e-3
            if unit == "B":
                ach, peak, u = w / t / 1e9, PEAK_HBM_GBS, "GB/s"
            else:
                ach, peak, u = w / t / 1e12, PEAK_FP64_TFLOPS, "TFLOP/s"
            kernels[k] = {"bound": bound, "achieved": round(ach, 3), "peak": peak, "unit": u,
                          "frac": round(ach / peak, 4), "work_per_launch": w, "launch_ms": round(ktimes[k], 4)}
        dom = max(ktimes, key=ktimes.get)
        roof = None
        if dom in kernels:
            r = kernels[dom]
            roof = {"bound": r["bound"], "kernel": dom, "achieved": r["achieved"], "peak": r["peak"],
                    "unit": r["unit"], "frac": r["frac"], "traffic": None,
                    "algorithmic_work_per_launch": r["work_per_launch"], "launch_ms": r["launch_ms"]}
            tr = _traffic(args.traffic_json, dom)
            if tr is not None:
                roof["traffic"] = tr["bytes_per_launch"]
                roof["traffic_source"] = tr["source"]
        if "hvi_fwd_bwd" in kernels:
            kernels["hvi_fwd_bwd"]["scan"] = {
                "dense_pairs": b * sum_cells, "group_tests": counts["group_tests"], "group_pairs": counts["group_pairs"],
                "terms": counts["terms"],
                "dense_equivalent_TFLOPs": round(b * sum_cells * (6 * m + 2) / (ktimes["hvi_fwd_bwd"] * 1e-3) / 1e12, 2)}
        cpu = None
        if not args.no_cpu_baseline:
            torch.set_num_threads(min(16, os.cpu_count() or 1))
            t_cpu, nc = cpu_baseline(acqf, hypers, X, Y, Xc.cpu())
            cpu = {"value": round(nc / t_cpu, 3), "unit": "candidates/s", "cores": torch.get_num_threads(),
                   "kind": "port", "sample": f"oracle reference-structure forward+backward over the first {nc} "
                   f"of the same {b} candidates in chunks of 8 (batch_limit), same state (n={args.n}, "
                   f"n_base={acqf.nb}, S={args.S}), {t_cpu:.1f} s of CPU wall time"}
        ask = None
        if world == 1 and not args.no_ask:
            ask = ask_throughput(args.n, args.S)
        out = {
            "metric": "QnehviStrategy.ask() candidates/sec + GP posterior ms, n=512 d=6 m=5",
            "value": round(value, 2),
            "unit": "candidates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (DTLZ2 d=6 m=5 train set, Sobol candidates; GPs fitted on device)",
            "config": {"workload": "qNEHVI fwd+bwd eval pass, DTLZ2(d=6,m=5) n_train=512 S=256 b=512 q=1",
                       "n_train": args.n, "d": args.d, "m": m, "mc_samples": args.S, "candidates_per_gpu": b,
                       "n_base": acqf.nb, "cells_total": sum_cells, "cells_max": st.max_cells,
                       "parallelism": f"candidate-shard x{world}"},
            "roofline": roof,
            "kernels": kernels,
            "cpu_baseline": cpu,
            "gp_posterior_ms": round(gp_posterior_ms(device), 4),
            "kernel_ms": {k: round(v, 4) for k, v in ktimes.items()},
            "setup_s": {"gp_fit": round(t_fit, 3), "qnehvi_build": round(t_build, 3)},
            "ask": ask,
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
