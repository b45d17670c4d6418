"""Per-wave wall-clock records of the one-launch restart scans (hvi_kd3, hvi_kdb) on the EVR_KD_PROF=2
build (EVR_LIB_PATH=everest_amd/_libprof/libeverest_amd.so): per phase — staging, thresholds,
filter + prefix, cell windows + term rounds, final reduction — the mean / p90 / max over waves,
the launch span, and per-sample totals, at b = 20 on Sobol and optimised restart candidates.
s_memrealtime runs at 100 MHz (10 ns units, reported in us).  One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
from everest_amd import ops

dev = torch.device("cuda", 0)
X, Y, gp, hypers, acqf, _, _ = bench.build_state(512, 6, 5, 256, dev)
p = acqf.plan(20, True)
xo, _, _ = p.minimize(np.random.default_rng(0).uniform(size=20 * 6), np.zeros(120), np.ones(120), 2000)
Xopt = torch.tensor(np.asarray(xo).reshape(20, 6), device=dev)
from everest_amd import _native

lib = _native.load()
out = {}
for variant, tag, Xc in ((1, "kd3_b20opt", Xopt), (2, "kdb_b20", bench.candidates(20, 6, seed=2, device=dev)),
                         (2, "kdb_b20opt", Xopt)):
    _native.check(lib.evr_hvi_set_restart_variant(variant), "set variant")
    b = Xc.shape[0]
    R, P = ops.qnehvi_project(acqf.state, acqf.M, gp.cross(Xc), b)
    G, L22, flags = ops.qnehvi_samples_norms(acqf.state, R, P, b)
    ops.hvi_restart_fb(acqf.state, G, b)
    S = int(acqf.state.S)
    ctr = torch.zeros(16 + 8 * S * 16, dtype=torch.int64, device=dev)
    acqf.state.scan_counters = ctr.data_ptr()
    ops.hvi_restart_fb(acqf.state, G, b)
    torch.cuda.synchronize()
    acqf.state.scan_counters = None
    rec = ctr.cpu().numpy()[16:].reshape(S, 16, 8)
    # the launch's device time (10 launches captured in one graph, HIP events; uninstrumented
    # timing needs the production library: this build adds the stamps only)
    gph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gph):
        for _ in range(10):
            ops.hvi_restart_fb(acqf.state, G, b)
    gph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gph.replay()
    e1.record()
    torch.cuda.synchronize()
    launch_us = round(e0.elapsed_time(e1) * 100.0, 2)
    if not rec[:, :, 0].any():      # production build: no stamps, the launch time only
        out[tag] = dict(launch_us=launch_us)
        continue
    if variant == 2:
        t0 = rec[:, :, 0].min()
        T = (rec[:, :, :7] - t0) / 100.0
        names = ["stage", "thresholds", "A_entries", "B_pairs", "C_terms", "final"]
        q = lambda a, x: round(float(np.percentile(a, x)), 2)
        stat = lambda a: dict(mean=round(float(a.mean()), 2), p90=q(a, 90), max=q(a, 100))
        wg_span = T[:, :, 6].max(1) - T[:, :, 0].min(1)
        out[tag] = dict(launch_us=launch_us, span_us=round(float(T[:, :, 6].max()), 2), wg_span=stat(wg_span),
                        phases={nm: stat(T[:, :, k + 1] - T[:, :, k]) for k, nm in enumerate(names)},
                        terms_per_wave=stat(rec[:, :, 7].astype(float)),
                        terms_per_sample=stat(rec[:, :, 7].sum(1).astype(float)))
        continue
    act = (rec[:, :, 7] >> 48) & 1
    t0 = rec[:, :, 0].min()
    T = (rec[:, :, :6] - t0) / 100.0
    ph = {"stage": T[:, :, 1] - T[:, :, 0], "thresholds": T[:, :, 2] - T[:, :, 1],
          "filter_prefix": T[:, :, 3] - T[:, :, 2], "terms": T[:, :, 4] - T[:, :, 3],
          "reduce_wait": T[:, :, 5] - T[:, :, 4]}
    q = lambda a, x: round(float(np.percentile(a, x)), 2)
    stat = lambda a: dict(mean=round(float(a.mean()), 2), p90=q(a, 90), max=q(a, 100))
    a = act.astype(bool)
    terms = (rec[:, :, 7] & ((1 << 40) - 1)).astype(float)
    pairs = rec[:, :, 6].astype(float)
    wg_span = T[:, :, 5].max(1) - T[:, :, 0].min(1)
    out[tag] = dict(launch_us=launch_us, span_us=round(float(T[:, :, 5].max()), 2),
                    start_skew_us=stat(T[:, :, 0].min(1)),
                    wg_span=stat(wg_span), phases={k: stat(v[a]) for k, v in ph.items()},
                    terms_per_wave=stat(terms[a]), pairs_per_wave=stat(pairs[a]),
                    terms_per_sample=stat(terms.sum(1)), slowest_samples=np.argsort(-wg_span)[:5].tolist(),
                    slowest_sample_terms=terms.sum(1)[np.argsort(-wg_span)[:5]].tolist())
_native.check(lib.evr_hvi_set_restart_variant(2), "set variant")
print(json.dumps(out))
