"""Per-wave wall-clock records of the sparse HVI scan (EVR_KD_PROF=1 build via EVR_LIB_PATH):
span of the launch, wave durations, dispatch skew and per-sample load, at the restart batch
(b = 20, Sobol and optimised candidates) and the evaluation pass (b = 512).  s_memrealtime
runs at 100 MHz, so times are in units of 10 ns (reported in us)."""
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
out = {}
NW = 1 << 17
for tag, Xc in (("b20", bench.candidates(20, 6, seed=2, device=dev)), ("b20opt", Xopt),
                ("b512", bench.candidates(512, 6, seed=2, device=dev))):
    b = Xc.shape[0]
    R, P = ops.qnehvi_project(acqf.state, acqf.M, gp.cross(Xc), b)
    G, L22, flags = ops.qnehvi_samples_norms(acqf.state, R, P, b)
    ops.hvi_forward_backward(acqf.state, G, b, flags)     # warm
    ctr = torch.zeros(16 + 8 * NW, dtype=torch.int64, device=dev)
    acqf.state.scan_counters = ctr.data_ptr()
    ops.hvi_forward_backward(acqf.state, G, b, flags)
    torch.cuda.synchronize()
    acqf.state.scan_counters = None
    c = ctr.cpu().numpy()
    rec = c[16:].reshape(-1, 8)
    widx = np.nonzero(rec[:, 3] > 0)[0] % 4      # wave of its workgroup
    rec = rec[rec[:, 3] > 0]
    t0 = rec[:, 0].min()
    st, en = (rec[:, 0] - t0) / 100.0, (rec[:, 3] - t0) / 100.0   # us
    dur = en - st
    stage = (rec[:, 1] - rec[:, 0]) / 100.0
    prefix = (rec[:, 2] - rec[:, 1]) / 100.0
    rest = (rec[:, 3] - rec[:, 2]) / 100.0
    samp = np.bincount(rec[:, 4].astype(int), weights=dur)
    q = lambda a, x: round(float(np.percentile(a, x)), 2)
    pct = lambda a: dict(mean=round(float(a.mean()), 2), p50=q(a, 50), p90=q(a, 90), max=q(a, 100))
    npairs, nterms = rec[:, 6].astype(float), rec[:, 7].astype(float)
    # least squares: windows-and-rounds time ~ a + b * pairs/64 + c * terms/64
    A = np.c_[np.ones(len(rec)), np.ceil(npairs / 64), np.ceil(nterms / 64)]
    coef = np.linalg.lstsq(A, rest, rcond=None)[0]
    top = np.argsort(-dur)[:5]
    out[tag] = dict(waves=int(len(rec)), span_us=round(float(en.max()), 2), start_us=pct(st), dur_us=pct(dur),
                    stage_us=pct(stage), groupA_prefix_us=pct(prefix), windows_us=pct(rest),
                    pairs=pct(npairs), terms=pct(nterms),
                    fit_windows_us=dict(fixed=round(coef[0], 3), per_B_window=round(coef[1], 3),
                                        per_C_round=round(coef[2], 3)),
                    longest=[dict(dur=round(float(dur[i]), 2), stage=round(float(stage[i]), 2),
                                  prefix=round(float(prefix[i]), 2), pairs=int(npairs[i]), terms=int(nterms[i]),
                                  sample=int(rec[i, 4]), split=int(rec[i, 5])) for i in top],
                    by_split={int(k): dict(terms=round(float(nterms[rec[:, 5] == k].mean()), 1),
                                           dur=round(float(dur[rec[:, 5] == k].mean()), 2))
                              for k in np.unique(rec[:, 5])},
                    by_wave={int(k): dict(terms=round(float(nterms[widx == k].mean()), 1),
                                          dur=round(float(dur[widx == k].mean()), 2)) for k in range(4)},
                    sample_wave_us=dict(mean=round(float(samp.mean()), 2), max=round(float(samp.max()), 2)))
print(json.dumps(out, indent=1))
