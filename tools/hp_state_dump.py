"""Dump the BASELINE config-3 state (DTLZ2(6, 5), n = 512, S = 256, the bench's fitted GPs and
pruned baseline) and the device's qNEHVI / qLogNEHVI values and gradients at the candidates the
high-precision truth (tools/hp_truth.py) adjudicates:

* ``sobol20``: the b = 20 Sobol batch of seed 2 (the restart-batch size; r05aw's c = 12, 8, 14,
  7, 15 are in it);
* ``near16``: 16 candidates placed 1e-2 ... 1e-6 (log-spaced) from training points in seeded
  random directions, 12 next to baseline rows (where the new point's variance given the
  baseline samples cancels) and 4 next to non-baseline rows;
* ``sobol512sub``: the 16-candidate subset (every 32nd) of the b = 512 Sobol batch of seed 2.

The GP hyperparameters are the device fit's (an input of the truth, like X and Y); the test
(tests/test_gpu_hp_truth.py) rebuilds the device state from them, so a later change of the
fit's rounding does not move the adjudicated state.  Writes JSON to argv[1].
usage: python tools/hp_state_dump.py out.json"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

import bench
from everest_amd import ops
from everest_amd.acquisition import QLogNEHVI


def near_candidates(X: np.ndarray, base_rows: np.ndarray, seed: int = 11) -> np.ndarray:
    rng = np.random.default_rng(seed)
    nonbase = np.setdiff1d(np.arange(X.shape[0]), base_rows)
    rows = np.concatenate([rng.choice(np.sort(base_rows), 12, replace=False), rng.choice(nonbase, 4, replace=False)])
    dist = 10.0 ** (-2.0 - 4.0 * np.arange(16) / 15.0)
    out = []
    for r, h in zip(rows, dist):
        u = rng.normal(size=X.shape[1])
        u /= np.linalg.norm(u)
        x = X[r] + h * u
        if (x < 0).any() or (x > 1).any():
            x = X[r] - h * u
        out.append(x)
    return np.stack(out), rows, dist


def device_eval(acqf, qa, Xc, L22_of):
    a, g = acqf.forward_backward(Xc)
    la, lg = qa.forward_backward(Xc)
    return dict(qnehvi=a.cpu().tolist(), qnehvi_grad=g.cpu().tolist(), qlog=la.cpu().tolist(),
                qlog_grad=lg.cpu().tolist(), L22=L22_of(Xc))


def main():
    dev = torch.device("cuda", 0)
    n, d, m, S = 512, 6, 5, 256
    X, Y, gp, hypers, acqf, _, _ = bench.build_state(n, d, m, S, dev)
    qa = QLogNEHVI(acqf.gp, X, X, -1.1 * np.ones(m), -np.ones(m), np.zeros(m), S=S, sampler_seed=1234,
                   prune_baseline=True, prune_seed=4321)
    base_rows = np.sort(np.asarray(acqf.base_rows))

    def L22_of(Xc):
        b = Xc.shape[0]
        if ops.qnehvi_small_applies(acqf.state, b, d):
            R, P = ops.qnehvi_small_forward(acqf.state, acqf.model, gp.cross(Xc), b)
            L22 = ops.qnehvi_small_samples(acqf.state, R, P, b)[1]
        else:
            R, P = ops.qnehvi_project(acqf.state, acqf.M, gp.cross(Xc), b)
            L22 = ops.qnehvi_samples_norms(acqf.state, R, P, b)[1]
        return L22.cpu().tolist()

    sets = {}
    sets["sobol20"] = bench.candidates(20, d, seed=2, device="cpu").numpy()
    near, rows, dist = near_candidates(X, base_rows)
    sets["near16"] = near
    sets["sobol512sub"] = bench.candidates(512, d, seed=2, device="cpu").numpy()[0:512:32]
    out = dict(n=n, d=d, m=m, S=S, x_seed=0, prune_seed=4321, sampler_seed=1234, ref=-1.1,
               hypers=[dict(lengthscale=h.lengthscale.tolist(), noise=float(h.noise), constant=float(h.constant),
                            y_mean=float(h.y_mean), y_std=float(h.y_std)) for h in hypers],
               base_rows=base_rows.tolist(), near_rows=rows.tolist(), near_dist=dist.tolist(),
               total_cells=int(acqf.stats.total_cells), sets={k: v.tolist() for k, v in sets.items()}, device={})
    # each set at its own batch size (b <= 32: the restart-batch kernels) and all 52 inside one
    # b = 512 batch (the b > 32 MFMA-engine path)
    big = bench.candidates(512, d, seed=5, device="cpu").numpy()
    allc = np.concatenate([sets["sobol20"], sets["near16"], sets["sobol512sub"]])
    big[:allc.shape[0]] = allc
    for k, v in sets.items():
        out["device"][k] = device_eval(acqf, qa, torch.tensor(v, device=dev), L22_of)
    e = device_eval(acqf, qa, torch.tensor(big, device=dev), L22_of)
    out["device"]["b512"] = {k: (v[:allc.shape[0]] if k != "L22" else [r[:allc.shape[0]] for r in v])
                             for k, v in e.items()}
    with open(sys.argv[1], "w") as f:
        json.dump(out, f)
    print("wrote", sys.argv[1], "base", len(base_rows), "cells", out["total_cells"])


if __name__ == "__main__":
    main()
