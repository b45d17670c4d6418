"""Diagnosis of a qLogNEHVI-vs-oracle difference at the BASELINE config-3 state (the
tests/test_gpu_baseline_sizes.py fixtures): for the b = 20 Sobol candidates (seed 2) the
device and oracle qLogNEHVI, the device and oracle qNEHVI (hard max), and the device L22 of
the new point per output, for the candidates whose log values differ most.  One JSON line
per candidate.  usage: python tools/qlog_diag.py"""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

import bench
from everest_amd import ops
from everest_amd.acquisition import QLogNEHVI
from oracle import gp as ogp
from oracle import qnehvi as oq


def main():
    dev = torch.device("cuda", 0)
    n, d, m, S = 512, 6, 5, 256
    X, Y, gp, hypers, acqf, _, _ = bench.build_state(n, d, m, S, dev)
    Xn = torch.tensor(X)
    states = []
    for j, h in enumerate(hypers):
        y = torch.tensor(Y[:, j])
        states.append(ogp.GPState(X=Xn, y=(y - h.y_mean) / h.y_std, lengthscale=torch.tensor(h.lengthscale),
                                  noise=h.noise, constant=h.constant, y_mean=h.y_mean, y_std=h.y_std))
    objective = oq.Objective(-torch.ones(m, dtype=torch.float64), torch.zeros(m, dtype=torch.float64))
    ref = torch.full((m,), -1.1, dtype=torch.float64)
    nb = acqf.nb
    idx = torch.as_tensor(np.sort(acqf.base_rows))
    zb = oq.base_samples(S, nb, m, 1234)
    zn = oq.base_samples(S, nb + 1, m, 1234)[:, nb:nb + 1]
    orc = oq.QNEHVI(states, Xn[idx], objective, ref, zb, zn)
    qa = QLogNEHVI(acqf.gp, X, X, -1.1 * np.ones(m), -np.ones(m), np.zeros(m), S=S, sampler_seed=1234,
                   prune_baseline=True, prune_seed=4321)
    olog = oq.QLogNEHVI(states, Xn[idx], objective, ref, zb, zn, cells=orc.cells)
    Xc = bench.candidates(20, d, seed=2, device=dev)
    a_log = qa.forward(Xc).cpu()
    a_hv = acqf.forward(Xc).cpu()
    xt = Xc.cpu().unsqueeze(1)
    with torch.no_grad():
        r_log = olog.forward(xt)
        r_hv = orc.forward(xt)
    R, P = ops.qnehvi_small_forward(qa.state, qa.model, qa.gp.cross(Xc), 20)
    L22 = ops.qnehvi_small_samples(qa.state, R, P, 20)[1].cpu()
    err = (a_log - r_log).abs()
    for c in torch.argsort(err, descending=True)[:5].tolist():
        print(json.dumps({"c": c, "log_dev": float(a_log[c]), "log_orc": float(r_log[c]),
                          "dlog": float(a_log[c] - r_log[c]), "hv_dev": float(a_hv[c]), "hv_orc": float(r_hv[c]),
                          "dlog_hv": float(math.log(max(float(a_hv[c]), 1e-300)) - math.log(max(float(r_hv[c]), 1e-300))),
                          "L22": [float(v) for v in L22[:, c]],
                          "L22_rel": [float(v) for v in (L22[:, c] ** 2 / (qa.gp.ys.cpu() ** 2 * qa.gp.kxx.cpu()))]}))


if __name__ == "__main__":
    main()
