"""Device qNEHVI / qLogNEHVI at the tests/golden/hp_state.json state against the 60-digit truth
(tests/golden/hp_truth.json) for both forward operators (root = fused / split), per candidate
set and batch path.  One JSON line per (root, set, path, acquisition): max value error (relative
for qNEHVI where HVI > 1e-9, |d log| for qLog) and max row-relative gradient error, plus the
per-candidate errors.  usage: python tools/hp_eval.py [out.json]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

import bench
from everest_amd.acquisition import QLogNEHVI, QNEHVI
from everest_amd.gp import GPBatch, GPHyper

G = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def errs(a, ga, T, GT, log):
    a, ga, T, GT = (np.asarray(v, dtype=np.float64) for v in (a, ga, T, GT))
    if log:
        verr, big = np.abs(a - T), T > np.log(1e-9)
    else:
        verr = np.abs(a - T) / np.maximum(np.abs(T), 1e-300)
        verr[(a == 0) & (T == 0)] = 0.0
        big = T > 1e-9
    gerr = np.abs(ga - GT).max(1) / np.maximum(np.abs(GT).max(1), 1e-300)
    return verr, gerr, big


def main():
    st = json.load(open(os.path.join(G, "hp_state.json")))
    tr = json.load(open(os.path.join(G, "hp_truth.json")))["sets"]
    dev = torch.device("cuda", 0)
    n, d, m, S = st["n"], st["d"], st["m"], st["S"]
    X = np.random.default_rng(st["x_seed"]).uniform(size=(n, d))
    Y = bench.dtlz2(X, m)
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev)  # noqa: E731
    hypers = [GPHyper(np.asarray(h["lengthscale"]), h["noise"], h["constant"], h["y_mean"], h["y_std"])
              for h in st["hypers"]]
    gp = GPBatch(t(X), t(Y), hypers, 0, t(np.zeros(d)), t(np.ones(d)))
    kw = dict(S=S, sampler_seed=st["sampler_seed"], prune_baseline=True, prune_seed=st["prune_seed"])
    rows = []
    for root in ("fused", "split"):
        acqs = {"qnehvi": QNEHVI(gp, X, X, st["ref"] * np.ones(m), -np.ones(m), np.zeros(m), root=root, **kw),
                "qlog": QLogNEHVI(gp, X, X, st["ref"] * np.ones(m), -np.ones(m), np.zeros(m), root=root, **kw)}
        for which, xs in st["sets"].items():
            xs = np.asarray(xs)
            big = bench.candidates(512, d, seed=5, device="cpu").numpy()
            big[:len(xs)] = xs
            for path, Xc in (("own_b", xs), ("b512", big)):
                for key, acq in acqs.items():
                    a, g = acq.forward_backward(torch.tensor(Xc, device=dev))
                    a, g = a.cpu().numpy()[:len(xs)], g.cpu().numpy()[:len(xs)]
                    verr, gerr, bigm = errs(a, g, tr[which][key], tr[which][key + "_grad"], key == "qlog")
                    row = dict(root=root, set=which, path=path, acq=key,
                               max_value_err=float(verr[bigm].max()) if bigm.any() else 0.0,
                               max_grad_err=float(gerr[bigm].max()) if bigm.any() else 0.0,
                               value_err=[float(v) for v in verr], grad_err=[float(v) for v in gerr],
                               hvi_gt_1e9=[bool(v) for v in bigm])
                    rows.append(row)
                    print(json.dumps({k: v for k, v in row.items() if not isinstance(v, list)}), flush=True)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(rows, f)


if __name__ == "__main__":
    main()
