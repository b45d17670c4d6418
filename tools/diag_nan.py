"""Diagnosis of a NaN restart evaluation (kd state of test_kd_scan_matches_tiled_scan[40-3-2-16-1]):
each piece of the b <= 32 chain against its reference, per restart-scan variant."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from everest_amd import ops, _native
from tests.test_gpu_hvi_kd import _pair

lib = _native.load()
for (n, d, m, S, b) in ((40, 3, 2, 16, 1), (120, 6, 5, 256, 20)):
    kd, dense, lo, hi, d = _pair(n, d, m, S, seed=n + m)
    Xc = torch.tensor(lo + (hi - lo) * np.random.default_rng(b).uniform(size=(b, d)), device="cuda")
    st, md = kd.state, kd.model
    Kx = kd.gp.cross(Xc)
    R, P = ops.qnehvi_small_forward(st, md, Kx, b)
    Rref = torch.matmul(kd.M, Kx)
    print("case", (n, d, m, S, b), "R finite", bool(torch.isfinite(R).all()), "R err",
          float((R.view_as(Rref) - Rref).abs().max()), flush=True)
    G, L22, flags = ops.qnehvi_small_samples(st, R, P, b)
    G2, L2b, fl2 = ops.qnehvi_samples_norms(st, *ops.qnehvi_project(st, kd.M, Kx, b), b)
    print("  G finite", bool(torch.isfinite(G).all()), "flags", int(flags.sum()), "G vs proj path",
          float((G - G2).abs().max()), "flags2", int(fl2.sum()), flush=True)
    a1, d1 = ops.hvi_forward_backward(st, G, b, flags)
    for v in (1, 2, 3):
        _native.check(lib.evr_hvi_set_restart_variant(v), "variant")
        sval, dG = ops.hvi_restart_fb(st, G, b)
        print("  variant", v, "sval finite", bool(torch.isfinite(sval).all()), "acq", ops.mean_over_samples(sval).cpu().numpy()[:4],
              "ref", a1.cpu().numpy()[:4], "dG err", float((dG - d1).abs().max()), flush=True)
        kd._plans = {}
        a, g = kd.forward_backward(Xc)
        print("    plan acq", a.cpu().numpy()[:4], "g finite", bool(torch.isfinite(g).all()), flush=True)
    _native.check(lib.evr_hvi_set_restart_variant(3), "variant")
