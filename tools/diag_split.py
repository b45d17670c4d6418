"""Diagnostic: the b = 512 projection path (qnehvi_proj.hip, the gemm_core engine) against the
b = 20 restart-batch kernels (qnehvi_small.hip) at the config-3 bench state, and both against
an extended-precision (x87 long double) restatement of R = M K_x and L22 for the candidates
where the acquisition values differ most.  Prints one JSON object.

usage: python tools/diag_split.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from everest_amd import ops

    dev = torch.device("cuda", 0)
    X, Y, gp, hypers, acqf, _, _ = bench.build_state(512, 6, 5, 256, dev)
    st, M = acqf.state, acqf.M
    Xc = bench.candidates(512, 6, seed=3, device=dev)
    a_full, _ = acqf.forward_backward(Xc)
    a_p = torch.cat([acqf.forward_backward(Xc[i:i + 20])[0] for i in range(0, 500, 20)])
    diff = (a_full[:500] - a_p).abs().cpu().numpy()
    worst = np.argsort(-diff)[:6]
    Kx = acqf._cross(Xc)
    RA, PA = ops.qnehvi_project(st, M, Kx, 512)
    GA, LA, fA = ops.qnehvi_samples_norms(st, RA, PA, 512)
    n = acqf.Rr - acqf.S - 1
    Mh = M.cpu().numpy().astype(np.longdouble)
    out = {"n": n, "Rr": acqf.Rr, "max_abs_diff": float(diff.max()), "cands": []}
    for c in worst:
        c = int(c)
        c0 = (c // 20) * 20
        Kc = Kx[:, :, c0:c0 + 20].contiguous()
        RB, PB = ops.qnehvi_small_forward(st, acqf.model, Kc, 20)
        GB, LB, fB = ops.qnehvi_small_samples(st, RB, PB, 20)
        row = {"c": c, "a_full": float(a_full[c]), "a_p": float(a_p[c]), "diff": float(diff[c]), "outputs": []}
        kx = Kx[:, :, c].cpu().numpy().astype(np.longdouble)
        for j in range(M.shape[0]):
            Re = Mh[j] @ kx[j]                                   # Rr, extended precision
            ss_e = float(np.sum(Re[:n] * Re[:n]))
            rA = RA[j, :, c].cpu().numpy()
            rB = RB[j, :, c - c0].cpu().numpy()
            errA = float(np.max(np.abs(rA - Re.astype(np.float64))))
            errB = float(np.max(np.abs(rB - Re.astype(np.float64))))
            kxx, ys = float(acqf.gp.kxx[j]), float(acqf.gp.ys[j])
            br = np.longdouble(ys) ** 2 * (np.longdouble(kxx) - np.sum(Re[:n] * Re[:n]))
            row["outputs"].append({"j": j, "ss_exact": ss_e, "br_exact": float(br),
                                   "L22_exact": float(np.sqrt(br)) if br > 0 else None,
                                   "L22_A": float(LA[j, c]), "L22_B": float(LB[j, c - c0]),
                                   "R_err_A": errA, "R_err_B": errB})
        out["cands"].append(row)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
