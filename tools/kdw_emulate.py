"""Host (numpy) emulation of hvi_kdw's filter and terms on a device kd state, against the
three-launch chain's per-sample values: locates the terms / thresholds where the kernel and
the algorithm part ways (diagnosis of a NaN restart scan)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from everest_amd import ops, _native
from tests.test_gpu_hvi_kd import _pair


def fb(m):
    return 16 if m <= 4 else (12 if m == 5 else 64 // m)


def main(n=40, d=3, m=2, S=16, b=1):
    lib = _native.load()
    kd, dense, lo, hi, d = _pair(n, d, m, S, seed=n + m)
    Xc = torch.tensor(lo + (hi - lo) * np.random.default_rng(b).uniform(size=(b, d)), device="cuda")
    st = kd.state
    R, P = ops.qnehvi_small_forward(st, kd.model, kd.gp.cross(Xc), b)
    G, L22, flags = ops.qnehvi_small_samples(st, R, P, b)
    _native.check(lib.evr_hvi_set_restart_variant(1), "v")
    sv1, dg1 = ops.hvi_restart_fb(st, G, b)
    _native.check(lib.evr_hvi_set_restart_variant(3), "v")
    sv3, dg3 = ops.hvi_restart_fb(st, G, b)
    torch.cuda.synchronize()
    K = kd.cells.kd
    goff = K.goff.cpu().numpy().astype(np.int64)
    gkeys = K.keys.cpu().numpy().view(np.uint64)
    grk = K.rank.cpu().numpy().view(np.uint16)
    gbox = K.box.cpu().numpy().view(np.uint16)
    sv = K.sorted_lo.cpu().numpy()
    pts = kd.cells.pts.cpu().numpy()
    stride = kd.cells.stride
    Gh = G.cpu().numpy()
    print("stride", stride, "max_groups", K.max_groups, "groups", goff[-1], "pts finite", bool(np.isfinite(pts).all()),
          "sv finite", bool(np.isfinite(sv).all()), flush=True)
    F = fb(m)
    mask = (1 << F) - 1
    bad = 0
    for s in range(S):
        for c in range(b):
            y = Gh[s, :, c]
            t = np.ones(8, dtype=np.int64)
            tp = np.ones(8, dtype=np.int64)
            for j in range(m):
                t[j] = np.searchsorted(sv[s, j], y[j], side="right")
                # the kernel's two probes
                B1 = (stride + 63) // 64
                i1 = np.minimum((np.arange(64) + 1) * B1, stride) - 1
                base = min(int((sv[s, j][i1] <= y[j]).sum()) * B1, stride)
                i2 = base + np.arange(64)
                ok = (np.arange(64) < B1) & (i2 < stride)
                v2 = np.where(ok, sv[s, j][np.minimum(i2, stride - 1)], np.inf)
                tp[j] = base + int((ok & (v2 <= y[j])).sum())
            if not np.array_equal(t, tp):
                print("threshold mismatch s", s, "c", c, t[:m], tp[:m], flush=True)
            g0, g1 = goff[s], goff[s + 1]
            acc = 0.0
            nterms = 0
            for g in range(g1 - g0):
                gm = gbox[(g0 + g) * 8:(g0 + g) * 8 + 8].astype(np.int64)
                if not (gm < tp).all():
                    continue
                rk = grk[(g0 + g) * m * 16:(g0 + g + 1) * m * 16].reshape(m, 16).astype(np.int64)
                cm = (rk < tp[:m, None]).all(0)
                for c16 in np.nonzero(cm)[0]:
                    key = int(gkeys[(g0 + g) * 16 + c16])
                    Pj = [(key >> (F * (m - 1 - j))) & mask for j in range(m)]
                    lj, uj = np.empty(m), np.empty(m)
                    for j in range(m):
                        bl = -np.inf
                        for k in range(j):
                            bl = max(bl, pts[s, Pj[k], j])
                        lj[j] = -pts[s, Pj[j], j]
                        uj[j] = -bl
                    ln = np.maximum(np.minimum(y, uj) - lj, 0.0)
                    v = float(np.prod(ln))
                    nterms += 1
                    if not np.isfinite(v) and bad < 10:
                        bad += 1
                        print("NaN term s", s, "c", c, "g", g, "cell", c16, "P", Pj, "l", lj, "u", uj, "y", y,
                              "ranks", rk[:, c16], "t", tp[:m], flush=True)
                    acc += v
            print("s", s, "c", c, "terms", nterms, "emul", acc, "kd3", float(sv1[s, c]), "kdw", float(sv3[s, c]),
                  flush=True)


if __name__ == "__main__":
    main()
