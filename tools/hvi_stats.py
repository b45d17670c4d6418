"""Diagnostics for the HVI scan at the bench state: how many (cell, candidate) pairs
contribute, and how many a given tile-skip rule lets through."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import bench
from everest_amd import ops


def main(b=512):
    dev = torch.device("cuda", 0)
    X, Y, gp, hypers, acqf, _, _ = bench.build_state(512, 6, 5, 256, dev)
    Xc = bench.candidates(b, 6, seed=2, device=dev)
    Kx = gp.cross(Xc)
    R = ops.gemm(acqf.M, Kx)
    G, L22, flags = ops.qnehvi_samples(acqf.state, R, b)       # S x m x b
    lo, hi = acqf.cells.explicit()
    off = acqf.cells.off.cpu().tolist()
    S, m = acqf.S, acqf.m
    tot = contrib = prefix0 = tile44 = 0
    tile_cells = {16: 0, 64: 0, 256: 0}
    bbox_pass = {16: 0, 64: 0, 256: 0}
    sortc_tile = 0
    for s in range(S):
        l = lo[off[s]:off[s + 1]]               # C x m  (sorted by l0)
        y = G[s].T                               # b x m
        C = l.shape[0]
        ok = (y[None, :, :] > l[:, None, :])     # C x b x m
        tot += C * b
        contrib += int(ok.all(-1).sum())
        prefix0 += int(ok[..., 0].sum())
        # current rule: thread tile = 4 consecutive cells x 4 candidates (stride 16)
        Cp = (C + 3) // 4 * 4
        lpad = torch.full((Cp, m), float("inf"), dtype=l.dtype, device=dev)
        lpad[:C] = l
        lmin = lpad.view(Cp // 4, 4, m).amin(1)                      # T x m
        bp = (b + 63) // 64 * 64
        ypad = torch.full((bp, m), float("-inf"), dtype=y.dtype, device=dev)
        ypad[:b] = y
        ymax = ypad.view(bp // 64, 4, 16, m).amax(1).reshape(bp // 4, m)   # thread cand groups
        live = (ymax[None, :, :] > lmin[:, None, :]).all(-1)            # T x (b/4)
        tile44 += int(live.sum()) * 16
        # sorted candidates (by y0) in groups of 4 consecutive
        ys = ypad[torch.argsort(ypad[:, 0])]
        ymax2 = ys.view(bp // 4, 4, m).amax(1)
        live2 = (ymax2[None, :, :] > lmin[:, None, :]).all(-1)
        sortc_tile += int(live2.sum()) * 16
        # group bounding boxes (per candidate): a group of g cells passes for candidate c if
        # min-l over the group < y in every objective
        for g in tile_cells:
            Cg = (C + g - 1) // g * g
            lg = torch.full((Cg, m), float("inf"), dtype=l.dtype, device=dev)
            lg[:C] = l
            gm = lg.view(Cg // g, g, m).amin(1)
            bbox_pass[g] += int((y[None] > gm[:, None]).all(-1).sum()) * g
    out = {"pairs": tot, "contrib_frac": contrib / tot, "prefix0_frac": prefix0 / tot,
           "tile44_frac": tile44 / tot, "tile44_sortedcand_frac": sortc_tile / tot,
           "group_bbox_frac_per_candidate": {g: v / tot for g, v in bbox_pass.items()},
           "cells_total": acqf.stats.total_cells, "b": b}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
