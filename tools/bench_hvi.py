"""HVI scan timing at the bench state: sparse kd scan vs tiled scan, forward+backward,
several candidate batch sizes (HIP events on torch's current stream)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import bench
from everest_amd import ops


def main():
    dev = torch.device("cuda", 0)
    X, Y, gp, hypers, acqf, _, _ = bench.build_state(512, 6, 5, 256, dev)
    dense_state = ops.make_state(acqf.n, acqf.nb, acqf.S, acqf.m, gp.const, gp.ym, gp.ys, gp.kxx, acqf.zq,
                                 acqf.obj_a, acqf.obj_b, ops.Cells(acqf.cells.off, acqf.cells.counts, acqf.m,
                                                                   keys=acqf.cells.keys, pts=acqf.cells.pts,
                                                                   rank0=acqf.cells.rank0, stride=acqf.cells.stride))
    out = {"box_path": acqf.box_path}
    sizes = [int(v) for v in os.environ.get("HVI_SIZES", "20,64,128,512,1024").split(",")]
    variants = (("kd", acqf.state),) if os.environ.get("HVI_ONLY_KD") else (("kd", acqf.state), ("tiled", dense_state))
    for b in sizes:
        Xc = bench.candidates(b, 6, seed=2, device=dev)
        R = ops.gemm(acqf.M, gp.cross(Xc))
        G, L22, flags = ops.qnehvi_samples(acqf.state, R, b)
        row = {}
        for name, st in variants:
            for _ in range(3):
                ops.hvi_forward_backward(st, G, b, flags)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            e0.record()
            for _ in range(reps):
                a, dG = ops.hvi_forward_backward(st, G, b, flags)
            e1.record()
            torch.cuda.synchronize()
            row[name + "_ms"] = round(e0.elapsed_time(e1) / reps, 4)
            row[name + "_acq"] = a
        if "tiled_acq" in row:
            row["max_rel_diff"] = float(((row["kd_acq"] - row["tiled_acq"]).abs() / row["tiled_acq"].abs().clamp_min(1e-12)).max())
            del row["tiled_acq"]
        row["acq_sum"] = float(row.pop("kd_acq").sum())
        out[f"b{b}"] = row
    print(json.dumps(out))


if __name__ == "__main__":
    main()
