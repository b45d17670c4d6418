"""Projection GEMM timing (forward with norm epilogue, backward with generated gR) at the
bench state, several batch sizes (HIP events)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from everest_amd import ops


def t_ms(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps, 4)


dev = torch.device("cuda", 0)
X, Y, gp, hypers, acqf, _, _ = bench.build_state(512, 6, 5, 256, dev)
st = acqf.state
out = {}
for b in (20, 128, 512, 1024):
    Xc = bench.candidates(b, 6, seed=2, device=dev)
    Kx = gp.cross(Xc)
    R, P = ops.qnehvi_project(st, acqf.M, Kx, b)
    G, L22, flags = ops.qnehvi_samples_norms(st, R, P, b)
    acq, dG = ops.hvi_forward_backward(st, G, b, flags)
    out[f"b{b}"] = {"fwd": t_ms(lambda: ops.qnehvi_project(st, acqf.M, Kx, b)),
                    "bwd": t_ms(lambda: ops.qnehvi_project_backward(st, acqf.M, R, L22, dG, b)),
                    "kgrad": t_ms(lambda: ops.kernel_cross_grad(gp.Xn, Xc, gp.ls, Kx, gp.kind, shift2=gp.lo,
                                                                scale2=gp.inv_range)),
                    "kmat": t_ms(lambda: gp.cross(Xc))}
print(json.dumps(out))
