"""Kernel-matrix assembly bandwidth at config-5 shape (2048 x 2048 x d) vs a plain device
fill of the same output (the write-bandwidth ceiling)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from everest_amd import ops


def ev(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


out = {}
for (n, d, kind) in ((2048, 32, 3), (2048, 6, 0), (4096, 32, 3), (512, 6, 0)):
    X = torch.rand(n, d, dtype=torch.float64, device="cuda")
    ls = torch.full((1, d), 0.7, dtype=torch.float64, device="cuda")
    noise = torch.tensor([1e-3], dtype=torch.float64, device="cuda")
    K = torch.empty(n, n, dtype=torch.float64, device="cuda")
    t = ev(lambda: ops.kernel_matrix(X, X, ls, kind, diag_add=noise))
    tf = ev(lambda: K.fill_(1.0))
    byt = 8.0 * n * n
    out[f"n{n}_d{d}_k{kind}"] = {"kmat_ms": round(t, 4), "kmat_TBs": round(byt / t / 1e9, 3), "fill_ms": round(tf, 4),
                                 "fill_TBs": round(byt / tf / 1e9, 3)}
print(json.dumps(out))
