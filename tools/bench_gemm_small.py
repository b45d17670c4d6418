"""Small-GEMM latency at the blocked-Cholesky shapes (panel t x 64 x 64, trailing t x t x 64)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from everest_amd import ops

dev = torch.device("cuda", 0)
out = {}
for t in (448, 192, 64, 1984):
    P = torch.randn(1, t, 64, dtype=torch.float64, device=dev)
    D = torch.randn(1, 64, 64, dtype=torch.float64, device=dev)
    C = torch.randn(1, t, t, dtype=torch.float64, device=dev)
    for name, fn in (("panel", lambda: ops.gemm(P, D, transB=True)),
                     ("trail", lambda: ops.gemm(P, P, transB=True, alpha=-1.0, beta=1.0, out=C))):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(100):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[f"{name}_t{t}_us"] = round(e0.elapsed_time(e1) * 10, 2)
print(json.dumps(out))
