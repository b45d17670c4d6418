"""f64 batched GEMM time at the qNEHVI projection shapes through torch.matmul (rocBLAS):
forward R = M K_x with Rr = 769 rows (fused root: n + S + 1) vs 768 (mean row split off),
backward M^T gR, and the restart batch b = 20.  Probes the tile-count / CU balance of the
library kernel (13 vs 12 row tiles of 64)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


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
    return e0.elapsed_time(e1) / reps


out = {}
shapes = {"fwd769": (5, 769, 512, 512), "fwd768": (5, 768, 512, 512), "fwd832": (5, 832, 512, 512),
          "bwd769": (5, 512, 769, 512), "bwd768": (5, 512, 768, 512), "bwd512x8": (40, 64, 769, 512),
          "fwd769_b20": (5, 769, 512, 20), "fwd768_b20": (5, 768, 512, 20)}
for name, (B, M, K, N) in shapes.items():
    A = torch.randn(B, M, K, dtype=torch.float64, device="cuda")
    Bm = torch.randn(B, K, N, dtype=torch.float64, device="cuda")
    C = torch.empty(B, M, N, dtype=torch.float64, device="cuda")
    t = t_ms(lambda: torch.matmul(A, Bm, out=C))
    out[name] = {"ms": round(t, 4), "TF": round(2.0 * B * M * K * N / t / 1e9, 2)}
print(json.dumps(out))
