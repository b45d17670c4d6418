"""f64 GEMM throughput: everest_amd MFMA GEMM vs torch.matmul (rocBLAS) at the projection
shape and at a large square shape."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from everest_amd import ops


def t_ms(fn, reps=10):
    for _ in range(2):
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
for (B, M, K, N) in ((5, 1046, 512, 512), (5, 1046, 512, 20), (1, 4096, 4096, 4096), (1, 8192, 8192, 8192)):
    A = torch.randn(B, M, K, dtype=torch.float64, device="cuda")
    Bm = torch.randn(B, K, N, dtype=torch.float64, device="cuda")
    fl = 2.0 * B * M * K * N
    t1 = t_ms(lambda: ops.gemm(A, Bm))
    t2 = t_ms(lambda: torch.matmul(A, Bm))
    out[f"{B}x{M}x{K}x{N}"] = {"evr_ms": round(t1, 4), "evr_TF": round(fl / t1 / 1e9, 2), "torch_ms": round(t2, 4),
                               "torch_TF": round(fl / t2 / 1e9, 2)}
print(json.dumps(out))
