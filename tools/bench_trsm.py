"""Forward substitution at the qNEHVI operator's shape (G = L_base^-1 E: 5 outputs, the pruned
baseline n_b ~ 277 rows, 512 right-hand-side columns; trsm16_kernel) and at larger n_b, against
torch's solve_triangular on the CPU for the result.  HIP events over repeated calls."""
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
for (B, n, nrhs) in ((5, 277, 512), (5, 512, 512), (1, 2048, 256)):
    g = torch.Generator().manual_seed(n)
    A = torch.randn(B, n, n, generator=g, dtype=torch.float64)
    L = torch.linalg.cholesky(A @ A.transpose(1, 2) + n * torch.eye(n, dtype=torch.float64))
    E = torch.randn(B, n, nrhs, generator=g, dtype=torch.float64)
    Ld = L.cuda()
    E0 = E.cuda()
    X = E0.clone()
    t = ev(lambda: (X.copy_(E0), ops.trsm(Ld, X)))
    tc = ev(lambda: X.copy_(E0))
    ops.trsm(Ld, X.copy_(E0))
    ref = torch.linalg.solve_triangular(L, E, upper=False)
    err = float(((X.cpu() - ref).abs() / ref.abs().max()).max())
    out[f"B{B}_n{n}_rhs{nrhs}"] = {"ms": round(t - tc, 4), "rel_err": err}
print(json.dumps(out))
