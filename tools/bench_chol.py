"""Cholesky (+ inverse) timing at the GP-fit shapes: batch 1 and 5, n = 512 / 2048 (wall time per
call incl. the ladder's host sync; chol_inv_sep: EVR_TRIINV=col, the separate inverse)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from everest_amd import ops

dev = torch.device("cuda", 0)
out = {}
for B, n in ((1, 512), (5, 512), (1, 2048)):
    A = torch.randn(B, n, n, dtype=torch.float64, device=dev)
    A = A @ A.transpose(1, 2) + n * torch.eye(n, dtype=torch.float64, device=dev)
    for name, fn in (("chol", lambda: ops.cholesky(A)), ("chol_inv", lambda: ops.cholesky_inverse(A)),
                     ("chol_inv_sep", lambda: ops.cholesky_inverse(A))):
        if name == "chol_inv_sep":   # the separate triangular inverse (A/B)
            os.environ["EVR_TRIINV"] = "col"
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        out[f"{name}_B{B}_n{n}_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 3)
        os.environ.pop("EVR_TRIINV", None)
print(json.dumps(out))
