"""GP fit (tell) timing at the bench problem: 5 outputs, n=512, d=6 (device MLL + scipy)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import bench
from everest_amd.gp import fit_single
from everest_amd import ops

dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
X = rng.uniform(size=(512, 6))
Y = bench.dtlz2(X, 5)
Xn = torch.as_tensor(X, device=dev)
prior = (np.sqrt(2) + 0.5 * np.log(6), np.sqrt(3))
fit_single(Xn, Y[:, 0], 0, prior, (-4.0, 1.0))   # warm-up
torch.cuda.synchronize()
t0 = time.perf_counter()
hs = [fit_single(Xn, Y[:, j], 0, prior, (-4.0, 1.0)) for j in range(5)]
torch.cuda.synchronize()
t_fit = time.perf_counter() - t0
A = torch.randn(5, 512, 512, dtype=torch.float64, device=dev)
A = A @ A.transpose(1, 2) + 512 * torch.eye(512, dtype=torch.float64, device=dev)
for _ in range(3):
    ops.cholesky_inverse(A)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    ops.cholesky_inverse(A)
torch.cuda.synchronize()
t_chol = (time.perf_counter() - t0) / 20
print(json.dumps({"fit_5_outputs_s": round(t_fit, 3), "chol_inv_5x512_ms": round(t_chol * 1e3, 3),
                  "lengthscales_0": [round(float(v), 4) for v in hs[0].lengthscale]}))
