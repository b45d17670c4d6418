"""Batched Cholesky / Cholesky+inverse timing (HIP events, device-resident input), fused
look-ahead (la, default) vs fused right-looking (rl) vs v1, with TF/s against the f64 MFMA peak.  One JSON line.
Flops: n^3/3 per factorisation, + n^3/3 for the triangular inverse."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from everest_amd import ops

PEAK = 78.6e12


def run(n, B, inverse, reps):
    g = torch.Generator().manual_seed(n)
    A = torch.randn(B, n, n + 7, generator=g, dtype=torch.float64)
    A = (A @ A.transpose(1, 2) / n + 1e-2 * torch.eye(n, dtype=torch.float64)).cuda()
    f = (lambda: ops.cholesky_inverse(A)) if inverse else (lambda: ops.cholesky(A))
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    flops = B * n ** 3 / 3 * (2 if inverse else 1)
    return {"ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 3), "frac": round(flops / ms / 1e-3 / PEAK, 4)}


def main():
    out = {}
    for ver in ("la", "rl", "v1"):
        os.environ["EVR_CHOL"] = ver
        for n, B, inv in ((512, 5, False), (512, 5, True), (1024, 5, False), (2048, 1, False), (2048, 1, True),
                          (4096, 1, False)):
            out[f"{ver}/n{n}b{B}{'_inv' if inv else ''}"] = run(n, B, inv, 20 if n <= 1024 else 5)
    print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 1:      # one configuration: ver n B inv (for rocprofv3 runs)
        ver, n, B, inv = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4] == "1"
        os.environ["EVR_CHOL"] = ver
        print(json.dumps(run(n, B, inv, 20)))
    else:
        main()
