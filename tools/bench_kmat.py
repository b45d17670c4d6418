"""Kernel-matrix assembly bandwidth: the eval-chain cross-covariance (config 3: B=5 outputs,
512 train rows x b candidates, d=6, RBF), the GP-fit train matrix, and config 5 (2048 x 2048,
d=32, Matern-2.5), each against a plain device fill of the same output (the write-bandwidth
ceiling).  Output preallocated; HIP-graph replay between HIP events."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from everest_amd import ops
from everest_amd.ops import call, _stream, _p


def ev(fn, reps=20, per_graph=10):
    """ms per call: per_graph calls captured into one HIP graph, the graph replayed reps times
    between HIP events (no host enqueue in the timed region: a ctypes call per launch is
    ~7 us of host time, a floor above the short kernels)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * per_graph)


torch.manual_seed(0)
out = {"lib": os.environ.get("EVR_LIB_PATH", "everest_amd/_lib"), "timing": "hip-graph replay"}
cases = (("cfg3_cross_b512", 5, 512, 512, 6, 0), ("cfg3_cross_b20", 5, 512, 20, 6, 0),
         ("fit_train_n512", 1, 512, 512, 6, 0), ("cfg2_cross", 1, 256, 1024, 6, 0),
         ("cfg5_n2048_d32", 1, 2048, 2048, 32, 3), ("cfg5_train_sym", 1, 2048, 2048, 32, 3),
         ("n2048_d6", 1, 2048, 2048, 6, 0),
         ("cfg3_cross_b4096", 5, 512, 4096, 6, 0))
only = os.environ.get("KMAT_CASES")
for (name, B, n1, n2, d, kind) in cases:
    if only and name not in only.split(","):
        continue
    X1 = torch.rand(n1, d, dtype=torch.float64, device="cuda")
    sym = name.endswith("_sym")   # the fit's train matrix K(X, X): one tensor, no normalisation (kmat_mfma_sym)
    X2 = X1 if sym else torch.rand(n2, d, dtype=torch.float64, device="cuda")
    sh = None if sym else torch.zeros(d, dtype=torch.float64, device="cuda")
    sc = None if sym else torch.ones(d, dtype=torch.float64, device="cuda")
    ls = torch.rand(B, d, dtype=torch.float64, device="cuda") + 0.3
    K = torch.empty(B, n1, n2, dtype=torch.float64, device="cuda")
    Kref = ops.kernel_matrix(X1, X2, ls, kind, shift2=sh, scale2=sc)
    f = lambda: call("evr_kernel_matrix", _stream(), kind, B, n1, n2, d, X1.data_ptr(), 0, 0, X2.data_ptr(),  # noqa: E731
                     _p(sh), _p(sc), ls.data_ptr(), 0, 0, K.data_ptr())
    t = ev(f)
    # exactness vs a torch fp64 restatement (explicit differences)
    u1 = X1[None] / ls[:, None, :]
    u2 = X2[None] / ls[:, None, :]
    d2 = ((u1[:, :, None, :] - u2[:, None, :, :]) ** 2).sum(-1) if n1 * n2 * B <= 5 * 512 * 1024 else None
    err = rel = None
    if d2 is not None:
        if kind == 0:
            Kt = torch.exp(-0.5 * d2)
        else:
            r = torch.sqrt(d2.clamp_min(1e-30)); s5 = 5 ** 0.5 * r
            Kt = (1 + s5 + 5.0 / 3.0 * d2) * torch.exp(-s5)
        err = float((K - Kt).abs().max())
        rel = float(((K - Kt).abs() / Kt.abs().clamp_min(1e-300)).max())
    same = bool(torch.equal(K, Kref))
    tf = ev(lambda: K.fill_(1.0))
    byt = 8.0 * B * (n1 * n2 + n1 * d + n2 * d)
    out[name] = {"kmat_us": round(t * 1e3, 2), "kmat_GBs": round(byt / t / 1e6, 1), "fill_us": round(tf * 1e3, 2),
                 "fill_GBs": round(8.0 * B * n1 * n2 / tf / 1e6, 1), "max_abs_err": err,
                 "max_rel_err": rel, "repeat_equal": same}
print(json.dumps(out))
