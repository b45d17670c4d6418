"""Phase breakdown of the sparse HVI scan (needs the EVR_KD_PROF=1 build via EVR_LIB_PATH)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from everest_amd import ops
dev = torch.device("cuda", 0)
X, Y, gp, hypers, acqf, _, _ = bench.build_state(512, 6, 5, 256, dev)
import numpy as np
out = {}
# the restart batch at its optimised candidates (the ask's hot loop sees these)
p = acqf.plan(20, True)
xo, _, _ = p.minimize(np.random.default_rng(0).uniform(size=20 * 6), np.zeros(120), np.ones(120), 2000)
Xopt = torch.tensor(np.asarray(xo).reshape(20, 6), device=dev)
for b, Xc in ((20, None), ("20opt", Xopt), (512, None)):
    if Xc is None:
        Xc = bench.candidates(b, 6, seed=2, device=dev)
    b = Xc.shape[0] if isinstance(b, str) else b
    tag = "20opt" if Xc is Xopt else str(b)
    R, P = ops.qnehvi_project(acqf.state, acqf.M, gp.cross(Xc), b)
    G, L22, flags = ops.qnehvi_samples_norms(acqf.state, R, P, b)
    ctr = torch.zeros(16, dtype=torch.int64, device=dev)
    acqf.state.scan_counters = ctr.data_ptr()
    ops.hvi_forward_backward(acqf.state, G, b, flags)
    torch.cuda.synchronize()
    acqf.state.scan_counters = None
    c = ctr.cpu().numpy().astype(float)
    tot = c[4:9].sum()
    out[f"b{tag}"] = {"phase_frac": {n: round(c[4 + i] / tot, 3) for i, n in enumerate(("stage", "groupA", "cellB", "termC", "scan"))},
                    "wave_cycles_total": tot, "wave_cycles_max": c[9], "waves_timed": c[10], "group_pairs": c[0], "terms": c[1]}
print(json.dumps(out))
