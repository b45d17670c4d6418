"""GP posterior (mean + variance) at the metric's shape: the BASELINE config-3 model of
tests/golden/hp_state.json (n = 512, d = 6, m = 5) at 1024 Sobol test points — bench.py's
gp_posterior_ms.  HIP events over back-to-back calls (the op) and per kernel by
rocprofv3 --kernel-trace --stats around this script; checks the result against the 60-digit
truth's points (tests/golden/post_truth.json) on the way."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
from everest_amd.gp import GPBatch, GPHyper

G = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
st = json.load(open(os.path.join(G, "hp_state.json")))
tr = json.load(open(os.path.join(G, "post_truth.json")))["sets"]
dev = torch.device("cuda", 0)
t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev)  # noqa: E731
X = np.random.default_rng(st["x_seed"]).uniform(size=(st["n"], st["d"]))
Y = bench.dtlz2(X, st["m"])
hy = [GPHyper(np.asarray(h["lengthscale"]), h["noise"], h["constant"], h["y_mean"], h["y_std"]) for h in st["hypers"]]
gp = GPBatch(t(X), t(Y), hy, 0, t(np.zeros(st["d"])), t(np.ones(st["d"])))
ys = np.array([h["y_std"] for h in st["hypers"]])[:, None]
err_m = err_v = 0.0
for k, T in tr.items():
    m, v = gp.posterior(t(st["sets"][k]))
    err_m = max(err_m, float((np.abs(m.cpu().numpy() - np.asarray(T["mean"])) / ys).max()))
    err_v = max(err_v, float((np.abs(v.cpu().numpy() - np.asarray(T["var"])) / np.asarray(T["var"])).max()))
Xs = torch.quasirandom.SobolEngine(st["d"], scramble=True, seed=1).draw(1024, dtype=torch.float64).to(dev)
reps = int(os.environ.get("POST_REPS", "50"))
ms = bench._event_ms(lambda: gp.posterior(Xs), reps=reps)
# the same call through the C-ABI (ctypes: honours EVR_LIB_PATH, for A/B builds) and a digest of
# its result bytes (bitwise-neutral changes: equal digests)
from everest_amd import ops  # noqa: E402
import hashlib  # noqa: E402
call = lambda: ops.gp_posterior(gp.Xn, Xs, gp.lo, gp.inv_range, gp.ls, gp.M, gp.kind, gp.const, gp.ym,  # noqa: E731
                                gp.ys, gp.kxx)
ms_c = bench._event_ms(call, reps=reps)
m, v = call()
dig = hashlib.sha256(m.cpu().numpy().tobytes() + v.cpu().numpy().tobytes()).hexdigest()[:16]
print(json.dumps({"posterior_ms": round(ms, 4), "c_abi_ms": round(ms_c, 4), "digest": dig, "reps": reps,
                  "lib": os.environ.get("EVR_LIB_PATH", "_lib"), "truth_mean_err_ystd": err_m,
                  "truth_var_rel_err": err_v}))
