"""Print the config-5 SoboStrategy fit (hyperparameters + best_f) — run twice to check
run-to-run repeatability."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np

import everest_amd.data_models as dm
from everest_amd import strategies
from tests.helpers import mixed_domain, mixed_f

dom = mixed_domain()
X = strategies.map(dm.RandomStrategy(domain=dom, seed=13)).ask(2048)
exps = X.copy()
exps["y"] = mixed_f(X)
exps["valid_y"] = 1
h = hashlib.sha1(np.ascontiguousarray(exps.drop(columns=[c for c in exps.columns if c.startswith("c")]).values)
                 .tobytes()).hexdigest()[:12]
spec = dm.SingleTaskGPSurrogate(inputs=dom.inputs, outputs=dom.outputs, kernel=dm.MaternKernel(nu=2.5))
s = strategies.map(dm.SoboStrategy(domain=dom, acquisition_function=dm.qEI(), seed=1,
                                   surrogate_specs=dm.BotorchSurrogates(surrogates=[spec]),
                                   categorical_method="FREE", num_raw_samples=256, num_restarts=4))
s.tell(exps)
st = s.surrogates.surrogates[0].state
print(json.dumps({"data": h, "cats": str(X["c0"].values[:8]), "noise": st["noise"], "constant": st["constant"],
                  "ls": np.asarray(st["lengthscale"]).round(8).tolist(), "best_f": s._get_acqfs(1)[0].best_f}))
