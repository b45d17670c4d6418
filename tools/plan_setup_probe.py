"""Host cost of a restart plan's first use at the bench shape: plan creation, the first
host evaluation (graph capture + instantiate or update of a recycled executable inside), and
a warm evaluation (ms, median of 5 fresh plans on the last ask's acquisition; then the same
on 5 fresh acquisitions, as consecutive asks see it).  One JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

import bench
from everest_amd import ops

s, _ = bench.make_ask_strategy(512, 256, 1024, 20, 1)
s.ask(1)
s.ask(1)
acqf = s.last_acqf
x = np.random.default_rng(0).uniform(size=(20, 6))
rows = []
for _ in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    p = ops.QnehviPlan(acqf.state, acqf.model, 20, True, acqf.dev, graph=True)
    t1 = time.perf_counter()
    p.run_host(x)
    t2 = time.perf_counter()
    p.run_host(x)
    t3 = time.perf_counter()
    rows.append((t1 - t0, t2 - t1, t3 - t2))
    del p
med = np.median(np.array(rows), axis=0) * 1e3
out = {"plan_create_ms": round(med[0], 3), "first_eval_ms": round(med[1], 3), "warm_eval_ms": round(med[2], 3)}
rows = []
for _ in range(5):
    acqf = s._get_acqfs(1)[0]       # a new acquisition, the previous one (and its plans) dropped
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    p = acqf.plan(20, True)
    t1 = time.perf_counter()
    p.run_host(x)
    t2 = time.perf_counter()
    p.run_host(x)
    t3 = time.perf_counter()
    rows.append((t1 - t0, t2 - t1, t3 - t2))
med = np.median(np.array(rows), axis=0) * 1e3
out.update({"fresh_acqf_plan_create_ms": round(med[0], 3), "fresh_acqf_first_eval_ms": round(med[1], 3),
            "fresh_acqf_warm_eval_ms": round(med[2], 3)})
print(json.dumps(out))
