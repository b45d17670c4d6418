"""Host wall time of one warm QnehviStrategy.ask() split over its Python-level phases
(config-4 shape).  Wraps the ask's functions with timers (no device synchronisation added,
so a phase that waits on the device includes that wait) and prints, per phase, the
inclusive time of the last ask.  The gaps between the phases are the glue around them."""
import functools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import bench
from everest_amd import acquisition, ops, optim, strategies
from everest_amd.data_models import domain as dmod

T = {}


def timed(owner, name, label=None):
    f = getattr(owner, name)
    label = label or f"{getattr(owner, '__name__', owner)}.{name}"

    @functools.wraps(f)
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            T[label] = T.get(label, 0.0) + time.perf_counter() - t0
    setattr(owner, name, w)


for owner, name in [(strategies.QnehviStrategy, "_get_acqfs"), (acquisition.QNEHVI, "__init__"),
                    (strategies.BotorchStrategy, "_postprocess_candidates"),
                    (strategies.PredictiveStrategy, "predict"), (strategies.BotorchStrategy, "_predict"),
                    (strategies.BotorchStrategy, "get_categorical_combinations"),
                    (optim, "draw_sobol_samples"), (optim, "initialize_q_batch_nonneg"), (optim, "host_values"),
                    (acquisition.QNEHVI, "forward"), (acquisition.QNEHVI, "plan"),
                    (ops.QnehviPlan, "minimize"), (ops.QnehviPlan, "__init__"),
                    (dmod.Domain, "validate_candidates")]:
    try:
        timed(owner, name)
    except AttributeError:
        pass
# optimize_acqf is looked up through the strategies module
timed(strategies, "optimize_acqf", "optimize_acqf")
timed(strategies.PredictiveStrategy, "ask", "PredictiveStrategy.ask (total)")

s, _ = bench.make_ask_strategy(512, 256, 1024, 20, 1)
for _ in range(3):
    T.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.ask(1)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
out = {"ask_ms": round(wall * 1e3, 3),
       "phases_ms": {k: round(v * 1e3, 3) for k, v in sorted(T.items(), key=lambda kv: -kv[1])},
       "construction": s.last_acqf.timings}
print(json.dumps(out, indent=1, default=float))
