"""K warm QnehviStrategy.ask() calls at the bench shape (config 4) — the workload for a
rocprofv3 --kernel-trace capture of the ask's device timeline.  Prints the mean ask time."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import bench

K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
s, _ = bench.make_ask_strategy(512, 256, 1024, 20, 1)
for _ in range(2):
    s.ask(1)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    s.ask(1)
torch.cuda.synchronize()
print(f"ask_ms {(time.perf_counter() - t0) / K * 1e3:.3f} evals_last {s.last_ask_stats.opt_evals}")
