"""Build the bench state, then run exactly N instrumented-free bench steps and nothing
else (for rocprofv3 --pmc passes: the last N dispatches of each kernel are the steps).

usage: python tools/loop_step.py N b [ask]
With ``ask`` the state is bench.py's: the config-4 QnehviStrategy after one ask() (seed 1), and
the b candidates are that ask's optimised restart candidates — the batch bench.py's top-level
``roofline`` times (b must equal the restart count, 20)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import bench

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10
b = int(sys.argv[2]) if len(sys.argv) > 2 else 512
dev = torch.device("cuda", 0)
if len(sys.argv) > 3 and sys.argv[3] == "ask":
    s, _ = bench.make_ask_strategy(512, 256, 1024, b, 1, None, seed=1)
    s.ask(1)
    acqf = s.last_acqf
    Xc = torch.as_tensor(s.last_ask_stats.restart_X.reshape(b, -1), dtype=torch.float64, device=dev)
else:
    X, Y, gp, hypers, acqf, _, _ = bench.build_state(512, 6, 5, 256, dev)
    Xc = bench.candidates(b, 6, seed=2, device=dev)
chain = bench.op_chain(acqf, Xc)
for _ in range(2 + N):
    for f in chain.values():
        f()
torch.cuda.synchronize()
print("done")
