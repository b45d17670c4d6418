"""Build the bench state, then run exactly N instrumented-free bench steps and nothing
else (for rocprofv3 --pmc passes: the last N dispatches of each kernel are the steps)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import bench

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10
b = int(sys.argv[2]) if len(sys.argv) > 2 else 512
dev = torch.device("cuda", 0)
X, Y, gp, hypers, acqf, _, _ = bench.build_state(512, 6, 5, 256, dev)
Xc = bench.candidates(b, 6, seed=2, device=dev)
chain = bench.op_chain(acqf, Xc)
for _ in range(2 + N):
    for f in chain.values():
        f()
torch.cuda.synchronize()
print("done")
