"""cProfile of QnehviStrategy.ask() at the bench shape (host-side time per function)."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import bench

s, _ = bench.make_ask_strategy(512, 256, 1024, 20, 1)
for _ in range(2):
    s.ask(1)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    s.ask(1)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(45)
st.sort_stats("tottime").print_stats(40)
st.print_callers("ops.py.*cholesky|_native.py.*call|method .cpu.|method .item.|method .tolist.")
