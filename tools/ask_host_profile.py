"""Host-side profile of warm config-4 asks (cProfile over 5 asks after 2 warm-ups): where the
Python / pandas / ctypes time of an ask goes outside the device work — the set-up before the
restart loop, the candidate post-processing and validation after it.  Prints the top entries
by cumulative and by own time."""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench


def main():
    s, _ = bench.make_ask_strategy(512, 256, 1024, 20, 1, None, seed=1)
    for _ in range(2):
        s.ask(1)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        s.ask(1)
    torch.cuda.synchronize()
    pr.disable()
    for key in ("cumulative", "tottime"):
        buf = io.StringIO()
        pstats.Stats(pr, stream=buf).sort_stats(key).print_stats(45)
        print(buf.getvalue())


if __name__ == "__main__":
    main()
