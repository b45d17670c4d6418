"""Synchronised split times of the QNEHVI construction inside ask() at the bench shape
(EVR_CONSTRUCTION_PROBES=1): median over 5 asks of each probe (ms).  One JSON line."""
import json
import os
import sys

os.environ["EVR_CONSTRUCTION_PROBES"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np

import bench

s, _ = bench.make_ask_strategy(512, 256, 1024, 20, 1)
rows = []
for i in range(7):
    s.ask(1)
    if i >= 2:
        rows.append(s.last_acqf.timings)
out = {k: round(float(np.median([r[k] for r in rows])) * 1e3, 3) for k in rows[0]}
print(json.dumps(out))
