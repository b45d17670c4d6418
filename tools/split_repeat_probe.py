"""Intermittency probe for the config-3 batch-split check: in one process, builds the bench
state K times and per state evaluates the 512-candidate batch against 25 batches of 20 R times
(plans dropped every other repeat, so graph capture and replay both run); prints the max |diff|
per (state, repeat) and digests of a_full, so a rare race shows as an outlier.
usage: python tools/split_repeat_probe.py [K] [R]"""
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench

    K = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda", 0)
    Xc = bench.candidates(512, 6, seed=3, device=dev)
    rows = []
    for k in range(K):
        X, Y, gp, hypers, acqf, _, _ = bench.build_state(512, 6, 5, 256, dev)
        Mh = hashlib.sha256(acqf.M.cpu().numpy().tobytes()).hexdigest()[:10]
        for r in range(R):
            if r % 2 == 0:
                acqf._plans = {}
            a_full, g_full = acqf.forward_backward(Xc)
            a_p = torch.cat([acqf.forward_backward(Xc[i:i + 20])[0] for i in range(0, 500, 20)])
            d = (a_full[:500] - a_p).abs()
            rows.append({"state": k, "rep": r, "M": Mh, "max_diff": float(d.max()), "argmax": int(d.argmax()),
                         "a_full": hashlib.sha256(a_full.cpu().numpy().tobytes()).hexdigest()[:10],
                         "a_p": hashlib.sha256(a_p.cpu().numpy().tobytes()).hexdigest()[:10]})
            print(json.dumps(rows[-1]), flush=True)
    print(json.dumps({"worst": max(x["max_diff"] for x in rows),
                      "distinct_a_full": len({x["a_full"] for x in rows}),
                      "distinct_a_p": len({x["a_p"] for x in rows}), "distinct_M": len({x["M"] for x in rows})}))


if __name__ == "__main__":
    main()
