"""Run-to-run determinism of the bench state: builds bench.build_state (the config-3 GP fit,
prune, baseline, box decomposition, operator) in this process and prints digests of the fitted
hyperparameters, the operator M, the pruned baseline rows and the cells, plus the batch-split
difference of tests/test_gpu_baseline_sizes.py::test_config3_batch_split_equals_full_batch.
Run it twice in fresh processes and compare the lines.  usage: python tools/determinism_probe.py"""
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def h(x):
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().contiguous().numpy()
    return hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()[:12]


def main():
    import bench

    dev = torch.device("cuda", 0)
    X, Y, gp, hypers, acqf, _, _ = bench.build_state(512, 6, 5, 256, dev)
    out = {"hypers": h(np.concatenate([np.r_[hh.lengthscale, hh.noise, hh.constant] for hh in hypers])),
           "Linv": h(gp.Linv), "M": h(acqf.M), "base_rows": h(np.asarray(acqf.base_rows)),
           "cells_keys": h(acqf.cells.keys) if acqf.cells.keys is not None else None}
    Xc = bench.candidates(512, 6, seed=3, device=dev)
    a_full, _ = acqf.forward_backward(Xc)
    a_p = torch.cat([acqf.forward_backward(Xc[i:i + 20])[0] for i in range(0, 500, 20)])
    out["a_full"] = h(a_full)
    out["split_max_abs_diff"] = float((a_full[:500] - a_p).abs().max())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
