"""Per-kernel device time of one qNEHVI evaluation pass at several batch sizes, and the
construction sub-phases (HIP events on torch's current stream)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

import bench


def main():
    dev = torch.device("cuda", 0)
    X, Y, gp, hypers, acqf, t_fit, t_build = bench.build_state(512, 6, 5, 256, dev)
    out = {"fit_s": t_fit, "build_s": t_build, "build_phases": acqf.timings}
    for b in (20, 128, 512, 1024):
        Xc = bench.candidates(b, 6, seed=2, device=dev)
        for _ in range(3):
            bench.step(acqf, Xc)
        torch.cuda.synchronize()
        timer = bench.KernelTimer()
        for _ in range(10):
            bench.step(acqf, Xc, timer)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            acq, dX = acqf.forward_backward(Xc)
            dX.cpu()
        host = (time.perf_counter() - t0) / 10 * 1e3
        out[f"b{b}"] = {"kernel_ms": {k: round(v, 4) for k, v in timer.summary().items()},
                        "fwd_bwd_wall_ms_incl_sync": round(host, 4)}
    # construction phases with finer sync points
    from everest_amd.acquisition import sobol_base_samples
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    z = sobol_base_samples(2048, 512, 5, 1, dev)
    torch.cuda.synchronize()
    out["device_sobol_2048x2560_s"] = time.perf_counter() - t0
    print(json.dumps(out, default=float))


if __name__ == "__main__":
    main()
