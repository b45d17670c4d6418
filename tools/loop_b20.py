"""Small-batch evaluation loop (the L-BFGS restart shape) for rocprofv3 kernel traces."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench

dev = torch.device("cuda", 0)
X, Y, gp, hypers, acqf, t_fit, t_build = bench.build_state(512, 6, 5, 256, dev)
for b in (20, 512):
    Xc = bench.candidates(b, 6, seed=2, device=dev)
    for _ in range(30):
        acq, dX = acqf.forward_backward(Xc)
    torch.cuda.synchronize()
print("done")
