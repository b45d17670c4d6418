"""Loop the sparse HVI scan at one batch size (for rocprofv3 traces / counters)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from everest_amd import ops
b = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda", 0)
X, Y, gp, hypers, acqf, _, _ = bench.build_state(512, 6, 5, 256, dev)
Xc = bench.candidates(b, 6, seed=2, device=dev)
R = ops.gemm(acqf.M, gp.cross(Xc))
G, L22, flags = ops.qnehvi_samples(acqf.state, R, b)
for _ in range(10):
    ops.hvi_forward_backward(acqf.state, G, b, flags)
torch.cuda.synchronize()
print("done")
