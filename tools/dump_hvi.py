"""Dump the bench state's HVI inputs (samples G, cell lower/upper bounds, offsets) for
offline analysis of cell orderings / skip structures (float32 to fit the pull limit)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import bench
from everest_amd import ops
dev = torch.device("cuda", 0)
X, Y, gp, hypers, acqf, _, _ = bench.build_state(512, 6, 5, 256, dev)
Xc = bench.candidates(512, 6, seed=2, device=dev)
R = ops.gemm(acqf.M, gp.cross(Xc))
G, _, _ = ops.qnehvi_samples(acqf.state, R, 512)
lo, hi = acqf.cells.explicit()
acq = acqf.forward(Xc)
S = 128  # half the samples
off = acqf.cells.off.cpu().numpy()
np.savez_compressed(sys.argv[1], G=G[:S].cpu().numpy(), lo=lo[:off[S]].cpu().numpy().astype(np.float32),
                    hi=hi[:off[S]].cpu().numpy().astype(np.float32), off=off[:S + 1], acq=acq.cpu().numpy())
print("ok")
