import sys; sys.path.insert(0,'.')
import numpy as np, torch
from tests.test_gpu_gp_qnehvi import _matched_qnehvi
X, lo, hi, orc, dq, idx = _matched_qnehvi(60, 6, 5, 16, seed=60, prune=True)
rng = np.random.default_rng(5)
Xc = lo + (hi - lo) * rng.uniform(size=(37, 6)); Xc[0] = X[0]
acq, dX = dq.forward_backward(torch.tensor(Xc, device="cuda"))
xt = torch.tensor(Xc, requires_grad=True)
ref = orc.forward(((xt - torch.tensor(lo)) / torch.tensor(hi - lo)).unsqueeze(1))
ref.sum().backward()
a = acq.cpu(); r = ref.detach()
print('abs err', (a-r).abs().max().item(), 'per cand', ((a-r).abs()/(r.abs()+1e-12)).numpy().round(8)[:10])
print('acq', a[:5].numpy(), r[:5].numpy())
print('grad err', (dX.cpu()-xt.grad).abs().max().item())
print('base jitter', dq.base_jitter.cpu().numpy())
_, (Xd, R, G, L22, flags) = dq.forward(torch.tensor(Xc, device="cuda"), return_cache=True)
print('L22 cand0', L22[:,0].cpu().numpy())
