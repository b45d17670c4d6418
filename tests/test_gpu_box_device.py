"""Device box decomposition (box_device.hip) against the native host partition and the
oracle's exact hypervolume: same cell set per sample, bit for bit."""
import numpy as np
import pytest
import torch

from everest_amd import ops

pytestmark = pytest.mark.gpu


def _sorted_cells(lo, hi):
    a = np.concatenate([lo, hi], axis=1)
    return a[np.lexsort(a.T[::-1])]


def _front(S, n, m, seed, dup=False, discrete=False):
    rng = np.random.default_rng(seed)
    X = np.abs(rng.normal(size=(S, n, m)))
    X /= np.linalg.norm(X, axis=-1, keepdims=True)
    X *= 1 + 0.1 * rng.uniform(size=(S, n, 1))
    if discrete:                       # ties in coordinates
        X = np.round(X * 8) / 8
    if dup:                            # exact duplicate points
        X[:, n // 2] = X[:, 0]
    return -X                          # maximisation objective, ref -1.1


@pytest.mark.parametrize("m,n,S", [(1, 17, 4), (2, 40, 8), (3, 60, 16), (4, 50, 8), (5, 120, 32), (6, 40, 4)])
@pytest.mark.parametrize("variant", ["plain", "dup", "discrete"])
def test_device_box_decomposition_matches_host(m, n, S, variant):
    O = _front(S, n, m, seed=m * 100 + n, dup=variant == "dup", discrete=variant == "discrete")
    ref = -1.1 * np.ones(m)
    # a few points worse than the reference point and some dominated ones
    O[:, 1, 0] = -1.5
    O[:, 2] = O[:, 3] - 0.05
    lo_h, hi_h, off_h = ops.box_decompose(O, ref, None, 4, layout="sij")
    Od = torch.tensor(np.ascontiguousarray(O.transpose(2, 1, 0)), device="cuda")   # m x n x S
    cells = ops.box_decompose_device(Od, torch.tensor(ref, device="cuda"))
    lo_d, hi_d = cells.explicit()
    off_d = cells.off.cpu().numpy()
    assert np.array_equal(off_d, off_h)
    lo_d, hi_d = lo_d.cpu().numpy(), hi_d.cpu().numpy()
    for s in range(S):
        a, b = slice(off_h[s], off_h[s + 1]), slice(off_d[s], off_d[s + 1])
        assert np.array_equal(_sorted_cells(lo_h[a], hi_h[a]), _sorted_cells(lo_d[b], hi_d[b]))
        # device cells come sorted by first lower bound
        assert np.all(np.diff(lo_d[b][:, 0]) >= 0)


def test_device_box_decomposition_capacity_retry_and_determinism():
    O = _front(8, 80, 5, seed=3)
    Od = torch.tensor(np.ascontiguousarray(O.transpose(2, 1, 0)), device="cuda")
    ref = torch.full((5,), -1.1, dtype=torch.float64, device="cuda")
    c1 = ops.box_decompose_device(Od, ref, cap=4)         # overflows, reruns x4 ...
    c2 = ops.box_decompose_device(Od, ref)
    assert torch.equal(c1.off, c2.off) and torch.equal(c1.keys, c2.keys)
    (lo1, hi1), (lo2, hi2) = c1.explicit(), c2.explicit()
    assert torch.equal(lo1, lo2) and torch.equal(hi1, hi2)


def test_device_box_volume_equals_exact_hypervolume():
    """Sum of cell volumes clipped to a bounding box == exact HV of the front (oracle)."""
    from oracle import multiobjective as omo

    m, n = 3, 25
    O = _front(1, n, m, seed=11)[0]
    ref = -1.1 * np.ones(m)
    Od = torch.tensor(np.ascontiguousarray(O.T[:, :, None]), device="cuda")
    lo, hi = ops.box_decompose_device(Od, torch.tensor(ref, device="cuda")).explicit()
    lo, hi = lo.cpu().numpy(), hi.cpu().numpy()
    # cells partition the NON-dominated region above ref; HV = box(ref, cap) - non-dominated part
    cap = np.zeros(m)
    vol_nd = np.prod(np.clip(np.minimum(hi, cap) - lo, 0, None), axis=1).sum()
    P = omo.pareto_above_ref(torch.tensor(O), torch.tensor(ref)).numpy()
    hv = omo.hv_slicing(P, ref)
    assert abs((np.prod(cap - ref) - vol_nd) - hv) < 1e-10


@pytest.mark.parametrize("m,n,S", [(5, 280, 16), (3, 60, 8), (2, 300, 4)])
def test_device_box_lds_slab_equals_hbm_slab(m, n, S, monkeypatch):
    """The LDS-resident LUB slab (whole capacity beside an LDS staging area of A's indices and
    the step's new keys) gives bitwise the HBM slab's cells (EVR_BD_LDS=0)."""
    O = _front(S, n, m, seed=7 * m + n)
    Od = torch.tensor(np.ascontiguousarray(O.transpose(2, 1, 0)), device="cuda")
    ref = torch.full((m,), -1.1, dtype=torch.float64, device="cuda")
    monkeypatch.delenv("EVR_BD_LDS", raising=False)
    c1 = ops.box_decompose_device(Od, ref)
    monkeypatch.setenv("EVR_BD_LDS", "0")
    c2 = ops.box_decompose_device(Od, ref)
    assert torch.equal(c1.off, c2.off) and torch.equal(c1.keys, c2.keys)
    assert torch.equal(c1.pts, c2.pts) and torch.equal(c1.rank0, c2.rank0)


@pytest.mark.parametrize("m,n,S,cap", [(5, 120, 32, 16384), (3, 60, 16, 4), (2, 40, 8, 16384), (6, 40, 4, 64)])
def test_box_kd_pipeline_equals_op_sequence(m, n, S, cap):
    """evr_box_kd_pipeline (box, pack and kd order in one native call, capacity-sized outputs,
    the overflow rerun included at cap = 4 / 64) equals box_decompose_device + cells_kd_order
    bitwise: offsets, counts, keys, point tables, kd keys, rank coordinates, group minima,
    sorted lower bounds."""
    O = _front(S, n, m, seed=7 * m + n)
    Od = torch.tensor(np.ascontiguousarray(O.transpose(2, 1, 0)), device="cuda")
    ref = torch.tensor(-1.1 * np.ones(m), device="cuda")
    c1 = ops.box_decompose_device(Od, ref, cap=cap)
    k1 = ops.cells_kd_order(c1)
    c2, built = ops.box_decompose_kd_device(Od, ref, want_kd=True, cap=cap)
    assert built and c2.kd is not None
    assert np.array_equal(c1.counts, c2.counts)
    for a, b in ((c1.off, c2.off), (c1.keys, c2.keys), (c1.pts, c2.pts), (c1.rank0, c2.rank0),
                 (k1.goff, c2.kd.goff), (k1.keys, c2.kd.keys), (k1.rank, c2.kd.rank), (k1.box, c2.kd.box),
                 (k1.sorted_lo, c2.kd.sorted_lo)):
        assert torch.equal(a.cpu(), b.cpu())
