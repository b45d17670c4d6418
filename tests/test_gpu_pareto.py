"""evr_pareto_mask (prune_inferior_points' per-sample Pareto test and the partitions'
non-dominated filter) against a direct numpy statement of the rule, for the LDS-staged
kernel and the per-point fallback (points of one sample beyond the LDS budget), with ties,
duplicates and dedup on/off."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _reference(O, ref, dedup):
    m, n, S = O.shape
    mask = np.zeros((S, n), dtype=np.uint8)
    for s in range(S):
        Y = O[:, :, s].T
        better = (Y > ref).all(1)
        ge = (Y[None, :, :] >= Y[:, None, :]).all(2)      # [i, k]: k >= i everywhere
        gt = (Y[None, :, :] > Y[:, None, :]).any(2)
        dom = (ge & gt)
        np.fill_diagonal(dom, False)
        nd = better & ~dom.any(1)
        if dedup:
            eq = (Y[None, :, :] == Y[:, None, :]).all(2)
            dup = np.tril(eq, -1).any(1)                  # an earlier identical point
            nd &= ~dup
        mask[s] = nd
    return mask


@pytest.mark.parametrize("m,n,S", [(5, 300, 37), (3, 64, 130), (2, 1000, 9), (5, 2600, 3), (5, 509, 11),
                                   (3, 601, 7), (3, 1201, 3)])
@pytest.mark.parametrize("dedup", [False, True])
@pytest.mark.parametrize("near", [False, True])
def test_pareto_mask_matches_rule(m, n, S, dedup, near):
    """near: values a few f64 ulps apart, equal after rounding to f32 — the f32 pre-filter
    passes those pairs and the exact f64 test has to decide them.  n = 601 / 1201 with m = 3
    put an odd number of f64 values ahead of the f32 copy in LDS (3 and 1 samples per
    block): the f32 region must still start 16-byte aligned."""
    from everest_amd import ops

    rng = np.random.default_rng(n + S)
    O = np.round(rng.normal(size=(m, n, S)), 1)          # coarse grid: ties and duplicates
    if near:
        O = O + rng.integers(-2, 3, size=O.shape) * np.spacing(np.abs(O) + 1.0)
    O[:, 5, :] = O[:, 3, :]                              # exact duplicate points
    ref = np.full(m, -1.5)
    mask, counts = ops.pareto_mask(torch.tensor(O, device="cuda"), torch.tensor(ref, device="cuda"), dedup,
                                   want_mask=True, want_counts=True)
    want = _reference(O, ref, dedup)
    assert np.array_equal(mask.cpu().numpy(), want)
    assert np.array_equal(counts.cpu().numpy(), want.sum(0))


@pytest.mark.parametrize("m", [1, 2, 3])
@pytest.mark.parametrize("dedup", [False, True])
def test_pareto_mask_infinities(m, dedup):
    """Objectives beyond the f32 range and +inf: equal infinities compare equal (a duplicate
    of an infinite point, and a dominator that ties at +inf in some objective, must still be
    found by the f32 pre-filter)."""
    from everest_amd import ops

    rng = np.random.default_rng(m)
    n, S = 40, 5
    O = np.round(rng.normal(size=(m, n, S)), 1)
    O[:, 3, :] = np.inf
    O[:, 7, :] = np.inf                                  # duplicate of point 3
    O[0, 11, :] = 1e300                                  # beyond f32: rounds to +inf in the filter
    O[0, 12, :] = 1e300
    if m > 1:
        O[1:, 12, :] = O[1:, 11, :] + 1.0                # 12 dominates 11 (tie at 1e300)
    ref = np.full(m, -1.5)
    mask, counts = ops.pareto_mask(torch.tensor(O, device="cuda"), torch.tensor(ref, device="cuda"), dedup,
                                   want_mask=True, want_counts=True)
    want = _reference(O, ref, dedup)
    assert np.array_equal(mask.cpu().numpy(), want)
    assert np.array_equal(counts.cpu().numpy(), want.sum(0))
