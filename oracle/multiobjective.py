"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Multi-objective primitives restated from [upstream] BoTorch (called from
bofire/strategies/predictives/qnehvi.py:39-51 and bofire/utils/multiobjective.py:6-7):

* ``is_non_dominated`` (botorch.utils.multi_objective.pareto), maximisation, optional dedup.
* ``pad_batch_pareto_frontier`` (botorch.acquisition.multi_objective.utils._pad_batch_pareto_frontier).
* Local-upper-bound box decomposition of the non-dominated region
  (FastNondominatedPartitioning: Lacour, Klamroth & Fonseca 2017, Alg. 3; BoTorch
  ``compute_local_upper_bounds``), cells returned in maximisation space.
* Exact hypervolume by inclusion–exclusion and by slicing — independent checks.
"""
from __future__ import annotations

import itertools
from typing import List, Tuple

import numpy as np
import torch

TK = dict(dtype=torch.float64, device="cpu")


def is_non_dominated(Y: torch.Tensor, deduplicate: bool = True) -> torch.Tensor:
    """Y: ... x n x m (maximisation).  j dominates i iff Y_j >= Y_i all and > any."""
    n = Y.shape[-2]
    if n == 0:
        return torch.zeros(Y.shape[:-1], dtype=torch.bool)
    Y1 = Y.unsqueeze(-3)
    Y2 = Y.unsqueeze(-2)
    dominates = (Y1 >= Y2).all(dim=-1) & (Y1 > Y2).any(dim=-1)
    nd = ~dominates.any(dim=-1)
    if deduplicate:
        idx = (Y1 == Y2).all(dim=-1).long().argmax(dim=-1)
        keep = torch.zeros_like(nd)
        keep.scatter_(-1, idx, True)
        return nd & keep
    return nd


def pareto_above_ref(Y: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
    """Pareto set (dedup) of the points of Y (n x m) that are strictly better than ref."""
    mask = is_non_dominated(Y) & (Y > ref).all(-1)
    return Y[mask]


# ---------------------------------------------------------------------------------------
# Local upper bounds (minimisation frame)
# ---------------------------------------------------------------------------------------
def _init_lub(R: torch.Tensor):
    m = R.shape[0]
    U = R.clone().unsqueeze(0)                         # 1 x m
    Z = torch.full((1, m, m), -float("inf"), **TK)      # dummy defining points
    for j in range(m):
        Z[0, j, j] = R[j]
    return U, Z


def compute_local_upper_bounds(U, Z, z):
    """One incremental LUB update (minimisation) restated from BoTorch / Lacour17 Alg. 3."""
    m = U.shape[-1]
    dom = (U > z).all(dim=-1)
    if not dom.any():
        return U, Z
    A, AZ = U[dom], Z[dom]
    P, PZ = [], []
    mask = torch.ones(m, dtype=torch.bool)
    for j in range(m):
        mask[j] = False
        # m = 1: no other defining points, the projection is always admissible
        zmax = (AZ[:, mask, j].max(dim=-1).values if m > 1
                else torch.full((A.shape[0],), -float("inf"), dtype=A.dtype))
        add = z[j] >= zmax
        if add.any():
            uj = A[add].clone()
            uj[:, j] = z[j]
            P.append(uj)
            Zj = AZ[add].clone()
            Zj[:, j] = z
            PZ.append(Zj)
        mask[j] = True
    U = torch.cat([U[~dom]] + P, 0)
    Z = torch.cat([Z[~dom]] + PZ, 0)
    return U, Z


def nondominated_cells(pareto_Y: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
    """Disjoint boxes covering the region above ``ref`` not dominated by ``pareto_Y``
    (maximisation).  Returns 2 x C x m (lower, upper); upper may be +inf.

    Box for a local upper bound u (minimisation frame, z = -y):
        dim 0: (-inf, u_0);  dim j>=1: [max_{k<j} Z^k_j(u), u_j)
    mapped back to maximisation space by negation."""
    m = ref.shape[0]
    R = -ref
    U, Z = _init_lub(R)
    for p in pareto_Y:
        U, Z = compute_local_upper_bounds(U, Z, -p)
    C = U.shape[0]
    lo = torch.empty(C, m, **TK)
    lo[:, 0] = -float("inf")
    for j in range(1, m):
        lo[:, j] = Z[:, :j, j].max(dim=-1).values
    lower = -U
    upper = -lo
    keep = (upper > lower).all(-1)
    return torch.stack([lower[keep], upper[keep]], 0)


def approximate_cells(pareto_Y: torch.Tensor, ref: torch.Tensor, alpha: float) -> torch.Tensor:
    """[upstream] NondominatedPartitioning(ref, Y, alpha)._partition_space +
    get_hypercell_bounds for m > 2 (BoFire passes alpha at
    bofire/strategies/predictives/qnehvi.py:50 and mobo.py:83): binary partitioning over
    indices of the augmented front, minimisation frame z = -y.  Index 0 is the ideal point
    (per-objective minimum of the front; -inf in the reported bounds), 1..P the front sorted
    per objective (stable), P+1 the reference point.  A cell whose upper corner no front point
    dominates is kept; one whose lower corner passes is split along its widest index span
    (upper half minus round(span / 2), lower half plus the rest) while some span exceeds 1 and
    its volume / (ref - ideal volume) exceeds alpha, else dropped.  Returns 2 x C x m
    (maximisation lower, upper) in stack-pop order.  Parity unpinned: BoTorch is not
    available here; the ideal-point volume normaliser is this restatement's reading."""
    m = ref.shape[0]
    Z = -pareto_Y
    P = Z.shape[0]
    Rn = -ref
    idx = torch.argsort(Z, dim=0, stable=True)
    aug = torch.empty(P + 2, m, **TK)
    for j in range(m):
        aug[1:P + 1, j] = Z[idx[:, j], j]
    aug[0] = aug[1] if P else Rn
    aug[P + 1] = Rn
    total = float((Rn - aug[0]).prod())
    ar = torch.arange(m)
    out = []
    stack = [torch.stack([torch.zeros(m, dtype=torch.long), torch.full((m,), P + 1, dtype=torch.long)])]

    def undominated(corner):
        return bool((corner <= Z).any(dim=-1).all()) if P else True

    while stack:
        cell = stack.pop()
        vals = aug[cell, ar]                       # 2 x m
        if undominated(vals[1]):
            lo_z = vals[0].clone()
            lo_z[cell[0] == 0] = -float("inf")
            out.append(torch.stack([-vals[1], -lo_z]))
        elif undominated(vals[0]):
            dist = cell[1] - cell[0]
            vol = float((vals[1] - vals[0]).prod())
            if bool((dist > 1).any()) and vol / total > alpha:
                span, j = int(dist.max()), int(torch.argmax(dist))
                h1 = int(round(span / 2.0))
                for b, delta in ((1, -h1), (0, span - h1)):
                    c = cell.clone()
                    c[b, j] += delta
                    stack.append(c)
    if not out:
        return torch.empty(2, 0, m, **TK)
    cells = torch.stack(out, 1)
    keep = (cells[1] > cells[0]).all(-1)
    return cells[:, keep]


def hvi_from_cells(y: torch.Tensor, cells: torch.Tensor) -> torch.Tensor:
    """q=1 HVI of points y (... x m) w.r.t. cells (2 x C x m)."""
    lo, hi = cells[0], cells[1]
    lengths = (torch.minimum(y.unsqueeze(-2), hi) - lo).clamp_min(0.0)
    return lengths.prod(-1).sum(-1)


# ---------------------------------------------------------------------------------------
# exact hypervolume (independent checks)
# ---------------------------------------------------------------------------------------
def hv_inclusion_exclusion(P: np.ndarray, ref: np.ndarray) -> float:
    P = np.asarray(P, dtype=np.float64)
    n = P.shape[0]
    tot = 0.0
    for k in range(1, n + 1):
        sgn = 1.0 if k % 2 == 1 else -1.0
        for S in itertools.combinations(range(n), k):
            v = np.clip(P[list(S)].min(0) - ref, 0.0, None).prod()
            tot += sgn * v
    return tot


def hv_slicing(P: np.ndarray, ref: np.ndarray) -> float:
    """Hypervolume by recursive slicing along the last objective (maximisation)."""
    P = np.asarray(P, dtype=np.float64)
    P = P[(P > ref).all(1)]
    if P.shape[0] == 0:
        return 0.0
    m = P.shape[1]
    if m == 1:
        return float(P[:, 0].max() - ref[0])
    order = np.argsort(-P[:, -1])
    P = P[order]
    tot = 0.0
    for k in range(P.shape[0]):
        top = P[k, -1]
        bot = P[k + 1, -1] if k + 1 < P.shape[0] else ref[-1]
        if top > bot:
            tot += (top - bot) * hv_slicing(P[: k + 1, :-1], ref[:-1])
    return tot
