"""CPU, world_size 2 over gloo: the sharded raw screening + sharded restart evaluation of
optimize_acqf (RCCL all-gathers on the GPUs) returns exactly the single-process result.
The per-shard evaluator here is the CPU oracle (test infrastructure); on the MI355X the
same code path calls the HIP acquisition."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class OracleAcq:
    """forward / forward_backward over a fixed smooth multi-modal function (CPU)."""
    dev = torch.device("cpu")

    def _f(self, X):
        return torch.exp(-((X - 0.3) ** 2).sum(-1) * 8) + 0.5 * torch.exp(-((X - 0.8) ** 2).sum(-1) * 20)

    def forward(self, X):
        return self._f(X.to(torch.float64))

    def forward_backward(self, X):
        x = X.to(torch.float64).clone().requires_grad_(True)
        v = self._f(x)
        v.sum().backward()
        return v.detach(), x.grad


def _run(rank, world, port, ret):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from everest_amd.optim import optimize_acqf

    gen = torch.Generator().manual_seed(7)
    bounds = np.array([[0.0] * 3, [1.0] * 3])
    x, v, st = optimize_acqf(OracleAcq(), bounds, num_restarts=5, raw_samples=64,
                             options={"batch_limit": 5, "maxiter": 200}, gen=gen, dist=dist)
    ret[rank] = (x.tolist(), v, st.raw_evals)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_optimize_acqf_matches_single_process():
    from everest_amd.optim import optimize_acqf

    gen = torch.Generator().manual_seed(7)
    bounds = np.array([[0.0] * 3, [1.0] * 3])
    x1, v1, _ = optimize_acqf(OracleAcq(), bounds, num_restarts=5, raw_samples=64,
                              options={"batch_limit": 5, "maxiter": 200}, gen=gen)
    mgr = mp.Manager()
    ret = mgr.dict()
    port = _free_port()
    mp.spawn(_run, args=(2, port, ret), nprocs=2, join=True)
    for r in range(2):
        xr, vr, nraw = ret[r]
        assert np.allclose(xr, x1, atol=1e-12) and abs(vr - v1) < 1e-14 and nraw == 64
    assert v1 > 0.9


def test_boltzmann_init_nonneg_semantics():
    from everest_amd.optim import initialize_q_batch_nonneg

    gen = torch.Generator().manual_seed(0)
    X = np.arange(20, dtype=np.float64)[:, None]
    acq = np.linspace(0, 1, 20)
    Xs, a = initialize_q_batch_nonneg(X, acq, 5, gen)
    assert len(Xs) == 5 and 19.0 in Xs[:, 0]            # the max is always included
    Xs, a = initialize_q_batch_nonneg(X, np.zeros(20), 5, gen)   # all non-positive -> random
    assert len(Xs) == 5


class HostEvalAcq(OracleAcq):
    """Stand-in with the device acquisitions' ``eval_host`` round trip (the branch the
    single-rank GPU ask takes, optim.run_chunk) next to forward / forward_backward (the
    branch the sharded joint evaluation takes)."""

    def eval_host(self, x, backward):
        a, g = self.forward_backward(torch.as_tensor(x))
        return a.numpy(), (g.numpy() if backward else None)


class FlakyAcq(OracleAcq):
    """NaN acquisition values (a failed jitter ladder) on rank 1's restart chunks only."""

    def forward_backward(self, X):
        a, g = super().forward_backward(X)
        if dist.is_initialized() and dist.get_rank() == 1:
            a = torch.full_like(a, float("nan"))
        return a, g


class RaisingAcq(HostEvalAcq):
    """A rank-local launch failure (an exception, not NaN) on rank 1 inside the joint chunk's
    sharded evaluation: its group peer must not be left waiting in the per-evaluation gather."""

    def eval_host(self, x, backward):
        if dist.is_initialized() and dist.get_rank() == 1:
            raise RuntimeError("simulated native launch failure")
        return super().eval_host(x, backward)

    def forward(self, X):      # raw screening stays healthy on every rank
        return super().forward(X)


def _run_generic(rank, world, port, ret, acq_name, options):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from everest_amd.optim import optimize_acqf

    acq = {"host": HostEvalAcq, "flaky": FlakyAcq, "raising": RaisingAcq}[acq_name]()
    gen = torch.Generator().manual_seed(7)
    bounds = np.array([[0.0] * 3, [1.0] * 3])
    try:
        x, v, st = optimize_acqf(acq, bounds, num_restarts=4, raw_samples=64, options=options, gen=gen, dist=dist)
        ret[rank] = ("ok", x.tolist(), v)
    except Exception as e:  # noqa: BLE001
        ret[rank] = ("error", type(e).__name__, str(e))
    dist.destroy_process_group()


def _spawn(acq_name, options, timeout=120):
    mgr = mp.Manager()
    ret = mgr.dict()
    ctx = mp.start_processes(_run_generic, args=(2, _free_port(), ret, acq_name, options), nprocs=2, join=False,
                             start_method="spawn")
    deadline = timeout
    import time
    t0 = time.time()
    while not ctx.join(timeout=5):
        if time.time() - t0 > deadline:
            for p in ctx.processes:
                p.kill()
            raise AssertionError("ranks did not finish: a collective is waiting on a rank that left")
    return dict(ret)


def test_eval_host_branch_matches_sharded_branch():
    """The single-process eval_host path (native L-BFGS-B, Python callback) and the 2-rank
    sharded joint chunk (all-gather of (value, grad) per iteration) take identical steps."""
    from everest_amd.optim import optimize_acqf

    gen = torch.Generator().manual_seed(7)
    bounds = np.array([[0.0] * 3, [1.0] * 3])
    opts = {"batch_limit": 4, "maxiter": 200}
    x1, v1, st1 = optimize_acqf(HostEvalAcq(), bounds, num_restarts=4, raw_samples=64, options=opts, gen=gen)
    assert st1.chunks[0]["driver"] == "native"
    ret = _spawn("host", opts)
    for r in range(2):
        status, xr, vr = ret[r]
        assert status == "ok"
        assert np.allclose(xr, x1, atol=1e-12) and abs(vr - v1) < 1e-14


def test_own_chunk_failure_raises_on_every_rank():
    """batch_limit < num_restarts: each rank optimises its own chunks with no per-iteration
    collective; a NotPSD failure on rank 1 must raise on both ranks (not leave rank 0 waiting
    in the final all-gather)."""
    ret = _spawn("flaky", {"batch_limit": 1, "maxiter": 50})
    assert ret[0][0] == "error" and ret[1][0] == "error"
    assert ret[0][1] == "NotPSDError" and ret[1][1] == "NotPSDError"


def test_sharded_rank_exception_raises_on_every_member():
    """batch_limit = num_restarts: both ranks evaluate the joint chunk, rank 1's evaluation
    raises; the error flag travels with the gathered slice, so both raise (no hang)."""
    ret = _spawn("raising", {"batch_limit": 4, "maxiter": 50})
    assert ret[0][0] == "error" and ret[1][0] == "error", ret
    assert ret[1][1] == "RuntimeError" and "simulated" in ret[1][2]
    assert ret[0][1] == "RuntimeError" and "rank(s) [1]" in ret[0][2]


def test_restart_layout_no_idle_ranks():
    """Chunks >= ranks: whole chunks per rank; fewer chunks: one contiguous rank group per
    chunk, sizes within one, every rank used (the N = 6 / 8 case of 20 restarts in chunks)."""
    from everest_amd.optim import restart_layout

    assert restart_layout(1, 8) == [tuple(range(8))]
    assert restart_layout(3, 8) == [(0, 1, 2), (3, 4, 5), (6, 7)]
    assert restart_layout(7, 8) == [(0, 1), (2,), (3,), (4,), (5,), (6,), (7,)]
    assert restart_layout(5, 3) == [(0,), (1,), (2,), (0,), (1,)]
    for c in range(1, 12):
        for w in range(1, 10):
            lay = restart_layout(c, w)
            assert len(lay) == c
            used = sorted(r for g in lay for r in g)
            if c < w:
                assert used == list(range(w))             # no idle rank
                sz = [len(g) for g in lay]
                assert max(sz) - min(sz) <= 1


def _run_layout(rank, world, port, ret, acq_name, restarts, batch_limit):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from everest_amd.optim import optimize_acqf

    acq = {"plain": OracleAcq, "host": HostEvalAcq}[acq_name]()
    gen = torch.Generator().manual_seed(11)
    bounds = np.array([[0.0] * 3, [1.0] * 3])
    try:
        x, v, st = optimize_acqf(acq, bounds, num_restarts=restarts, raw_samples=64,
                                 options={"batch_limit": batch_limit, "maxiter": 200}, gen=gen, dist=dist)
        ret[rank] = ("ok", x.tolist(), v, st.opt_evals_global, [c["driver"] for c in st.chunks])
    except Exception as e:  # noqa: BLE001
        ret[rank] = ("error", type(e).__name__, str(e))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("restarts,batch_limit,acq_name", [(5, 5, "host"), (5, 2, "plain"), (6, 1, "host")])
def test_sharded_layouts_match_single_process(world, restarts, batch_limit, acq_name):
    """The reference's problem at every world size: one joint chunk (batch_limit =
    num_restarts) evaluated by all ranks, chunks >= ranks owned whole, and chunks < ranks
    evaluated by rank groups — best (x, value) and the global evaluation count equal the
    single-process run."""
    from everest_amd.optim import optimize_acqf

    acq = {"plain": OracleAcq, "host": HostEvalAcq}[acq_name]()
    gen = torch.Generator().manual_seed(11)
    bounds = np.array([[0.0] * 3, [1.0] * 3])
    x1, v1, st1 = optimize_acqf(acq, bounds, num_restarts=restarts, raw_samples=64,
                                options={"batch_limit": batch_limit, "maxiter": 200}, gen=gen)
    mgr = mp.Manager()
    ret = mgr.dict()
    ctx = mp.start_processes(_run_layout, args=(world, _free_port(), ret, acq_name, restarts, batch_limit),
                             nprocs=world, join=False, start_method="spawn")
    import time
    t0 = time.time()
    while not ctx.join(timeout=5):
        if time.time() - t0 > 240:
            for p in ctx.processes:
                p.kill()
            raise AssertionError("ranks did not finish")
    ret = dict(ret)
    n_chunks = -(-restarts // batch_limit)
    for r in range(world):
        status, xr, vr, evals, drivers = ret[r]
        assert status == "ok", ret[r]
        assert np.allclose(xr, x1, atol=1e-12) and abs(vr - v1) < 1e-14
        assert evals == st1.opt_evals_global
    if n_chunks < world:
        assert any("sharded" in dv for r in range(world) for dv in ret[r][4])
