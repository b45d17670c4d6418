"""Config 4 sharded over ranks (BASELINE configs[3]) on the GPU: the full
QnehviStrategy.ask() at n = 512, S = 256, 1024 raw Sobol candidates, 20 restarts as one joint
L-BFGS-B problem (batch_limit = num_restarts,
bofire/data_models/strategies/predictives/botorch.py:101-108), run once by one rank and once
by two ranks that split the raw screening and the restart batch and exchange (value, gradient)
every evaluation (optim._Shard) — both through the HIP acquisition.  The two-rank ask must
return bitwise the one-rank candidate, best value and global evaluation count.

The ranks are fresh interpreters started by tools/sharded_ask_check.py (subprocess children;
each touches HIP only after it starts) and share the box's one GPU over gloo; on a multi-GPU
node the same code runs one rank per GPU over RCCL (bench.py, EVR_DIST_BACKEND)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_config4_two_rank_ask_bitwise_equals_one_rank(tmp_path):
    out = tmp_path / "sharded"
    cmd = [sys.executable, os.path.join(ROOT, "tools", "sharded_ask_check.py"), "--ranks", "2", "--asks", "2",
           "--out", str(out)]
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, f"sharded ask failed (rc {r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    res = json.loads((out / "sharded_ask.json").read_text())
    print(json.dumps(res))
    assert res["ranks"] == 2 and len(res["asks"]) == 2
    for row in res["asks"]:
        assert row["x_bitwise_equal"] and row["best_value_bitwise_equal"], row
        p, q = row["opt_evals_global"]
        assert p == q, row
        # the 2-rank run really sharded the joint chunk: one group of two ranks, 10 restarts each
        assert row["drivers"][0] == ["native-plan"] and row["drivers"][1] == ["native-sharded2"], row
    w2 = json.loads((out / "w2.json").read_text())
    assert all(a["local_batch"] == [10] for a in w2["asks"]), w2


def test_config4_per_shard_argmax_two_ranks_bitwise_equals_one_rank(tmp_path):
    """The independent-restart layout (the north star's "all-gather of per-shard argmax"):
    batch_limit = 1 makes every one of the 20 restarts its own L-BFGS-B problem, as BoFire
    forces under NChooseK / product constraints (bofire/strategies/predictives/botorch.py:
    114-126).  With at least as many chunks as ranks, chunk c runs alone on rank c mod 2 with
    no per-iteration collective; one final all-gather of (error flag, best value, x) picks the
    argmax (optim.optimize_acqf).  Candidate, best value and global evaluation count must be
    bitwise those of one rank running all 20 chunks."""
    out = tmp_path / "sharded_bl1"
    cmd = [sys.executable, os.path.join(ROOT, "tools", "sharded_ask_check.py"), "--ranks", "2", "--asks", "2",
           "--batch-limit", "1", "--out", str(out)]
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, f"sharded ask failed (rc {r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    res = json.loads((out / "sharded_ask.json").read_text())
    print(json.dumps(res))
    assert res["ranks"] == 2 and len(res["asks"]) == 2
    for row in res["asks"]:
        assert row["x_bitwise_equal"] and row["best_value_bitwise_equal"], row
        p, q = row["opt_evals_global"]
        assert p == q, row
        # one rank ran all 20 single-restart problems; rank 0 of two ran its 10 (chunks 0, 2, ...)
        assert row["drivers"][0] == ["native-plan"] * 20 and row["drivers"][1] == ["native-plan"] * 10, row
    w2 = json.loads((out / "w2.json").read_text())
    assert all(a["local_batch"] == [1] * 10 for a in w2["asks"]), w2
