"""Host-side strategy logic that needs no device: the generator stream of the EXHAUSTIVE
categorical q > 1 ask (BotorchStrategy._ask_mixed_sequential)."""
import types

import numpy as np
import torch

from everest_amd import strategies


def test_mixed_sequential_rng_stream_follows_reference_order(monkeypatch):
    """[upstream] optimize_acqf_mixed(q > 1) runs on an acquisition built ONCE: its seed
    draws come first, then every round's optimiser draws follow one another.  The rebuilt
    per-round acquisitions must see the same seeds, round 1's optimiser must start after the
    build's draws (not replay them), and round k + 1 after round k's draws."""
    gen = torch.Generator().manual_seed(123)
    seen = {"build": [], "opt": []}

    def build(q):
        # the acquisition's two seed draws (prune / sampler seeds)
        seen["build"].append(torch.randint(10**6, (2,), generator=gen).tolist())
        return [object()]

    def fake_mixed(acqf, bounds, combos, nr, nraw, opts, g, ineq, eq, dist=None, q=1):
        # the optimiser's raw-sample seed + two Boltzmann draws
        seen["opt"].append(torch.randint(10**7, (3,), generator=g).tolist())
        return np.zeros(2), 0.5, object()

    monkeypatch.setattr(strategies, "optimize_acqf_mixed", fake_mixed)
    fake = types.SimpleNamespace(gen=gen, _get_acqfs=build, _bounds=lambda: np.zeros((2, 2)), num_restarts=2,
                                 num_raw_samples=4, _get_optimizer_options=lambda: {}, dist=None)
    strategies.BotorchStrategy._ask_mixed_sequential(fake, 3, [{}], [], [])

    ref = torch.Generator().manual_seed(123)
    build_ref = torch.randint(10**6, (2,), generator=ref).tolist()
    opt_ref = [torch.randint(10**7, (3,), generator=ref).tolist() for _ in range(3)]
    assert seen["build"] == [build_ref] * 3
    assert seen["opt"] == opt_ref
    assert torch.equal(gen.get_state(), ref.get_state())   # the stream ends where the reference's does
