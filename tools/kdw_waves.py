"""Per-(sample, candidate) wall-clock phases of the restart scan hvi_kdw on the EVR_KD_PROF=2
build (EVR_LIB_PATH=everest_amd/_libkdprof/libeverest_amd.so, make EXTRA=-DEVR_KD_PROF=2
OUT=../_libkdprof BUILD=../_buildkdprof): staging, sampling + thresholds, group / cell
phases, term rounds, reduction; means / p90 / max over waves, the launch span, term and
passing-group counts — at the bench state (config 4 after one ask, seed 1) on its optimised
restart candidates and on Sobol candidates (b = 20).  s_memrealtime: 100 MHz.  One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
from everest_amd import ops


def main():
    dev = torch.device("cuda", 0)
    s, _ = bench.make_ask_strategy(512, 256, 1024, 20, 1, None, seed=1)
    s.ask(1)
    acqf = s.last_acqf
    st = acqf.state
    Xopt = torch.tensor(s.last_ask_stats.restart_X.reshape(20, -1), device=dev)
    out = {}
    for tag, Xc in (("opt", Xopt), ("sobol", bench.candidates(20, 6, seed=5, device=dev))):
        b = Xc.shape[0]
        R, P = ops.qnehvi_small_forward(st, acqf.model, acqf.gp.cross(Xc), b)
        G, L22, flags = ops.qnehvi_small_samples(st, R, P, b)
        S = int(st.S)
        ctr = torch.zeros(16 + 8 * S * b, dtype=torch.int64, device=dev)
        st.scan_counters = ctr.data_ptr()
        try:
            ops.hvi_restart_fb(st, G, b)
            torch.cuda.synchronize()
        finally:
            st.scan_counters = None
        rec = ctr.cpu().numpy()[16:].reshape(S * b, 8).astype(np.float64)
        if not rec[:, 0].any():
            out[tag] = "production build: no stamps"
            continue
        t0 = rec[:, 0].min()
        stage = (rec[:, 1] - rec[:, 0]) / 100.0
        thr = (rec[:, 2] - rec[:, 1]) / 100.0
        grp = rec[:, 3] / 100.0
        term = rec[:, 4] / 100.0
        tot = (rec[:, 5] - rec[:, 0]) / 100.0
        red = tot - stage - thr - grp - term
        q = lambda v: {"mean": round(float(v.mean()), 2), "p90": round(float(np.percentile(v, 90)), 2),  # noqa: E731
                       "max": round(float(v.max()), 2)}
        out[tag] = {"span_us": round(float(rec[:, 5].max() - t0) / 100.0, 2),
                    "start_spread_us": round(float(rec[:, 0].max() - t0) / 100.0, 2),
                    "wave_total_us": q(tot), "staging_us": q(stage), "sampling_thresholds_us": q(thr),
                    "group_cell_us": q(grp), "term_rounds_us": q(term), "reduction_us": q(red),
                    "terms": q(rec[:, 6]), "passing_groups": q(rec[:, 7])}
        # what balancing the variable work (group / cell phases + term rounds) would leave:
        # within each workgroup's 4 candidates, and within each sample's b candidates
        var = (grp + term).reshape(S, b)
        fixed = (stage + thr + red).reshape(S, b)
        nwg = (b + 3) // 4
        wg_bal = [fixed[:, 4 * g:4 * g + 4].max(1) + var[:, 4 * g:4 * g + 4].mean(1) for g in range(nwg)]
        out[tag]["balance"] = {"max_wave_us": round(float(tot.max()), 2),
                               "max_wg_balanced_us": round(float(np.max(wg_bal)), 2),
                               "max_sample_balanced_us": round(float((fixed.max(1) + var.mean(1)).max()), 2),
                               "max_wave_of_heaviest_sample_us": round(float(tot.reshape(S, b).max(1)[
                                   int(np.argmax(var.mean(1)))]), 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
