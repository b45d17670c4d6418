"""Phases of the kd ordering kernel (cells_kd.hip) per MC sample on the EVR_CKD_PROF build
(EVR_LIB_PATH=everest_amd/_libprof4/libeverest_amd.so, make EXTRA=-DEVR_CKD_PROF
OUT=../_libprof4 BUILD=../_buildp4): rank tables, then per kd level the span reduction, key
formation, bitonic sort and split, then the outputs; means / max over the samples of the bench
state's last construction (config 4, seed 1).  s_memrealtime: 100 MHz.  One JSON line."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
from everest_amd import _native


def main():
    s, _ = bench.make_ask_strategy(512, 256, 1024, 20, 1, None, seed=1)
    s.ask(1)
    s.ask(1)
    torch.cuda.synchronize()
    lib = _native.load()
    if not hasattr(lib, "evr_ckd_prof_read"):
        print(json.dumps({"error": "production build: no stamps"}))
        return
    S = 256
    buf = (ctypes.c_ulonglong * (16 * S))()
    _native.check(lib.evr_ckd_prof_read(buf, S), "evr_ckd_prof_read")
    r = np.frombuffer(buf, dtype=np.uint64).reshape(S, 16).astype(np.float64)
    q = lambda v: {"mean": round(float(v.mean()), 2), "max": round(float(v.max()), 2)}  # noqa: E731
    out = {"span_us": round(float(r[:, 6].max() - r[:, 0].min()) / 100.0, 2),
           "sample_total_us": q((r[:, 6] - r[:, 0]) / 100.0),
           "rank_tables_us": q((r[:, 1] - r[:, 0]) / 100.0),
           "spans_us": q(r[:, 2] / 100.0), "keys_us": q(r[:, 3] / 100.0), "sorts_us": q(r[:, 4] / 100.0),
           "splits_us": q(r[:, 5] / 100.0), "levels": q(r[:, 7])}
    lv = r[:, 2] + r[:, 3] + r[:, 4] + r[:, 5]
    out["outputs_us"] = q((r[:, 6] - r[:, 1] - lv) / 100.0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
