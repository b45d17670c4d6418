"""Turn two rocprofv3 ``--pmc`` passes (FETCH_SIZE, WRITE_SIZE) over ``bench.py`` into the
per-launch HBM bytes of each bench op, written to profiles/hbm_traffic.json for bench.py's
``roofline.traffic``.

MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports half the bytes of a wide coalesced
read on gfx950 — doubled here; WRITE_SIZE is exact for 16 B/lane stores.  rocprofv3 reports
both in KiB.  Each bench op maps to the kernels it launches; the per-launch figure is the
sum over those kernels of their mean per-dispatch value.

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> [out.json]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

OPS = {
    "kernel_matrix": [r"kmat_kernel"],
    "proj_fwd": [r"qn_proj_fwd\(", r"qn_proj_fwd_reduce"],
    "samples": [r"qn_samples_norms"],
    "hvi_fwd_bwd": [r"hvi_thresholds", r"hvi_kd<", r"hvi_tiled<\d+, \d+, (true|false), true>", r"hvi_reduce_fwd",
                    r"hvi_reduce_bwd"],
    "proj_bwd": [r"qn_bwd_coef", r"qn_proj_bwd", r"qn_splitk_sum"],
    "kernel_grad": [r"kcross_grad_kernel"],
}
LAST = int(os.environ.get("PMC_LAST", "10"))   # tools/loop_step.py: the last N dispatches are the steps


def per_kernel(d, counter):
    vals = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            rows = [r for r in csv.DictReader(f) if r.get("Counter_Name") == counter]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        for row in rows:
            vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    vals = {k: v[-LAST:] for k, v in vals.items()}
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                                 "hbm_traffic.json")
    fetch, nf = per_kernel(fdir, "FETCH_SIZE")
    write, nw = per_kernel(wdir, "WRITE_SIZE")
    res = {}
    for op, pats in OPS.items():
        fb = wb = 0.0
        parts = {}
        for pat in pats:
            ks = [k for k in fetch if re.search(pat, k)]
            for k in ks:
                f_b = 2.0 * fetch[k] * 1024.0
                w_b = write.get(k, 0.0) * 1024.0
                fb += f_b
                wb += w_b
                parts[k[:80]] = {"fetch_bytes": f_b, "write_bytes": w_b, "dispatches": nf[k]}
        if parts:
            res[op] = {"bytes_per_launch": fb + wb, "fetch_bytes": fb, "write_bytes": wb, "kernels": parts,
                       "source": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE, KiB->B, mean per dispatch"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v["bytes_per_launch"] for k, v in res.items()}))


if __name__ == "__main__":
    main()
