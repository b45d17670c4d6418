"""Turn two rocprofv3 ``--pmc`` passes (FETCH_SIZE, WRITE_SIZE) over ``tools/loop_step.py``
into the per-launch HBM bytes of each bench op, written to profiles/hbm_traffic.json for
bench.py's ``roofline.traffic``.

MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports half the bytes of a wide coalesced
read on gfx950 — doubled here; WRITE_SIZE is exact for 16 B/lane stores.  rocprofv3 reports
both in KiB.  Dispatches are labelled with the bench op that launches them; a step starts at
each kmat_kernel dispatch; the per-launch figure of an op is its summed bytes per step,
averaged over the last PMC_LAST steps.

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> [out.json] [suffix]
(suffix, e.g. "@b20" for a tools/loop_step.py N 20 pass: keys become op@b20 and are merged into
an existing out.json)
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

OPS = [
    ("kernel_matrix", r"kmat_kernel"),
    ("proj_fwd", r"qn_proj_fwd|qs_fwd"),
    ("samples", r"qn_samples_norms"),
    ("hvi_fwd_bwd", r"hvi_thresholds|hvi_kd[23bw]?<|hvi_tiled<|hvi_reduce_fwd|hvi_reduce_bwd|hvi_reduce_fb"),
    ("proj_bwd", r"qn_bwd_coef|qn_proj_bwd|qn_splitk_sum|qs_bwd|qs_dx_reduce"),
    ("kernel_grad", r"kcross_grad"),
]
LAST = int(os.environ.get("PMC_LAST", "10"))   # tools/loop_step.py: the last N steps


def label(name, prev):
    for op, pat in OPS:
        if re.search(pat, name):
            return op
    return None


def per_step(d, counter):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            rows += [r for r in csv.DictReader(f) if r.get("Counter_Name") == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    steps, snames, cur, prev = [], [], None, None
    for r in rows:
        op = label(r["Kernel_Name"], prev)
        if op is None:
            continue
        if op == "kernel_matrix":
            cur = defaultdict(float)
            steps.append(cur)
            snames.append(defaultdict(set))
        if cur is None:
            continue
        cur[op] += float(r["Counter_Value"]) * 1024.0   # KiB -> B
        snames[-1][op].add(r["Kernel_Name"].split("(")[0][:80])
        prev = op
    names = defaultdict(set)   # the kernels of the steps counted (not of the set-up before them)
    for sn in snames[-LAST:]:
        for op, ks in sn.items():
            names[op] |= ks
    return steps[-LAST:], names


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                                 "hbm_traffic.json")
    suffix = sys.argv[4] if len(sys.argv) > 4 else ""
    fs, names = per_step(fdir, "FETCH_SIZE")
    ws, _ = per_step(wdir, "WRITE_SIZE")
    res = {}
    if os.path.exists(out):   # merge: keys of other passes (other suffixes) are kept
        with open(out) as fi:
            res = json.load(fi)
    for op, _ in OPS:
        f = [s.get(op, 0.0) for s in fs]
        w = [s.get(op, 0.0) for s in ws]
        if not f:
            continue
        fb = 2.0 * sum(f) / len(f)
        wb = sum(w) / len(w) if w else 0.0
        res[op + suffix] = {"bytes_per_launch": fb + wb, "fetch_bytes": fb, "write_bytes": wb, "steps": len(f),
                   "kernels": sorted(names[op]),
                   "source": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE per step of tools/loop_step.py"}
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps({k: v["bytes_per_launch"] for k, v in res.items() if k.endswith(suffix) or not suffix}))


if __name__ == "__main__":
    main()
