"""Summarise a rocprofv3 --pmc pass of SQ counters (tools/gpu_steps.sh pmc_sq*) per kernel:
average per dispatch and the wave-cycle split the MI355X guide defines (WAIT_ANY = parked on
s_waitcnt / barrier, WAIT_INST_ANY = issue stall, ACTIVE_INST_ANY = issuing; the three add up
to WAVE_CYCLES), plus LDS bank conflicts per LDS instruction.

usage: python tools/pmc_sq.py <pmc_dir> <out.json> [label]   (merges into out.json)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d, out = sys.argv[1], sys.argv[2]
    label = sys.argv[3] if len(sys.argv) > 3 else os.path.basename(d.rstrip("/"))
    acc = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r["Kernel_Name"].split("(")[0][:80]
                acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = json.load(open(out)) if os.path.exists(out) else {}
    summ = {}
    for k, cs in acc.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"dispatches": max(len(v) for v in cs.values()), "per_dispatch": avg}
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            e["wave_cycle_split"] = {c: round(avg[c] / wc, 4) for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                                        "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS")
                                     if c in avg}
        if avg.get("SQ_INSTS_LDS"):
            e["lds_bank_conflict_cycles_per_lds_inst"] = round(avg.get("SQ_LDS_BANK_CONFLICT", 0.0) / avg["SQ_INSTS_LDS"], 4)
        if avg.get("SQ_WAVES"):
            e["wave_cycles_per_wave"] = round(wc / avg["SQ_WAVES"], 1) if wc else None
        summ[k] = e
    res[label] = summ
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps({k: v.get("wave_cycle_split") for k, v in summ.items()}))


if __name__ == "__main__":
    main()
