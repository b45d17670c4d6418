"""Device timeline of one warm QnehviStrategy.ask() (config-4 shape).

Run under ``rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python
tools/ask_timeline.py`` and then ``python tools/ask_timeline.py --analyse DIR``: the last ask's
host window (printed as JSON, monotonic and boottime clocks) selects its kernels; the report
gives the device-busy fraction, the busiest kernels and the largest idle gaps with the
kernels either side of them (where the host holds the device up)."""
import csv
import glob
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(asks=3):
    import torch
    import bench

    s, _ = bench.make_ask_strategy(512, 256, 1024, 20, 1)
    for _ in range(asks - 1):
        s.ask(1)
    torch.cuda.synchronize()
    w = {}
    w["mono0"], w["boot0"] = time.monotonic_ns(), time.clock_gettime_ns(time.CLOCK_BOOTTIME)
    s.ask(1)
    torch.cuda.synchronize()
    w["mono1"], w["boot1"] = time.monotonic_ns(), time.clock_gettime_ns(time.CLOCK_BOOTTIME)
    st = s.last_ask_stats
    w["phases"] = dict(construction=s.last_acqf.timings, raw_s=st.t_raw, opt_s=st.t_opt, opt_evals=st.opt_evals)
    print("ASK_WINDOW " + json.dumps(w, default=float), flush=True)


def analyse(d, log):
    w = None
    for line in open(log):
        if line.startswith("ASK_WINDOW "):
            w = json.loads(line[len("ASK_WINDOW "):])
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    best = None
    for clk in ("mono", "boot"):
        a, b = w[clk + "0"], w[clk + "1"]
        sel = [r for r in rows if r[0] >= a and r[1] <= b]
        if best is None or len(sel) > len(best[1]):
            best = (clk, sel, a, b)
    clk, sel, a, b = best
    wall = (b - a) / 1e3
    busy = 0.0
    by = {}
    gaps = []
    prev_end, prev_name = a, "<ask start>"
    for s0, s1, n in sel:
        short = n.split("(")[0][-60:]
        busy += (s1 - max(s0, prev_end)) / 1e3 if s1 > prev_end else 0.0
        by.setdefault(short, [0, 0.0])
        by[short][0] += 1
        by[short][1] += (s1 - s0) / 1e3
        if s0 - prev_end > 0:
            gaps.append(((s0 - prev_end) / 1e3, prev_name, short, (prev_end - a) / 1e3))
        prev_end, prev_name = max(prev_end, s1), short
    gaps.append(((b - prev_end) / 1e3, prev_name, "<ask end>", (prev_end - a) / 1e3))
    gaps.sort(reverse=True)
    idle_gt20 = sum(g[0] for g in gaps if g[0] > 20)
    # restart evaluations: chain span (the evaluation's first kernel -> qs_dx_reduce end) and the
    # host turnaround (qs_dx_reduce end -> the next evaluation's first kernel), medians; the
    # kernels of one evaluation and their mean durations
    ends = [i for i, r in enumerate(sel) if "qs_dx_reduce" in r[2]]
    spans, turns, per = [], [], {}
    for k, i in enumerate(ends):
        j = i
        first = ends[k - 1] + 1 if k > 0 else max(0, i - 8)
        spans.append((sel[i][1] - sel[first][0]) / 1e3)
        for r in sel[first:i + 1]:
            short = r[2].split("(")[0][-40:]
            per.setdefault(short, []).append((r[1] - r[0]) / 1e3)
        if k + 1 < len(ends):
            turns.append((sel[i + 1][0] - sel[i][1]) / 1e3)
    med = lambda v: round(float(sorted(v)[len(v) // 2]), 2) if v else None  # noqa: E731
    restart = dict(evaluations=len(ends), chain_span_us_median=med(spans), turnaround_us_median=med(turns),
                   kernels={k: [len(v), med(v)] for k, v in per.items()})
    # construction: the kernels before the first restart-chain kernel, in order (offset, duration)
    first_eval = ends[0] - 4 if ends else len(sel)
    cons = [[round((r[0] - a) / 1e3, 1), round((r[1] - r[0]) / 1e3, 1), r[2].split("(")[0][-48:]]
            for r in sel[:max(0, first_eval)]]
    out = dict(clock=clk, wall_us=round(wall, 1), kernels=len(sel), busy_us=round(busy, 1), restart=restart,
               construction_kernels=cons[:400],
               busy_frac=round(busy / wall, 3), idle_in_gaps_over_20us=round(idle_gt20, 1),
               phases=w["phases"],
               top_kernels=sorted(([k, v[0], round(v[1], 1)] for k, v in by.items()), key=lambda x: -x[2])[:15],
               top_gaps=[[round(g[0], 1), g[1], g[2], round(g[3], 1)] for g in gaps[:25]])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--analyse":
        analyse(sys.argv[2], sys.argv[3])
    else:
        run()
