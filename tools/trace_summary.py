"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel total / count / mean, the busy time
(union of kernel intervals) and the idle gaps, over the whole capture or a time window.
usage: python tools/trace_summary.py <kernel_trace.csv> [top]"""
import csv
import sys
from collections import defaultdict


def main(path, top=25):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    tot = defaultdict(lambda: [0, 0])
    for s, e, k in rows:
        t = tot[k.split("(")[0][:80]]
        t[0] += e - s
        t[1] += 1
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = rows[-1][1] - rows[0][0]
    print(f"kernels {len(rows)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms ({100 * busy / span:.1f} %)")
    for k, (t, n) in sorted(tot.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{t / 1e6:10.3f} ms {n:7d} x {t / n / 1e3:9.2f} us  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
