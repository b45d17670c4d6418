"""A/B of the ask at the bench shape over environment variants, interleaved (A B C A B C ...)
in fresh child processes so that box-host noise hits every variant alike.  Each child runs
2 warm-up asks then K timed asks and reports the median ask time and the median of the
construction / restart phases.  usage: python tools/ask_ab.py K ROUNDS NAME=ENV[,ENV] ..."""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch, bench
K = int(sys.argv[1])
s, _ = bench.make_ask_strategy(512, 256, 1024, 20, 1)
for _ in range(2):
    s.ask(1)
torch.cuda.synchronize()
ask, con, res = [], [], []
for _ in range(K):
    t0 = time.perf_counter()
    s.ask(1)
    torch.cuda.synchronize()
    ask.append(time.perf_counter() - t0)
    con.append(s.last_acqf.timings["total"])
    res.append(s.last_ask_stats.t_opt)
print("AB " + json.dumps({"ask_ms": 1e3 * float(np.median(ask)), "construction_ms": 1e3 * float(np.median(con)),
                          "restarts_ms": 1e3 * float(np.median(res))}))
'''


def main():
    K, rounds = int(sys.argv[1]), int(sys.argv[2])
    variants = []
    for a in sys.argv[3:]:
        name, _, envs = a.partition("=")
        env = dict(e.split(":", 1) for e in envs.split(",") if e)
        variants.append((name, env))
    out = {n: [] for n, _ in variants}
    for _ in range(rounds):
        for name, env in variants:
            r = subprocess.run([sys.executable, "-c", CHILD, str(K)], env=dict(os.environ, **env),
                               capture_output=True, text=True, timeout=300)
            line = [x for x in r.stdout.splitlines() if x.startswith("AB ")]
            if r.returncode != 0 or not line:
                print(r.stdout[-2000:], r.stderr[-2000:])
                sys.exit(1)
            out[name].append(json.loads(line[-1][3:]))
            print(name, out[name][-1], flush=True)
    summ = {n: {k: round(sorted(x[k] for x in v)[len(v) // 2], 3) for k in v[0]} for n, v in out.items()}
    print(json.dumps(summ))


if __name__ == "__main__":
    main()
