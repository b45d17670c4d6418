"""Per-evaluation host cost of the restart loop (evr_qnehvi_plan_minimize with EVR_MIN_STATS=1:
time in the evaluation round trip vs the optimiser's own steps) for the config-4 ask, run once
per EVR_QUEUE setting in a fresh process.  usage: python tools/queue_probe.py"""
import os
import subprocess
import sys

CHILD = r'''
import os, sys, time
sys.path.insert(0, os.getcwd())
import torch, bench
s, _ = bench.make_ask_strategy(512, 256, 1024, 20, 1)
for _ in range(4):
    t0 = time.perf_counter(); s.ask(1); torch.cuda.synchronize()
    print("ask_ms %.3f restarts_ms %.3f evals %d" % (1e3 * (time.perf_counter() - t0), 1e3 * s.last_ask_stats.t_opt,
          bench._ask_evals(s)), flush=True)
'''


def main():
    for q in ("0", "1"):
        env = dict(os.environ, EVR_QUEUE=q, EVR_MIN_STATS="1")
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
        print(f"EVR_QUEUE={q}")
        for line in (r.stdout + r.stderr).splitlines():
            if "EVR_MIN_STATS" in line or line.startswith("ask_ms"):
                print("  " + line)


if __name__ == "__main__":
    main()
