"""Config 4's sharded ask through the HIP acquisition vs the 1-rank ask at the same seed.

Usage (one GPU box): ``python tools/sharded_ask_check.py --ranks 2 --asks 3 --out DIR``.
The parent never touches HIP: it starts one 1-rank child, then ``--ranks`` children that
share the box's GPU(s) round-robin and exchange over gloo (the RCCL path is the same code
with "nccl"; bench.py EVR_DIST_BACKEND).  Every child builds the config-4 QnehviStrategy
(bench.make_ask_strategy: DTLZ2(6, 5), n = 512, S = 256, 1024 raw, 20 restarts,
batch_limit 20 or ``--batch-limit``, seed 1) and runs ``--asks`` asks; rank 0 writes per ask the candidate x, the
best acquisition value, the global optimiser evaluation count, the restart driver label and
the ask time.  The parent compares the two runs and writes ``DIR/sharded_ask.json``.

Reference layout: bofire/data_models/strategies/predictives/botorch.py:101-108
(batch_limit = num_restarts: one joint problem) and SURVEY.md §8(e)."""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(args):
    import numpy as np
    import torch

    sys.path.insert(0, ROOT)
    import bench

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(rank % max(1, torch.cuda.device_count()))
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")
    s, tells = bench.make_ask_strategy(args.n, args.S, args.raw, args.restarts, world, dist, seed=1,
                                       batch_limit=args.batch_limit)
    out = []
    for _ in range(args.asks):
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        df = s.ask(1)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        st = s.last_ask_stats
        x = df[s.domain.inputs.get_keys()].values[0]
        out.append({"x": [float(v) for v in x], "x_hex": [float(v).hex() for v in x],
                    "best_value": float(st.best_value), "best_value_hex": float(st.best_value).hex(),
                    "opt_evals_global": int(st.opt_evals_global), "raw_evals": int(st.raw_evals),
                    "opt_iters": int(st.opt_iters), "drivers": [c["driver"] for c in st.chunks],
                    "local_batch": [c.get("local_batch") for c in st.chunks], "ask_s": round(dt, 4)})
    if rank == 0:
        with open(os.path.join(args.out, f"w{world}.json"), "w") as f:
            json.dump({"world": world, "tell_s": [round(t, 3) for t in tells], "asks": out}, f, indent=1)
    if dist is not None:
        dist.destroy_process_group()


def spawn(world, args):
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child"] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        r = p.wait()
        rc = rc or r
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--asks", type=int, default=3)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--S", type=int, default=256)
    ap.add_argument("--raw", type=int, default=1024)
    ap.add_argument("--restarts", type=int, default=20)
    ap.add_argument("--batch-limit", type=int, default=0, help="0: = restarts (one joint problem)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "sharded"))
    args = ap.parse_args()
    if args.child:
        return child(args)
    os.makedirs(args.out, exist_ok=True)
    for w in (1, args.ranks):
        rc = spawn(w, args)
        if rc != 0:
            print(f"world {w} failed with exit code {rc}", file=sys.stderr)
            return rc
    a = json.load(open(os.path.join(args.out, "w1.json")))
    b = json.load(open(os.path.join(args.out, f"w{args.ranks}.json")))
    rows = []
    for k, (p, q) in enumerate(zip(a["asks"], b["asks"])):
        rows.append({"ask": k, "x_bitwise_equal": p["x_hex"] == q["x_hex"],
                     "best_value_bitwise_equal": p["best_value_hex"] == q["best_value_hex"],
                     "max_abs_dx": max(abs(u - v) for u, v in zip(p["x"], q["x"])),
                     "rel_dvalue": abs(p["best_value"] - q["best_value"]) / max(abs(p["best_value"]), 1e-300),
                     "opt_evals_global": [p["opt_evals_global"], q["opt_evals_global"]],
                     "drivers": [p["drivers"], q["drivers"]], "ask_s": [p["ask_s"], q["ask_s"]]})
    res = {"ranks": args.ranks, "backend": "gloo (ranks share the box's GPU; RCCL on a multi-GPU node)",
           "config": f"DTLZ2(6,5) n={args.n} S={args.S} raw={args.raw} restarts={args.restarts} batch_limit="
                     f"{args.batch_limit or args.restarts} seed=1", "asks": rows,
           "all_bitwise_equal": all(r["x_bitwise_equal"] and r["best_value_bitwise_equal"] for r in rows)}
    with open(os.path.join(args.out, "sharded_ask.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
