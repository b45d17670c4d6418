"""Digest of two consecutive warm bench asks (config 4): the proposed candidates, their
predictions and the restart optimiser's evaluation counts, as hex of the raw f64 bytes — two
builds that should be bitwise equal on the whole ask (every kernel, the optimiser's path) print
the same line.  usage: [EVR_LIB_PATH=...] python tools/ask_digest.py"""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench

    s, _ = bench.make_ask_strategy(512, 256, 1024, 20, 1)
    out = []
    for _ in range(2):
        df = s.ask(1)
        vals = np.ascontiguousarray(df.select_dtypes(include=[np.number]).to_numpy(dtype=np.float64))
        st = s.last_ask_stats
        out.append({"digest": hashlib.sha256(vals.tobytes()).hexdigest()[:16], "opt_evals": int(st.opt_evals),
                    "x0": float(vals[0, 0])})
    print(json.dumps({"lib": os.environ.get("EVR_LIB_PATH", "everest_amd/_lib"), "asks": out}))


if __name__ == "__main__":
    main()
