#!/usr/bin/env python3
"""All-sources G100 kernel time vs the order the batch lists its sources (tuning aid:
tail balance of the dynamically scheduled solves). Orders: row-major, random, longest
first (eccentricity descending), shortest first.

  python scripts/order_probe.py [--reps 10]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch

    from openr_amd import topology as T
    from openr_amd.engine import SpfEngine

    n = 100
    g = T.grid_fast(n)
    V = g.num_nodes
    r, c = np.divmod(np.arange(V), n)
    ecc = np.maximum(r, n - 1 - r) + np.maximum(c, n - 1 - c)
    rng = np.random.default_rng(3)
    orders = {"row-major": np.arange(V), "random": rng.permutation(V),
              "longest-first": np.argsort(-ecc, kind="stable"), "shortest-first": np.argsort(ecc, kind="stable")}
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    eng = SpfEngine([0])
    eng.set_graph(g)
    nb = eng.nh_bytes
    d_dist = torch.empty((V, V), dtype=torch.int64, device=dev)
    d_nh = torch.empty((V, V, nb), dtype=torch.uint8, device=dev)
    for rnd in range(2):
        for name, p in orders.items():
            src = torch.from_numpy(np.ascontiguousarray(p, dtype=np.int32)).to(dev)
            ts = []
            for i in range(args.reps + 1):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                eng.solve_device(src.data_ptr(), V, d_dist.data_ptr(), d_nh.data_ptr(), nb, True,
                                 stream=stream.cuda_stream)
                b.record(stream)
                torch.cuda.synchronize(dev)
                if i:
                    ts.append(a.elapsed_time(b))
            print(json.dumps({"round": rnd, "order": name, "median_ms": float(np.median(ts)),
                              "min_ms": float(np.min(ts))}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
